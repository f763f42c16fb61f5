#!/bin/bash
# cfg 3's window PMC (FETCH_SIZE, WRITE_SIZE in separate passes) into the PMC summary, then the cfg 3 line reading it
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06/g29
mkdir -p $O
cp profiles/r06/pmc_window.json $O/pmc_window.json
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc3/fetch -o run -- python3 profiles/r06/pmc_window.py run cfg3 5 20 > $O/pmc_f.log 2>&1 || { echo pmc fetch failed; tail $O/pmc_f.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc3/write -o run -- python3 profiles/r06/pmc_window.py run cfg3 5 20 > $O/pmc_w.log 2>&1 || { echo pmc write failed; tail $O/pmc_w.log; exit 1; }
python3 profiles/r06/pmc_window.py summarize $O/pmc3 cfg3 $O/pmc_window.json > /dev/null || { echo "pmc summarize failed"; exit 1; }
cp $O/pmc_window.json profiles/r06/pmc_window.json
timeout -k 10 900 python -u bench.py --config cfg3 --steps 20 --warmup 5 > $O/bench_cfg3.json 2> $O/bench_cfg3.err || { echo cfg3 bench failed; tail -20 $O/bench_cfg3.err; exit 1; }
tail -c 300 $O/bench_cfg3.json

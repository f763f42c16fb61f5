#!/bin/bash
# the final binary's cfg 5 rocprof kernel stats and window PMC (into the PMC summary), then the cfg 5 line reading it
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06/g35
mkdir -p $O
cp profiles/r06/pmc_window.json $O/pmc_window.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 20 --warmup 5 --no-converge --no-cpu-baseline --no-lock-off > $O/bench_trace.json 2> $O/trace.err || { echo trace failed; tail $O/trace.err; exit 1; }
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc5/fetch -o run -- python3 profiles/r06/pmc_window.py run cfg5 5 20 > $O/pmc_f.log 2>&1 || { echo pmc fetch failed; tail $O/pmc_f.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc5/write -o run -- python3 profiles/r06/pmc_window.py run cfg5 5 20 > $O/pmc_w.log 2>&1 || { echo pmc write failed; tail $O/pmc_w.log; exit 1; }
python3 profiles/r06/pmc_window.py summarize $O/pmc5 cfg5 $O/pmc_window.json > /dev/null || { echo "pmc summarize failed"; exit 1; }
cp $O/pmc_window.json profiles/r06/pmc_window.json
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { echo cfg5 bench failed; tail -20 $O/bench_cfg5.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench_cfg5.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline'], d['roofline_merge'], d['roofline_send'])"

#!/bin/bash
# Profiles the cfg5 bench (rocprofv3): kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in
# separate --pmc passes (MI355X_MICROARCH.md §rocprofv3 PMC slots). Run on the GPU box from the
# repo root; outputs land in gpurun_out/prof_<tag>/. Summarise with profiles/summarize.py.
set -e
TAG=${1:-r01}
STEPS=${2:-30}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --config cfg5 --steps $STEPS --no-converge --no-cpu-baseline --no-lock-off > $OUT/bench_trace.json
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
  python3 bench.py --config cfg5 --steps 100 --no-converge --no-cpu-baseline --no-lock-off > $OUT/bench_fetch.json
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
  python3 bench.py --config cfg5 --steps 100 --no-converge --no-cpu-baseline --no-lock-off > $OUT/bench_write.json

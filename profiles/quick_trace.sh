#!/bin/bash
# Kernel trace of one short cfg5 bench run plus per-dispatch push-pull/storm times (A/B checks).
set -e
TAG=${1:-ab}
export TMPDIR=/tmp
OUT=gpurun_out/trace_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 bench.py --config cfg5 --steps 100 --no-converge --no-cpu-baseline > $OUT/bench.json
python3 profiles/trace_dispatch.py $OUT/run_kernel_trace.csv > $OUT/dispatch.txt

#!/bin/bash
# Round 4: bench lines at the other BASELINE configs and Sidecar's defaults, with the queue report
# (faithful = no LOST job) and, after a heal, the version spread. Run on the GPU box from the repo root.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
for c in ${CONFIGS:-cfg2 cfg4 cfg3 cfg5_defaults}; do
  timeout -k 10 900 python3 bench.py --config $c --no-cpu-baseline > gpurun_out/r04/bench_$c.json
  echo "done $c"
done

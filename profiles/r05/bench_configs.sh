#!/bin/bash
# Round-5 bench lines, one per configuration (the driver's default run is cfg5):
#   bash profiles/r05/bench_configs.sh [tag] [configs...]
# Lines land in gpurun_out/r05/<tag>/bench_<cfg>.json (stderr beside them). Stops at the first
# failure (set -e; every step under its own time limit).
set -e
TAG=${1:-bench}
shift || true
CFGS=${@:-cfg5 cfg2 cfg3 cfg4 cfg5_defaults}
O=gpurun_out/r05/$TAG
mkdir -p $O
for c in $CFGS; do
  extra="--no-cpu-baseline"
  [ "$c" = cfg5 ] && extra=""
  timeout -k 10 400 python -u bench.py --config $c $extra > $O/bench_$c.json 2> $O/bench_$c.err
  echo "$c done"
done

#!/bin/bash
# round-6 bench lines on the final build: cfg 2, 3, 4 and Sidecar's defaults
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g23
mkdir -p $O
for c in cfg3 cfg5_defaults cfg2 cfg4; do
  timeout -k 10 900 python -u bench.py --config $c --steps 20 --warmup 5 > $O/bench_$c.json 2> $O/bench_$c.err || { echo $c bench failed; tail -20 $O/bench_$c.err; exit 1; }
  tail -c 200 $O/bench_$c.json; echo
done

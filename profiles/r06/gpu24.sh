#!/bin/bash
# the cfg 5 line again, reading the window's PMC summary with k_lock_append in the merge class
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g24
mkdir -p $O
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { echo cfg5 bench failed; tail -20 $O/bench_cfg5.err; exit 1; }
tail -c 300 $O/bench_cfg5.json

#!/bin/bash
# N = 4 rehearsal of the multi-rank bench (4 ranks on one GPU, collectives over gloo), final build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g27
mkdir -p $O
GX_BENCH_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 4 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_n4_gloo.json 2> $O/bench_n4_gloo.err || { echo n4 failed; tail -30 $O/bench_n4_gloo.err; exit 1; }
tail -c 600 $O/bench_n4_gloo.json

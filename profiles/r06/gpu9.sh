#!/bin/bash
# merge / send variants A/B on the cfg 5 gossip stretches, then the bench's N = 2 path rehearsed over
# gloo on one GPU (both ranks share the card: correctness of the distributed path, not scaling)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g9
mkdir -p $O
L=profiles/r06/ablib
timeout -k 10 900 python -u profiles/r06/ab_spans.py --libs $L/libgx_r6.so $L/libgx_rpl8.so $L/libgx_rpl2.so $L/libgx_wpe6.so $L/libgx_pr64.so --reps 3 > $O/ab_variants.jsonl 2>&1 || { echo ab failed; tail $O/ab_variants.jsonl; exit 1; }
tail -1 $O/ab_variants.jsonl
GX_BENCH_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err || { echo n2 failed; tail -30 $O/bench_n2_gloo.err; exit 1; }
tail -c 400 $O/bench_n2_gloo.json

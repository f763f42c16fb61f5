#!/bin/bash
# Rehearsal of bench.py's multi-process path at N = 4 on the one GPU of the box: four ranks, each a
# DistShard over a quarter of the cfg 5 hosts, collectives over gloo staged through the host
# (RCCL refuses several ranks on one device). The driver's window [5, 25): the storm, two
# partitioned push-pull rounds and gossip rounds whose packets cross shards inside each half.
# Timings are not scaling data (four ranks share one GPU).
set -e
export TMPDIR=/tmp
O=gpurun_out/r03n4
mkdir -p $O
GX_BENCH_BACKEND=gloo timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 4 --steps 20 --warmup 5 --no-cpu-baseline \
  --converge-max 200 > $O/bench_n4_gloo.json 2> $O/bench_n4_gloo.err
tail -c 1500 $O/bench_n4_gloo.json

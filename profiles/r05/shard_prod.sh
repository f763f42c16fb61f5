#!/bin/bash
# The product build's sharded round at G = 8 (cfg 5, rounds 51-59), both lock models, kernel trace.
set -e
OUT=gpurun_out/r05/sab2
mkdir -p $OUT
for lm in 0 1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/libgx_lm$lm -o run -- python3 -u profiles/r05/shard_round.py \
    --lock-model $lm > $OUT/libgx_lm$lm.json 2> $OUT/libgx_lm$lm.err
done

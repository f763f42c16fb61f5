#!/bin/bash
# A/B of the merge with 16 receivers per block below 16384 local hosts (libgx_nr16, now the product) against
# 64 always: a shard of cfg 5 at G = 8, and cfg 2 / cfg 4 on one engine, lock on and off.
set -e
O=gpurun_out/r05/mnr
mkdir -p $O
L="sidecar_amd/libgx.so profiles/r05/lib/libgx_nr16.so"
for lib in $L; do
  n=$(basename $lib .so)
  timeout -k 10 200 python3 -u profiles/r05/shard_round.py --lock-model 1 --lib $lib > $O/shard_$n.json 2> $O/shard_$n.err
done
for c in cfg2 cfg4; do
  for lm in 1 0; do
    timeout -k 10 300 python3 -u profiles/r04/ab_kernels.py --config $c --skip 0 --rounds 60 --reps 2 --lock-model $lm --libs $L > $O/ab_${c}_lm$lm.jsonl 2> $O/ab_${c}_lm$lm.err
  done
done

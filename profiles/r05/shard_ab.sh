#!/bin/bash
# k_send and the sharded round at G = 8 (cfg 5, rounds 51-59) for three builds: before k_send packed
# the planned exchange (libgx_pf1), packing with one claim per packet (libgx_claim1), and the product
# (one claim per destination and wave). Kernel trace per build; run on the GPU box.
set -e
OUT=gpurun_out/r05/sab
mkdir -p $OUT
for lm in 0 1; do
  for lib in profiles/r05/lib/libgx_pf1.so profiles/r05/lib/libgx_claim1.so sidecar_amd/libgx.so; do
    n=$(basename $lib .so)_lm$lm
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/$n -o run -- python3 -u profiles/r05/shard_round.py \
      --lock-model $lm --lib $lib > $OUT/$n.json 2> $OUT/$n.err
  done
done

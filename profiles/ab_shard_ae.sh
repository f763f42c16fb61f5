#!/bin/bash
# Sharded push-pull kernels (LocalShards, G = 2, H = 16384 on one GPU: profiles/shard_overlap.py)
# per GX_AB_FLAGS variant given as arguments; the shard tests under each variant first.
set -e
export TMPDIR=/tmp
for f in "$@"; do
  GX_AB_FLAGS=$f timeout -k 10 300 python -u -m pytest tests/test_gpu_shards.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_sae_tests_$f.log 2>&1
  tail -1 gpurun_out/ab_sae_tests_$f.log
  mkdir -p gpurun_out/ab_sae_$f
  GX_AB_FLAGS=$f timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab_sae_$f -o run -- python3 profiles/shard_overlap.py 2 16384 > gpurun_out/ab_sae_$f/overlap.json
  echo "== GX_AB_FLAGS=$f"
  python3 profiles/kernel_totals.py gpurun_out/ab_sae_$f/run_kernel_trace.csv k_ae
done

#!/bin/bash
# A/B: k_ae / k_scan with __syncthreads_or (libgx_base) vs the LDS vote block_any256 (libgx_any)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04
for c in cfg4 cfg2 cfg3; do
  timeout -k 10 240 python3 -u $R/profiles/r04/ab_kernels.py --config $c --skip 5 --rounds 60 --reps 2 --libs $R/profiles/r04/lib/libgx_any.so $R/profiles/r04/lib/libgx_fast.so > $O/ab_fast_$c.jsonl
  tail -1 $O/ab_fast_$c.jsonl
done
timeout -k 10 240 python3 -u $R/profiles/r04/ab_kernels.py --config cfg5 --skip 9 --rounds 42 --reps 2 --libs $R/profiles/r04/lib/libgx_any.so $R/profiles/r04/lib/libgx_fast.so > $O/ab_fast_cfg5.jsonl
tail -1 $O/ab_fast_cfg5.jsonl

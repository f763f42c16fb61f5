#!/bin/bash
# A/B of the expiry scan at cfg 3: HEAD vs the quiet-wave fast path (libgx_squiet)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04
L=$R/profiles/r04/lib
timeout -k 10 400 python3 -u $R/profiles/r04/ab_kernels.py --config cfg3 --skip 100 --rounds 30 --reps 2 --libs $L/libgx_base.so $L/libgx_squiet.so > $O/ab_squiet_cfg3.jsonl
tail -1 $O/ab_squiet_cfg3.jsonl

#!/bin/bash
# k_ae lock off at cfg 2 (the bench window's two push-pull rounds): two tiles in flight, plain
# (temporal) row loads and stores, and two tiles at 3 waves per SIMD, against the current build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g30
mkdir -p $O
L=profiles/r06/ablib
timeout -k 10 600 python -u profiles/r04/ab_kernels.py --config cfg2 --skip 5 --rounds 20 --reps 4 --lock-model 0 \
  --libs $L/libgx_ae_base.so $L/libgx_ae_pf2.so $L/libgx_ae_nont.so $L/libgx_ae_pf2w3.so > $O/ab_ae_cfg2.jsonl 2>&1 || { echo ab failed; tail $O/ab_ae_cfg2.jsonl; exit 1; }
tail -1 $O/ab_ae_cfg2.jsonl

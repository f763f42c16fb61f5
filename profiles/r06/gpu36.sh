#!/bin/bash
# chunks per row for the wave-level scan (SCAN_ITEMS 1024 / 2048 / 4096) at cfg 3, lock off and on
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g36
mkdir -p $O
L=profiles/r06/ablib
for lm in 0 1; do
timeout -k 10 500 python -u profiles/r04/ab_kernels.py --config cfg3 --skip 100 --rounds 30 --reps 3 --lock-model $lm \
  --libs $L/libgx_si2048.so $L/libgx_si4096.so $L/libgx_si1024.so > $O/ab_si_cfg3_lm$lm.jsonl 2>&1 || { echo ab failed; tail $O/ab_si_cfg3_lm$lm.jsonl; exit 1; }
tail -1 $O/ab_si_cfg3_lm$lm.jsonl
done

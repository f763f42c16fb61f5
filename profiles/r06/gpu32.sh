#!/bin/bash
# merge blocks of 64 receivers when k_lock_append takes the locked ones (cfg 5): parity at full size, then gossip stretches
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g32
mkdir -p $O
L=profiles/r06/ablib
timeout -k 10 600 python -u profiles/r06/ab_spans.py --libs $L/libgx_m_nr16.so $L/libgx_m_nr64.so --reps 3 > $O/ab_nr64.jsonl 2>&1 || { echo ab failed; tail $O/ab_nr64.jsonl; exit 1; }
tail -1 $O/ab_nr64.jsonl

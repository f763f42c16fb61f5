#!/bin/bash
# merge blocks of 16 receivers at cfg 5 (GX_MERGE_SMALL_HL raised): gossip stretches, lock on and off
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g6
mkdir -p $O
timeout -k 10 600 python -u profiles/r06/ab_spans.py --libs profiles/r06/ablib/libgx_si4096.so profiles/r06/ablib/libgx_nr16.so --reps 3 > $O/ab_nr16.jsonl 2>&1 || { echo ab nr16 failed; tail $O/ab_nr16.jsonl; exit 1; }
tail -1 $O/ab_nr16.jsonl

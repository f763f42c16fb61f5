#!/bin/bash
# Dev by pointer (GX_DEVPTR) A/B on the gossip stretches, after a parity spot-check of the variant
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g3
mkdir -p $O
timeout -k 10 300 python -u profiles/r06/check_lib.py profiles/r06/ablib/libgx_dp.so > $O/check_dp.log 2>&1 || { echo check failed; tail -20 $O/check_dp.log; exit 1; }
tail -1 $O/check_dp.log
timeout -k 10 600 python -u profiles/r06/ab_spans.py --libs profiles/r06/ablib/libgx_base.so profiles/r06/ablib/libgx_dp.so --reps 4 > $O/ab_dp.jsonl 2>&1 || { echo ab failed; tail -20 $O/ab_dp.jsonl; exit 1; }
tail -1 $O/ab_dp.jsonl

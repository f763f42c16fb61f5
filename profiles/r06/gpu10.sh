#!/bin/bash
# PLAN_CH (GetBroadcasts calls planned per chunk) 2 / 4 / 8: parity spot-check, then the gossip
# stretches at Sidecar's defaults (GossipMessages 15) and at cfg 5
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g10
mkdir -p $O
L=profiles/r06/ablib
for v in pc8 pc2; do
  timeout -k 10 300 python -u profiles/r06/check_lib.py $L/libgx_$v.so > $O/check_$v.log 2>&1 || { echo check $v failed; tail -5 $O/check_$v.log; exit 1; }
done
timeout -k 10 900 python -u profiles/r06/ab_spans.py --config cfg5_defaults --libs $L/libgx_r6.so $L/libgx_pc8.so $L/libgx_pc2.so --reps 3 > $O/ab_pc_defaults.jsonl 2>&1 || { echo ab failed; tail $O/ab_pc_defaults.jsonl; exit 1; }
tail -1 $O/ab_pc_defaults.jsonl
timeout -k 10 600 python -u profiles/r06/ab_spans.py --config cfg5 --libs $L/libgx_r6.so $L/libgx_pc8.so --reps 2 > $O/ab_pc_cfg5.jsonl 2>&1 || { echo ab failed; tail $O/ab_pc_cfg5.jsonl; exit 1; }
tail -1 $O/ab_pc_cfg5.jsonl

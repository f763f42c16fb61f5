#!/bin/bash
# In-process A/B of the routed merge (0) against round 2's merge (GX_AB_FLAGS=2048), both stretches.
set -e
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03m3}
mkdir -p $O
timeout -k 10 400 python3 profiles/r03/ab_span.py --flags 0 2048 --reps 3 > $O/ab_span.jsonl 2>/dev/null
tail -1 $O/ab_span.jsonl

#!/bin/bash
# Merge blocks of 16 receivers under GossipMessages 15 (default there) against 64 (bit 4096), and
# the same flip at GossipMessages 1 (64 default); parity of the GM scenarios first.
set -e
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03wpe6}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -k "gossip or wide or plan_gm" -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
timeout -k 10 500 python3 profiles/r03/ab_span.py --config cfg5_defaults --flags 0 8192 --reps 2 --starts 51 > $O/ab_gm15.jsonl 2>/dev/null
tail -1 $O/ab_gm15.jsonl



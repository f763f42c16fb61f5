#!/bin/bash
# k_lock_append with a wave-level early exit: lock tests, then gossip stretches vs GX_LOCK_APPEND=0
# (cfg 5, with the full-pipeline stretch 51..59)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g21
mkdir -p $O
L=profiles/r06/ablib
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lock.py tests/test_gpu_lock_readers.py \
  tests/test_gpu_parity.py -m gpu > $O/tests.log 2>&1 || { echo tests failed; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u profiles/r06/ab_spans.py --libs $L/libgx_la0.so $L/libgx_la1.so --reps 3 > $O/ab_la_cfg5.jsonl 2>&1 || { echo ab failed; tail $O/ab_la_cfg5.jsonl; exit 1; }
tail -1 $O/ab_la_cfg5.jsonl

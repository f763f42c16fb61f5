#!/bin/bash
# k_lock_append with its routing, count and header loads in one round trip: the full-size cfg 5 parity
# (the only tests whose engines launch it) and lock suites, then gossip stretches A/B against HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g28
mkdir -p $O
L=profiles/r06/ablib
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread "tests/test_gpu_fullsize.py::test_cfg5_full_h32768_parity" \
  tests/test_gpu_lock.py -m gpu > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u profiles/r06/ab_spans.py --libs $L/libgx_la_head.so $L/libgx_la_pre.so --reps 3 > $O/ab_la_pre.jsonl 2>&1 || { echo ab failed; tail $O/ab_la_pre.jsonl; exit 1; }
tail -1 $O/ab_la_pre.jsonl

#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g16
mkdir -p $O
timeout -k 10 300 python -u profiles/r06/hq_diag.py depart_gm4_buf100 > $O/diag.log 2>&1; rc=$?
cat $O/diag.log | head -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_fd_handoff.py -m gpu > $O/tests.log 2>&1
grep -E "PASS|FAIL" $O/tests.log

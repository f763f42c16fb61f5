#!/bin/bash
# sanity on the final binary (rebuilt after a comment-only change): smoke, ABI, scan split, lock and parity suites
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g37
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_abi.py tests/test_gpu_scan_split.py tests/test_gpu_lock.py \
  tests/test_gpu_lock_readers.py tests/test_gpu_parity.py tests/test_golden.py -m gpu > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log

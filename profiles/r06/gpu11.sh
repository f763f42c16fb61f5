#!/bin/bash
# lock_readers (push-pull with a read-locked side): the lock KATs, the new parity scenarios, and the
# round-model parity suites that the lock-word and capacity changes touch
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g11
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_lock_readers.py tests/test_gpu_lock.py \
  tests/test_gpu_parity.py tests/test_golden.py -m gpu > $O/tests.log 2>&1
rc=$?
tail -15 $O/tests.log
exit $rc

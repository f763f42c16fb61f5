#!/bin/bash
# the rest of the GPU suite after test_gpu_fullsize.py::test_cfg5_full_h32768_parity[1], then smoke
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g13
mkdir -p $O
timeout -k 10 1100 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests -m gpu --durations=15 \
  --deselect "tests/test_gpu_fullsize.py::test_cfg5_full_h32768_parity[0]" > $O/suite.log 2>&1 || { echo suite failed; tail -30 $O/suite.log; exit 1; }
tail -20 $O/suite.log
grep "cfg5@32768 lock_readers" $O/suite.log || true
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log

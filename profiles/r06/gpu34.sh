#!/bin/bash
# the full GPU suite and smoke on HEAD at the end of round 6
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g34
mkdir -p $O
timeout -k 10 1100 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests -m gpu --durations=10 > $O/suite.log 2>&1 || { echo suite failed; grep -E "FAIL|Error" $O/suite.log | head; tail -30 $O/suite.log; exit 1; }
tail -14 $O/suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log

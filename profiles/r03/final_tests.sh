#!/bin/bash
# Final round-3 tree on the GPU box: every -m gpu test, then smoke().
set -e
export TMPDIR=/tmp
O=gpurun_out/r03final
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -3 $O/gputests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
cat $O/smoke.log

#!/bin/bash
# fd_handoff_shared: parity of the new scenarios and the fd / lock suites; then the cfg 5 bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g15
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fd_handoff.py tests/test_gpu_fd.py \
  tests/test_gpu_lock_readers.py tests/test_gpu_lock.py tests/test_gpu_parity.py tests/test_golden.py tests/test_abi.py -m gpu > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAIL|Error|error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 600 python -u bench.py > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { echo bench failed; tail -20 $O/bench_cfg5.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench_cfg5.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['gossip']['device_us_per_round'], d['gossip']['round_span_us_accepting'], d['gossip']['lock_off']['round_span_us'], d['gossip']['lock_off']['round_span_us_accepting'])"

#!/bin/bash
# 64-receiver merge blocks beside k_lock_append: full-size cfg 5 parity (the engines that take this path),
# lock and parity suites, then the cfg 5 line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g33
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread "tests/test_gpu_fullsize.py::test_cfg5_full_h32768_parity" \
  "tests/test_gpu_fullsize.py::test_cfg5_properties_and_determinism" tests/test_gpu_lock.py tests/test_gpu_parity.py -m gpu > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { echo cfg5 bench failed; tail -20 $O/bench_cfg5.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench_cfg5.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_merge'], d['gossip']['device_us_per_round'], d['gossip']['round_span_us'], d['gossip']['round_span_us_accepting'])"

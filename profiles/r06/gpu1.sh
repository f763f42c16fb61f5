#!/bin/bash
# round 6, first GPU session: new parity tests, RCCL teardown, then the long faithful runs of cfg 2 / cfg 4
set -o pipefail
mkdir -p gpurun_out/r06/g1
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_probe.py \
  tests/test_gpu_lock.py tests/test_gpu_shards.py tests/test_gpu_rccl.py tests/test_abi.py \
  > gpurun_out/r06/g1/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06/g1/tests.log; exit 1; }
tail -3 gpurun_out/r06/g1/tests.log
timeout -k 10 300 python -u profiles/r06/converge_long.py cfg2 --rounds 60000 --every 500 --queue-cap 1048576 \
  > gpurun_out/r06/g1/cfg2_long.jsonl 2>&1 || { echo "cfg2 failed"; tail -5 gpurun_out/r06/g1/cfg2_long.jsonl; exit 1; }
tail -2 gpurun_out/r06/g1/cfg2_long.jsonl
timeout -k 10 400 python -u profiles/r06/converge_long.py cfg4 --rounds 60000 --every 500 --queue-cap 1048576 \
  > gpurun_out/r06/g1/cfg4_long.jsonl 2>&1 || { echo "cfg4 failed"; tail -5 gpurun_out/r06/g1/cfg4_long.jsonl; exit 1; }
tail -2 gpurun_out/r06/g1/cfg4_long.jsonl

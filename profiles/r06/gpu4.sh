#!/bin/bash
# row-split expiry scan: parity (new test + full-size cfg 2 / cfg 3), then the cfg 3 A/B against the
# previous build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g4
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_scan_split.py \
  "tests/test_gpu_fullsize.py::test_cfg3_bench_schedule_51_rounds" tests/test_gpu_parity.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cp sidecar_amd/libgx.so /tmp/libgx_split.so
for lm in 0 1; do
timeout -k 10 300 python -u profiles/r04/ab_kernels.py --config cfg3 --skip 100 --rounds 30 --reps 3 --lock-model $lm \
  --libs profiles/r06/ablib/libgx_base.so /tmp/libgx_split.so > $O/ab_scan_cfg3_lm$lm.jsonl 2>&1 || { echo ab failed; tail $O/ab_scan_cfg3_lm$lm.jsonl; exit 1; }
tail -1 $O/ab_scan_cfg3_lm$lm.jsonl
done

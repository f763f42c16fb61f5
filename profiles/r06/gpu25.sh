#!/bin/bash
# wave scan with buffer loads/stores (a fixed vector-memory count per tile): scan-split parity on the
# in-tree build, then cfg 3 scan A/B against the committed global-memory version
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g25
mkdir -p $O
L=profiles/r06/ablib
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_scan_split.py \
  "tests/test_gpu_fullsize.py::test_cfg3_bench_schedule_51_rounds" "tests/test_gpu_fullsize.py::test_cfg3_full_parity" -m gpu > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for lm in 0 1; do
timeout -k 10 500 python -u profiles/r04/ab_kernels.py --config cfg3 --skip 100 --rounds 30 --reps 3 --lock-model $lm \
  --libs $L/libgx_sg2.so $L/libgx_bw2.so $L/libgx_bw3.so > $O/ab_scan_cfg3_lm$lm.jsonl 2>&1 || { echo ab failed; tail $O/ab_scan_cfg3_lm$lm.jsonl; exit 1; }
tail -1 $O/ab_scan_cfg3_lm$lm.jsonl
done

#!/bin/bash
# k_lock_append + the wave-level chunk scan (scan_chunk_waves): parity suites on the in-tree build,
# then A/B: gossip stretches vs GX_LOCK_APPEND=0 (cfg 5, Sidecar's defaults), scan at cfg 3 vs the block scan
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g18
mkdir -p $O
L=profiles/r06/ablib
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_scan_split.py tests/test_gpu_lock.py tests/test_gpu_lock_readers.py \
  tests/test_gpu_parity.py tests/test_gpu_fd_handoff.py tests/test_gpu_fd.py tests/test_golden.py \
  "tests/test_gpu_fullsize.py::test_cfg3_bench_schedule_51_rounds" -m gpu > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAIL|Error" $O/tests.log | head; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for lm in 0 1; do
timeout -k 10 500 python -u profiles/r04/ab_kernels.py --config cfg3 --skip 100 --rounds 30 --reps 3 --lock-model $lm \
  --libs $L/libgx_scan_base.so $L/libgx_sw_w2.so $L/libgx_sw_w3.so $L/libgx_sw_w4.so > $O/ab_scan_cfg3_lm$lm.jsonl 2>&1 || { echo ab failed; tail $O/ab_scan_cfg3_lm$lm.jsonl; exit 1; }
tail -1 $O/ab_scan_cfg3_lm$lm.jsonl
done
timeout -k 10 600 python -u profiles/r06/ab_spans.py --libs $L/libgx_la0.so $L/libgx_la1.so --reps 3 > $O/ab_la_cfg5.jsonl 2>&1 || { echo ab failed; tail $O/ab_la_cfg5.jsonl; exit 1; }
tail -1 $O/ab_la_cfg5.jsonl
timeout -k 10 600 python -u profiles/r06/ab_spans.py --config cfg5_defaults --libs $L/libgx_la0.so $L/libgx_la1.so --reps 2 > $O/ab_la_defaults.jsonl 2>&1 || { echo ab failed; tail $O/ab_la_defaults.jsonl; exit 1; }
tail -1 $O/ab_la_defaults.jsonl

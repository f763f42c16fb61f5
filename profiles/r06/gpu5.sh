#!/bin/bash
# row-split scan with the adaptive chunk count: parity, then cfg 3 A/B (whole rows vs 4096 / 2048 items)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g5
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_scan_split.py \
  "tests/test_gpu_fullsize.py::test_cfg3_bench_schedule_51_rounds" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cp sidecar_amd/libgx.so /tmp/libgx_si4096.so
for lm in 0 1; do
timeout -k 10 400 python -u profiles/r04/ab_kernels.py --config cfg3 --skip 100 --rounds 30 --reps 3 --lock-model $lm \
  --libs profiles/r06/ablib/libgx_base.so /tmp/libgx_si4096.so profiles/r06/ablib/libgx_si2048.so > $O/ab_scan_cfg3_lm$lm.jsonl 2>&1 || { echo ab failed; tail $O/ab_scan_cfg3_lm$lm.jsonl; exit 1; }
tail -1 $O/ab_scan_cfg3_lm$lm.jsonl
done
# merge blocks of 16 receivers at cfg 5 (GX_MERGE_SMALL_HL raised): gossip stretches, lock on and off
if [ -f profiles/r06/ablib/libgx_nr16.so ]; then
timeout -k 10 600 python -u profiles/r06/ab_spans.py --libs /tmp/libgx_si4096.so profiles/r06/ablib/libgx_nr16.so --reps 3 > $O/ab_nr16.jsonl 2>&1 || { echo ab nr16 failed; tail $O/ab_nr16.jsonl; exit 1; }
tail -1 $O/ab_nr16.jsonl
fi

#!/bin/bash
# Routed gossip merge on the GPU box: parity (round model, shards, processes), the span of both
# stretches (in-process), merge routing counts, kernel traces of both stretches.
set -e
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03m2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1
tail -2 $O/parity.log
timeout -k 10 300 python3 profiles/r03/ab_span.py --flags 0 --reps 3 > $O/ab_span.jsonl
tail -1 $O/ab_span.jsonl
GX_KPROF=1 timeout -k 10 120 python3 profiles/kprof.py --rounds 25 51 55 > $O/kprof.jsonl
grep -o '"merge_paths.*' $O/kprof.jsonl
for st in 21 51; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$st -o run -- \
    python3 profiles/gossip_span.py cfg5 $st 9 > /dev/null
  python3 profiles/r03/stretch_timeline.py $O/trace_$st/run_kernel_trace.csv $st | tail -1
done

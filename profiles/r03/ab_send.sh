#!/bin/bash
# k_send A/B on the GPU box: parity of the round model, the gossip spans of both stretches, the
# k_send phase marks and merge path counts (GX_KPROF), kernel traces of both stretches.
set -e
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03ab}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1
tail -2 $O/parity.log
timeout -k 10 120 python3 profiles/gossip_span.py cfg5 21 9 | tee $O/span21.txt
timeout -k 10 120 python3 profiles/gossip_span.py cfg5 51 9 | tee $O/span51.txt
GX_KPROF=1 timeout -k 10 120 python3 profiles/kprof.py --rounds 21 25 51 52 55 > $O/kprof.jsonl
cat $O/kprof.jsonl
for st in 21 51; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$st -o run -- \
    python3 profiles/gossip_span.py cfg5 $st 9 > /dev/null
  python3 profiles/r03/stretch_timeline.py $O/trace_$st/run_kernel_trace.csv $st | tail -1
done

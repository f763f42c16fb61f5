#!/bin/bash
# Worklist merge (k_merge_wl) A/B on the GPU box: parity, gossip spans of both stretches with the
# worklist merge and with the flag scan (GX_AB_FLAGS=2048), merge path counts, kernel traces; then
# k_ae with two tiles in flight (GX_AB_FLAGS=1024) against one on the accept-heavy configs.
set -e
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03m}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1
tail -2 $O/parity.log
for st in 21 51; do
  timeout -k 10 120 python3 profiles/gossip_span.py cfg5 $st 9 | tee $O/span${st}_wl.txt
  GX_AB_FLAGS=2048 timeout -k 10 120 python3 profiles/gossip_span.py cfg5 $st 9 2>/dev/null | tee $O/span${st}_scan.txt
done
GX_KPROF=1 timeout -k 10 120 python3 profiles/kprof.py --rounds 25 51 55 > $O/kprof.jsonl
cut -c 1-80 $O/kprof.jsonl; grep -o '"merge_paths.*' $O/kprof.jsonl
for st in 21 51; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$st -o run -- \
    python3 profiles/gossip_span.py cfg5 $st 9 > /dev/null
  python3 profiles/r03/stretch_timeline.py $O/trace_$st/run_kernel_trace.csv $st | tail -1
done
for cfg in cfg4 cfg2; do
  for ab in 0 1024; do
    GX_AB_FLAGS=$ab timeout -k 10 200 python3 bench.py --config $cfg --no-converge --no-cpu-baseline > $O/bench_${cfg}_ab$ab.json 2>/dev/null
    python3 -c "import json,sys; d=json.loads(open('$O/bench_${cfg}_ab$ab.json').read().strip().splitlines()[-1]); print('$cfg ab=$ab', round(d['ms_per_step'],4), d['kernels']['ae'])"
  done
done

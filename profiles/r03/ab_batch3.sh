#!/bin/bash
# In-process A/B on the GPU box: the gossip round span (both stretches) for PLAN_RECS 48 (a second
# build, libgx_v48.so) against 32, and the merge variants (64 receivers per block: bit 4096; 4 waves
# per SIMD: bit 8192); then k_ae with default cache policies (bit 32) on the accept-heavy configs.
set -e
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03ab3}
mkdir -p $O
timeout -k 10 500 python3 profiles/r03/ab_span.py --libs sidecar_amd/libgx.so sidecar_amd/libgx_v48.so --flags 0 --reps 3 > $O/ab_plan.jsonl 2>/dev/null
tail -1 $O/ab_plan.jsonl
timeout -k 10 500 python3 profiles/r03/ab_span.py --flags 0 4096 8192 --starts 51 --reps 3 > $O/ab_merge.jsonl 2>/dev/null
tail -1 $O/ab_merge.jsonl
for cfg in cfg4 cfg2; do
  for ab in 0 32 0 32; do
    GX_AB_FLAGS=$ab timeout -k 10 200 python3 bench.py --config $cfg --no-converge --no-cpu-baseline > $O/bench_${cfg}_ab$ab.json 2>/dev/null
    python3 -c "import json; d=json.loads(open('$O/bench_${cfg}_ab$ab.json').read().strip().splitlines()[-1]); print('$cfg ab=$ab', round(d['ms_per_step'],4), d['kernels']['ae']['ms'])"
  done
done

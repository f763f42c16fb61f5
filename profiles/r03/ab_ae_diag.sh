#!/bin/bash
# Diagnosis of k_ae's accept-heavy launches (cfg4, cfg2): server-time bookkeeping skipped (bit
# 16384), retransmit compaction skipped (bit 32768), both; results are not the engine's, only times.
set -e
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03aed}
mkdir -p $O
for cfg in cfg4 cfg2; do
  for ab in 0 16384 32768 49152 0; do
    GX_AB_FLAGS=$ab timeout -k 10 200 python3 bench.py --config $cfg --no-converge --no-cpu-baseline > $O/bench_${cfg}_ab$ab.json 2>/dev/null
    python3 -c "import json; d=json.loads(open('$O/bench_${cfg}_ab$ab.json').read().strip().splitlines()[-1]); print('$cfg ab=$ab', round(d['ms_per_step'],4), d['kernels']['ae']['ms'])"
  done
done

#!/bin/bash
# cfg3 (16384 x 16, 5% churn, 5% aged records): expiry scans in the fused k_send prologue (0) vs
# owner ticks in k_owner and scans in k_scan over the whole chip (12); cfg5 for the gossip round.
set -e
for f in 0 12; do
  GX_AB_FLAGS=$f timeout -k 10 200 python3 bench.py --config cfg3 --no-converge --no-cpu-baseline > gpurun_out/ab_cfg3_$f.json
  python3 -c "import json; d=json.load(open('gpurun_out/ab_cfg3_$f.json')); k=d['kernels']; print('cfg3 flags $f ms/step', round(d['ms_per_step'],3), {n:(v['ms'],v['launches']) for n,v in k.items()})" | tee -a gpurun_out/ab_cfg3.log
done

#!/bin/bash
# A/B of the departure-storm kernel (k_storm_p2): nontemporal row loads and stores (the shipped
# kernel since round 2) vs default ones (GX_AB_FLAGS=16; before this A/B the flag selected NT). The driver's bench window [5, 25) holds the storm; per-kernel
# device time from the bench's split pass, three runs per variant.
set -e
for f in 0 16 0 16 0 16; do
  GX_AB_FLAGS=$f timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-converge --no-cpu-baseline > gpurun_out/ab_storm_$f.json
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_storm_$f.json')); k=d['kernels']['storm']; print('flags $f storm ms', k['ms'], 'GBps', k['GBps'], 'ms/step', round(d['ms_per_step'],3))" | tee -a gpurun_out/ab_storm.log
done

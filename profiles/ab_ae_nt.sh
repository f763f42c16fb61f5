#!/bin/bash
# A/B of the push-pull kernel's cache policy (run before the switch; see profiles/ab/ae_nt_ab_r02.log):
# GX_AB_FLAGS=32 nontemporal stores of changed slots,
# 64 nontemporal loads and stores, 0 the shipped k_ae. The bench's default 100-round window
# (ten push-pull rounds, four of them after the heal with heavy write-back).
set -e
for f in 0 32 64 0 32 64; do
  GX_AB_FLAGS=$f timeout -k 10 200 python3 bench.py --no-converge --no-cpu-baseline > gpurun_out/ab_ae_$f.json
  python3 -c "import json; d=json.load(open('gpurun_out/ab_ae_$f.json')); k=d['kernels']; print('flags $f ae ms', k['ae']['ms'], 'GBps', k['ae']['GBps'], 'storm ms', k['storm']['ms'], 'ms/step', round(d['ms_per_step'],3))" | tee -a gpurun_out/ab_ae.log
done

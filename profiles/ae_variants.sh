#!/bin/bash
# A/B of the push-pull kernel variants (GX_AE_VARIANT: 0 PF1, 1 PF1+nt, 2 PF2, 3 PF2+nt) on cfg5.
set -o pipefail
mkdir -p gpurun_out
for v in 0 1 2 3 0; do
  GX_AE_VARIANT=$v timeout -k 10 240 python3 bench.py --config cfg5 --steps 30 --no-converge --no-cpu-baseline \
    > gpurun_out/aev_$v.json || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/aev_$v.json').readline());k=d['kernels']['ae'];print('variant $v', round(k['ms']/k['launches'],3),'ms/launch', k['GBps'],'GB/s')"
done

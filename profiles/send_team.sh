#!/bin/bash
# A/B of the GetBroadcasts team size (GX_SEND_TEAM lanes per host) on cfg5, 30 rounds.
set -o pipefail
mkdir -p gpurun_out
for t in 1 4 8 16 64 8; do
  GX_SEND_TEAM=$t timeout -k 10 240 python3 bench.py --config cfg5 --steps 30 --no-converge --no-cpu-baseline \
    > gpurun_out/send_$t.json || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/send_$t.json').readline());k=d['kernels']['send'];m=d['kernels']['merge'];print('team $t send', round(1000*k['ms']/k['launches'],1),'us  merge', round(1000*m['ms']/m['launches'],1), 'us', d['merges'])"
done

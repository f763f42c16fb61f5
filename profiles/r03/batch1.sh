#!/bin/bash
# One GPU call: round-model parity tests + gossip-stretch profiles, the streaming kernels at
# cfg2/cfg4/cfg3, and the full-size 8-way LocalShards check (profiles/sharded_local_cfg5.py).
set -e
bash profiles/r03/gossip_prof.sh
bash profiles/r03/stream_prof.sh
mkdir -p gpurun_out/r03g
timeout -k 10 420 python3 -u profiles/sharded_local_cfg5.py 8 91 32768 51,61,91 > gpurun_out/r03g/sharded_g8_h32768.json
tail -c 600 gpurun_out/r03g/sharded_g8_h32768.json

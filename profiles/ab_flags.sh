#!/bin/bash
# A/B of gossip-path kernel variants selected by GX_AB_FLAGS (bit 0: sequential GetBroadcasts instead
# of the planned record-mode send; bit 1: 16 lanes x 8 records per receiver in k_merge_lean) on the
# cfg5 bench, kernel trace per variant; then SQ counters of variant $1 in one --pmc pass.
set -e
export TMPDIR=/tmp
for f in 0 1 2 3; do
  mkdir -p gpurun_out/ab_flags_$f
  GX_AB_FLAGS=$f timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_flags_$f -o run -- python3 bench.py --config cfg5 --steps 30 --no-converge --no-cpu-baseline --no-kernel-split > gpurun_out/ab_flags_$f/bench.json
done
mkdir -p gpurun_out/ab_pmc
GX_AB_FLAGS=${1:-1} timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d gpurun_out/ab_pmc -o run -- python3 bench.py --config cfg5 --steps 12 --no-converge --no-cpu-baseline --no-kernel-split > gpurun_out/ab_pmc/bench.json

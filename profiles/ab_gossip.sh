#!/bin/bash
# Kernel trace of the cfg5 gossip rounds per GX_AB_FLAGS variant given as arguments (bit 2: the
# expiry scans in their own k_scan launch instead of k_send's prologue); per-round timeline each.
set -e
export TMPDIR=/tmp
for f in "$@"; do
  mkdir -p gpurun_out/ab_g_$f
  GX_AB_FLAGS=$f timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_g_$f -o run -- python3 bench.py --config cfg5 --steps 30 --no-converge --no-cpu-baseline --no-kernel-split > gpurun_out/ab_g_$f/bench.json
  echo "== GX_AB_FLAGS=$f"
  python3 profiles/round_timeline.py gpurun_out/ab_g_$f/run_kernel_trace.csv
done

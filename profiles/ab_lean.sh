#!/bin/bash
# A/B of k_merge_lean's inline-record loads (GX_AB_FLAGS bit 0: speculative loads of the first
# `fanout` slots only; bit 1: no speculation, records loaded once the lengths are known) on the
# cfg5 bench, kernel trace per variant; then FETCH_SIZE and WRITE_SIZE passes (variant 0).
set -e
export TMPDIR=/tmp
for f in 0 1 2; do
  mkdir -p gpurun_out/ab_lean_$f
  GX_AB_FLAGS=$f timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_lean_$f -o run -- python3 bench.py --config cfg5 --steps 30 --no-converge --no-cpu-baseline --no-kernel-split > gpurun_out/ab_lean_$f/bench.json
  python3 profiles/round_timeline.py gpurun_out/ab_lean_$f/run_kernel_trace.csv > gpurun_out/ab_lean_$f/timeline.txt
done
for c in FETCH_SIZE WRITE_SIZE; do
  mkdir -p gpurun_out/pmc_$c
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_$c -o run -- python3 bench.py --config cfg5 --steps 12 --no-converge --no-cpu-baseline --no-kernel-split > gpurun_out/pmc_$c/bench.json
done

#!/bin/bash
# A/B of the receiver inbox's inline packet slots (DR) on the cfg5 bench: kernel trace per variant.
set -e
export TMPDIR=/tmp
for dr in 4 8 2; do
  mkdir -p gpurun_out/ab_inline_$dr
  GX_AB_INLINE_SLOTS=$dr timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_inline_$dr -o run -- python3 bench.py --config cfg5 --steps 30 --no-converge --no-cpu-baseline --no-kernel-split > gpurun_out/ab_inline_$dr/bench.json
done

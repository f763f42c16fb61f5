#!/bin/bash
# Round 4, first GPU pass after the stored-window FIFO: the default bench (cfg 5), the driver's
# window, and a kernel trace of the window. Run on the GPU box from the repo root.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 600 python3 bench.py > gpurun_out/r04/bench_cfg5_default.json
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04/bench_cfg5_driver_window.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04/trace -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-converge --no-cpu-baseline > gpurun_out/r04/bench_trace.json

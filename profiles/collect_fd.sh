#!/bin/bash
# Kernel trace + stats of the failure-detection bench (fd_depart: 16384 x 16, 2% of hosts crash at
# round 5) and of cfg5fd, for the fd kernels' per-launch times. Outputs under gpurun_out/prof_fd_<tag>/.
set -e
TAG=${1:-r01}
export TMPDIR=/tmp
OUT=gpurun_out/prof_fd_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/fd_depart -o run -- \
  python3 bench.py --config fd_depart --steps 100 --no-converge --no-cpu-baseline > $OUT/fd_depart_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/cfg5fd -o run -- \
  python3 bench.py --config cfg5fd --steps 100 --no-converge --no-cpu-baseline > $OUT/cfg5fd_bench.json

#!/bin/bash
# Final round-3 bench lines and profiles: the driver's window, the default 100-round window, then a
# kernel trace + stats of the default window and FETCH_SIZE / WRITE_SIZE passes (profiles/collect.sh).
set -e
export TMPDIR=/tmp
O=gpurun_out/r03final
mkdir -p $O
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err
tail -c 400 $O/bench_driver.json
timeout -k 10 300 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err
tail -c 300 $O/bench_default.json
bash profiles/collect.sh r03f 20

#!/bin/bash
# Streaming kernels at the other configs: for each config a kernel trace +
# stats of the default bench window, then FETCH_SIZE and WRITE_SIZE passes (separate --pmc runs)
# and one SQ pass (busy / wave cycles). Outputs under gpurun_out/${TAG:-r03s}/<cfg>/.
set -e
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03s}
for cfg in ${CONFIGS:-cfg2 cfg4 cfg3}; do
  D=$O/$cfg
  mkdir -p $D
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- \
    python3 bench.py --config $cfg --no-converge --no-cpu-baseline --no-kernel-split > $D/bench_trace.json
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o run -- \
    python3 bench.py --config $cfg --no-converge --no-cpu-baseline --no-kernel-split > $D/bench_fetch.json
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o run -- \
    python3 bench.py --config $cfg --no-converge --no-cpu-baseline --no-kernel-split > $D/bench_write.json
  echo "$cfg done"
done

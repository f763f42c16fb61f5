#!/bin/bash
# Storm kernel: one 16-B server-time store and no division per EXPIRE job (libgx.so) against the
# previous build (libgx_prev.so), alternating processes on the driver's cfg 5 window; parity after.
set -e
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03st}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kat.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
for lib in libgx.so libgx_prev.so libgx.so libgx_prev.so libgx.so libgx_prev.so; do
  GX_LIB=sidecar_amd/$lib timeout -k 10 200 python3 profiles/r03/bench_lib.py --steps 20 --warmup 5 --no-converge --no-cpu-baseline > $O/bench_$lib.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('$O/bench_$lib.json').read().strip().splitlines()[-1]); print('$lib', round(d['ms_per_step'],4), d['kernels']['storm']['ms'], d['kernels']['ae']['ms'])"
done

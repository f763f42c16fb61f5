#!/bin/bash
# k_ae FIFO positions without a division per job (libgx.so) against the previous build
# (libgx_prev.so), alternating processes on cfg2, cfg4, cfg5; then the parity tests on the new build.
set -e
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03aent}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards.py tests/test_gpu_codec.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
for cfg in cfg2 cfg4 cfg5; do
  for lib in libgx.so libgx_prev.so libgx.so libgx_prev.so; do
    GX_LIB=sidecar_amd/$lib timeout -k 10 200 python3 profiles/r03/bench_lib.py --config $cfg --no-converge --no-cpu-baseline > $O/bench_${cfg}_$lib.json 2>/dev/null
    python3 -c "import json; d=json.loads(open('$O/bench_${cfg}_$lib.json').read().strip().splitlines()[-1]); print('$cfg $lib', round(d['ms_per_step'],4), d['kernels']['ae']['ms'])"
  done
done

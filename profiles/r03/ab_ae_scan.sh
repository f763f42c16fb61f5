#!/bin/bash
# k_ae retransmit scan with one barrier (default) against the barrier-or + two-barrier scan (bit
# 65536), interleaved, on cfg4, cfg2 and the default cfg5 window; then the push-pull parity tests.
set -e
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03aes}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards.py tests/test_gpu_codec.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
for cfg in cfg2 cfg5 cfg4; do
  for ab in 0 65536 0 65536; do
    GX_AB_FLAGS=$ab timeout -k 10 200 python3 bench.py --config $cfg --no-converge --no-cpu-baseline > $O/bench_${cfg}_ab$ab.json 2>/dev/null
    python3 -c "import json; d=json.loads(open('$O/bench_${cfg}_ab$ab.json').read().strip().splitlines()[-1]); print('$cfg ab=$ab', round(d['ms_per_step'],4), d['kernels']['ae']['ms'])"
  done
done

#!/bin/bash
# Final round-3 bench lines at the other configs and a kernel-stats profile of cfg5_defaults.
set -e
export TMPDIR=/tmp
O=gpurun_out/r03final3
mkdir -p $O
for cfg in cfg2 cfg4 cfg3; do
  timeout -k 10 300 python3 -u bench.py --config $cfg --no-cpu-baseline > $O/bench_$cfg.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('$O/bench_$cfg.json').read().strip().splitlines()[-1]); print('$cfg', round(d['ms_per_step'],4), '%.3e' % d['value'], d['roofline']['kernel'], d['roofline']['frac'], (d['converge'] or {}).get('rounds_to_converge'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gm15 -o run -- \
  python3 bench.py --config cfg5_defaults --steps 60 --warmup 45 --no-converge --no-cpu-baseline > $O/gm15_bench.json

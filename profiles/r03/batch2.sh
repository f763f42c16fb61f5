#!/bin/bash
# GossipMessages 15 at scale and the churn config: the H = 16384 GM 15 parity test and the full-size
# tests, cfg5_defaults (Sidecar's defaults) and cfg3 (dissemination latency) bench lines, cfg5fd
# with GossipMessages 15 over 3000 rounds (does the catalog settle?).
set -e
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03b2}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 600 --timeout-method thread > $O/fullsize.log 2>&1
grep -E "PASSED|FAILED|passed|failed" $O/fullsize.log | tail -12
timeout -k 10 300 python3 -u bench.py --config cfg5_defaults --no-cpu-baseline > $O/bench_cfg5_defaults.json 2> $O/bench_cfg5_defaults.err
python3 -c "import json; d=json.loads(open('$O/bench_cfg5_defaults.json').read().strip().splitlines()[-1]); print('cfg5_defaults', d['ms_per_step'], d['value'], d['converge'], d['gossip']['round_span_us'], d['gossip'].get('round_span_us_accepting'))"
timeout -k 10 300 python3 -u bench.py --config cfg3 --no-cpu-baseline > $O/bench_cfg3.json 2> $O/bench_cfg3.err
python3 -c "import json; d=json.loads(open('$O/bench_cfg3.json').read().strip().splitlines()[-1]); print('cfg3', d['ms_per_step'], d['value'], d['dissemination'])"
timeout -k 10 400 python3 -u profiles/fd_reconverge.py 32768 3000 50 100 gpu 15 > $O/cfg5fd_gm15_reconverge_3000.jsonl
tail -3 $O/cfg5fd_gm15_reconverge_3000.jsonl

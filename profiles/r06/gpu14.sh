#!/bin/bash
# bench sanity after lock_readers (default 0): cfg 5 default line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g14
mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { echo bench failed; tail -20 $O/bench_cfg5.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench_cfg5.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['gossip']['device_us_per_round'], d['gossip']['round_span_us_accepting'], d['gossip']['lock_off']['round_span_us'], d['gossip']['lock_off']['round_span_us_accepting'])"

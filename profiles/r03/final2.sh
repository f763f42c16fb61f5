#!/bin/bash
# Final round-3 tree: every -m gpu test, smoke(), and the cfg5_defaults bench line (GossipMessages 15).
set -e
export TMPDIR=/tmp
O=gpurun_out/r03final2
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
cat $O/smoke.log
timeout -k 10 300 python3 -u bench.py --config cfg5_defaults --no-cpu-baseline --converge-max 1000 > $O/bench_cfg5_defaults.json 2>/dev/null
python3 -c "import json; d=json.loads(open('$O/bench_cfg5_defaults.json').read().strip().splitlines()[-1]); g=d['gossip']; print(d['ms_per_step'], g['round_span_us'], g['roofline']['frac'], g['round_span_us_accepting'], g['roofline_accepting']['frac'])"

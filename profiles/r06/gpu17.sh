#!/bin/bash
# scan at cfg 3: occupancy variants (waves per EU 6 / 8 with spills, two tiles in flight) against the base build;
# then the cfg 5 bench line at the driver's K/W
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g17
mkdir -p $O
L=profiles/r06/ablib
for lm in 0 1; do
timeout -k 10 500 python -u profiles/r04/ab_kernels.py --config cfg3 --skip 100 --rounds 30 --reps 3 --lock-model $lm \
  --libs $L/libgx_scan_base.so $L/libgx_scan_wpe6.so $L/libgx_scan_wpe8.so $L/libgx_scan_pf2w6.so > $O/ab_scan_cfg3_lm$lm.jsonl 2>&1 || { echo ab failed; tail $O/ab_scan_cfg3_lm$lm.jsonl; exit 1; }
tail -1 $O/ab_scan_cfg3_lm$lm.jsonl
done
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { echo bench failed; tail -20 $O/bench_cfg5.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench_cfg5.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['gossip']['device_us_per_round'], d['gossip']['round_span_us_accepting'], d['gossip']['lock_off']['round_span_us'], d['gossip']['lock_off']['round_span_us_accepting'])"

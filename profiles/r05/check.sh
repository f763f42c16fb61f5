#!/bin/bash
# After an engine change: the GPU parity suites, then the gossip phase marks and stretches.
#   bash profiles/r05/check.sh <tag> [full]
# "full" adds the full-size parity tests (cfg 5 and GossipMessages 15 at H = 32768, cfg 3).
set -e
TAG=${1:-chk}
O=gpurun_out/r05/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_lock.py tests/test_gpu_shards.py tests/test_gpu_kat.py > $O/parity.log 2>&1
tail -1 $O/parity.log
if [ "$2" = full ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 550 --timeout-method thread tests/test_gpu_fullsize.py \
    -k "h32768 or bench_schedule" > $O/fullsize.log 2>&1
  tail -1 $O/fullsize.log
fi
for lm in 1 0; do
  GX_KPROF=1 timeout -k 10 200 python -u profiles/kprof.py --rounds 21 51 --lock-model $lm > $O/kprof_cfg5_$lm.jsonl 2>&1
  GX_KPROF=1 timeout -k 10 200 python -u profiles/kprof.py --config cfg5_defaults --rounds 21 51 --lock-model $lm \
    > $O/kprof_gm15_$lm.jsonl 2>&1
done
timeout -k 10 300 python -u profiles/r05/spans.py > $O/spans.jsonl 2>&1
cat $O/spans.jsonl

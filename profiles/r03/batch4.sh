#!/bin/bash
# Round-model, detector, shard and process parity on the final merge routing, then cfg5fd with
# GossipMessages 15 (does the catalog settle?) and cfg5_defaults' disagreement trajectory.
set -e
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03b4}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fd.py tests/test_gpu_shards.py tests/test_gpu_dist.py tests/test_gpu_kat.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
timeout -k 10 500 python3 -u profiles/fd_reconverge.py 32768 3000 50 100 gpu 15 > $O/cfg5fd_gm15_reconverge_3000.jsonl
tail -2 $O/cfg5fd_gm15_reconverge_3000.jsonl
timeout -k 10 300 python3 -u bench.py --config cfg5_defaults --no-cpu-baseline --no-kernel-split > $O/bench_cfg5_defaults.json 2>/dev/null
python3 -c "import json; d=json.loads(open('$O/bench_cfg5_defaults.json').read().strip().splitlines()[-1]); print(d['converge'])"

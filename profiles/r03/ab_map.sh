#!/bin/bash
# Written-slot map in the multi-tile wave merge (libgx.so) against the previous build
# (libgx_prev.so): parity first (round model incl. GossipMessages and wide inboxes, full-size GM 15),
# then the gossip spans of cfg5_defaults (GossipMessages 15) and cfg5, in one process per config.
set -e
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03map}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards.py tests/test_gpu_fd.py "tests/test_gpu_fullsize.py::test_cfg5_gossip_messages15_h16384_parity" -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
timeout -k 10 400 python3 profiles/r03/ab_span.py --config cfg5_defaults --libs sidecar_amd/libgx.so sidecar_amd/libgx_prev.so --flags 0 --reps 2 > $O/ab_gm15.jsonl 2>/dev/null
tail -1 $O/ab_gm15.jsonl
timeout -k 10 400 python3 profiles/r03/ab_span.py --config cfg5 --libs sidecar_amd/libgx.so sidecar_amd/libgx_prev.so --flags 0 --reps 2 --starts 51 > $O/ab_cfg5.jsonl 2>/dev/null
tail -1 $O/ab_cfg5.jsonl

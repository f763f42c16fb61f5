#!/bin/bash
# Pipelined planned sends under GossipMessages 15 (default there) against the unpipelined loop
# (bit 16384); parity of the GossipMessages scenarios and the H = 16384 GM 15 test first.
set -e
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03pipe}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fd.py tests/test_gpu_shards.py "tests/test_gpu_fullsize.py::test_cfg5_gossip_messages15_h16384_parity" -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
timeout -k 10 500 python3 profiles/r03/ab_span.py --config cfg5_defaults --flags 0 16384 --reps 2 > $O/ab_gm15.jsonl 2>/dev/null
tail -1 $O/ab_gm15.jsonl

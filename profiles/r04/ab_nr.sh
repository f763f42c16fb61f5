#!/bin/bash
# A/B of the gossip merge's receivers per block at GossipMessages 1 (cfg 5 accepting rounds 51..58,
# and the dead rounds 21..28)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04
L=$R/profiles/r04/lib
timeout -k 10 300 python3 -u $R/profiles/r04/ab_kernels.py --config cfg5 --skip 51 --rounds 8 --reps 3 --libs $L/libgx_base.so $L/libgx_nr32.so $L/libgx_nr16.so > $O/ab_nr_gm1.jsonl
tail -1 $O/ab_nr_gm1.jsonl

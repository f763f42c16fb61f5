#!/bin/bash
# A/B of the gossip merge: libgx_base (HEAD) vs libgx_mpipe (two-deep tile pipeline in
# merge_receiver), accepting rounds at GossipMessages 15 and 1
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04
timeout -k 10 300 python3 -u $R/profiles/r04/ab_kernels.py --config cfg5_defaults --skip 50 --rounds 9 --reps 2 --libs $R/profiles/r04/lib/libgx_base.so $R/profiles/r04/lib/libgx_mpipe.so $R/profiles/r04/lib/libgx_mset.so > $O/ab_mset_gm15.jsonl
tail -1 $O/ab_mset_gm15.jsonl
timeout -k 10 300 python3 -u $R/profiles/r04/ab_kernels.py --config cfg5 --skip 51 --rounds 8 --reps 2 --libs $R/profiles/r04/lib/libgx_base.so $R/profiles/r04/lib/libgx_mpipe.so $R/profiles/r04/lib/libgx_mset.so > $O/ab_mset_gm1.jsonl
tail -1 $O/ab_mset_gm1.jsonl

#!/bin/bash
# A/B of the push-pull accept path: server times stored by the group's flagged lane (libgx_stimes)
# vs shuffled to the group's first lane (libgx_base), accept-heavy launches
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04
L=$R/profiles/r04/lib
timeout -k 10 300 python3 -u $R/profiles/r04/ab_kernels.py --config cfg4 --skip 5 --rounds 60 --reps 2 --libs $L/libgx_base.so $L/libgx_acc.so > $O/ab_acc_cfg4.jsonl
tail -1 $O/ab_acc_cfg4.jsonl
timeout -k 10 300 python3 -u $R/profiles/r04/ab_kernels.py --config cfg5 --skip 49 --rounds 22 --reps 2 --libs $L/libgx_base.so $L/libgx_acc.so > $O/ab_acc_cfg5.jsonl
tail -1 $O/ab_acc_cfg5.jsonl
timeout -k 10 300 python3 -u $R/profiles/r04/ab_kernels.py --config cfg2 --skip 5 --rounds 60 --reps 2 --libs $L/libgx_base.so $L/libgx_acc.so > $O/ab_acc_cfg2.jsonl
tail -1 $O/ab_acc_cfg2.jsonl

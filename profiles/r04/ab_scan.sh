#!/bin/bash
# A/B of the expiry scan at cfg 3: compiled for 4 (HEAD), 5 and 6 waves per SIMD (more rows resident)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04
L=$R/profiles/r04/lib
timeout -k 10 400 python3 -u $R/profiles/r04/ab_kernels.py --config cfg3 --skip 100 --rounds 30 --reps 2 --libs $L/libgx_base.so $L/libgx_swpe5.so $L/libgx_swpe6.so > $O/ab_swpe_cfg3.jsonl
tail -1 $O/ab_swpe_cfg3.jsonl

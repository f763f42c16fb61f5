#!/bin/bash
# A/B of k_ae resident waves per SIMD (GX_AE_WPE 4 = product, 5, 6; spills at 5 and 6), lock off.
set -e
O=gpurun_out/r05/wpe
mkdir -p $O
L="profiles/r05/lib/libgx_nodf.so profiles/r05/lib/libgx_wpe5.so profiles/r05/lib/libgx_wpe6.so"
timeout -k 10 300 python3 -u profiles/r04/ab_kernels.py --config cfg2 --skip 0 --rounds 60 --reps 2 --lock-model 0 --libs $L > $O/ab_cfg2.jsonl 2> $O/ab_cfg2.err
timeout -k 10 300 python3 -u profiles/r04/ab_kernels.py --config cfg4 --skip 0 --rounds 40 --reps 2 --lock-model 0 --libs $L > $O/ab_cfg4.jsonl 2> $O/ab_cfg4.err
timeout -k 10 300 python3 -u profiles/r04/ab_kernels.py --config cfg5 --skip 49 --rounds 2 --reps 2 --lock-model 0 --libs $L > $O/ab_cfg5.jsonl 2> $O/ab_cfg5.err

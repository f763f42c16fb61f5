#!/bin/bash
# A/B of k_ae's deferred retransmit compaction (DF) against the build before it, lock off (the
# kernel measurement), cfg 2 / 4 / 5.
set -e
O=gpurun_out/r05/df
mkdir -p $O
L="sidecar_amd/libgx.so profiles/r05/lib/libgx_nodf.so"
timeout -k 10 300 python3 -u profiles/r04/ab_kernels.py --config cfg2 --skip 0 --rounds 60 --reps 2 --lock-model 0 --libs $L > $O/ab_cfg2.jsonl 2> $O/ab_cfg2.err
timeout -k 10 300 python3 -u profiles/r04/ab_kernels.py --config cfg4 --skip 0 --rounds 40 --reps 2 --lock-model 0 --libs $L > $O/ab_cfg4.jsonl 2> $O/ab_cfg4.err
timeout -k 10 300 python3 -u profiles/r04/ab_kernels.py --config cfg5 --skip 49 --rounds 2 --reps 2 --lock-model 0 --libs $L > $O/ab_cfg5.jsonl 2> $O/ab_cfg5.err

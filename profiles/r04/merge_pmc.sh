#!/bin/bash
# SQ counters of the gossip merge (k_merge_seg) and send (k_send) over cfg5_defaults rounds 0..60
# (GossipMessages 15: dead partition rounds, the heal at 50, accepting rounds 51..59), one pass.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04/merge_pmc
mkdir -p $O
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex "k_merge_seg|k_send" -d $O/gm15 -o pmc -- python3 $R/profiles/kprof.py --config cfg5_defaults --rounds 55

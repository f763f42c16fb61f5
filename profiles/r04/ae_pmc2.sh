#!/bin/bash
# SQ counters of k_ae in a partitioned (10) and a post-heal (60) push-pull round of cfg 5
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04/ae_pmc2
mkdir -p $O
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR"
timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex "k_ae" -d $O/sq -o pmc -- python3 $R/profiles/kprof.py --config cfg5 --rounds --ae-rounds 10 60

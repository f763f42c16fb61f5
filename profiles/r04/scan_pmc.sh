#!/bin/bash
# SQ counters of the expiry scan (k_scan) at cfg 3 (rounds 101..102), one pass
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04/scan_pmc
mkdir -p $O
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD"
timeout -s KILL 200 rocprofv3 --pmc $C --kernel-include-regex "k_scan" -d $O/sq -o pmc -- python3 $R/profiles/kprof.py --config cfg3 --rounds --scan-rounds 101 102
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_scan" -d $O/fetch -o pmc -- python3 $R/profiles/kprof.py --config cfg3 --rounds --scan-rounds 101 102
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_scan" -d $O/write -o pmc -- python3 $R/profiles/kprof.py --config cfg3 --rounds --scan-rounds 101 102

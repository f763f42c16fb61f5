#!/bin/bash
# SQ counters of the push-pull kernel (cfg 5, AE round 10) and of the pair-stream microbenchmark's
# kernels, one rocprofv3 pass each (8 SQ counters), for the instruction/wait mix of k_ae against
# a pure stream of the same rows.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04/ae_pmc
mkdir -p $O
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD"
timeout -s KILL 200 rocprofv3 --pmc $C --kernel-include-regex "k_ae" -d $O/eng -o pmc -- python3 $R/profiles/kprof.py --config cfg5 --rounds --ae-rounds 10
timeout -s KILL 200 rocprofv3 --pmc $C --kernel-include-regex "k_reg" -d $O/mb -o pmc -- $R/profiles/r04/stream_pair_bench
# per-block push-pull marks at the accept-heavy configs (cold start cfg 2, cfg 4) and cfg 3
for c in cfg2 cfg4 cfg3; do
  GX_KPROF=1 timeout -k 10 200 python3 -u $R/profiles/kprof.py --config $c --rounds --ae-rounds 10 20 50 > $R/gpurun_out/r04/kprof_ae_$c.jsonl
done

#!/bin/bash
# Round 3 gossip-path profile on the GPU box: the parity tests of the round model, then for the
# dead stretch (cfg 5 rounds 21..29) and the accepting stretch (51..59) a kernel trace and
# FETCH_SIZE / WRITE_SIZE passes (separate --pmc runs, MI355X_MICROARCH.md §HBM) of
# profiles/gossip_span.py. Outputs under gpurun_out/r03g/; summarise with profiles/r03/gossip_pmc.py.
set -e
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03g}
mkdir -p $O
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1
  tail -2 $O/parity.log
fi
for st in ${STRETCHES:-21 51}; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$st -o run -- \
    python3 profiles/gossip_span.py cfg5 $st 9 > $O/span_$st.txt
  cat $O/span_$st.txt
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$st -o run -- \
    python3 profiles/gossip_span.py cfg5 $st 9 > $O/span_fetch_$st.txt
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$st -o run -- \
    python3 profiles/gossip_span.py cfg5 $st 9 > $O/span_write_$st.txt
done

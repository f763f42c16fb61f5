#!/bin/bash
# cfg5_defaults (GossipMessages 15): kernel traces of a dead and an accepting gossip stretch,
# k_send phase marks and merge routing counts.
set -e
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03gm}
mkdir -p $O
for st in 21 51; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$st -o run -- \
    python3 profiles/gossip_span.py cfg5_defaults $st 9 > $O/span_$st.txt
  cat $O/span_$st.txt
  python3 profiles/r03/stretch_timeline.py $O/trace_$st/run_kernel_trace.csv $st | tail -3
done
GX_KPROF=1 timeout -k 10 120 python3 profiles/kprof.py --config cfg5_defaults --rounds 25 55 > $O/kprof.jsonl
cat $O/kprof.jsonl | cut -c 1-1200

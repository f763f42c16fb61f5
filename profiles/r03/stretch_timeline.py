"""Per-round kernel durations of one gossip stretch from a rocprofv3 kernel trace of
profiles/gossip_span.py: round r's k_send and merge launch are the r-th of each (one per round).

  python profiles/r03/stretch_timeline.py <run_kernel_trace.csv> r0 [n=9]
"""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
r0 = int(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 9
seq = {}
for r in rows:
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
    seq.setdefault(k, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
merge = next(k for k in ("k_merge_wl", "k_merge_seg", "k_merge") if k in seq)
sends, merges, spans, gaps = [], [], [], []
for r in range(r0, r0 + n):
    s, m = seq["k_send"][r], seq[merge][r]
    sends.append((s[1] - s[0]) / 1e3)
    merges.append((m[1] - m[0]) / 1e3)
    gaps.append((m[0] - s[1]) / 1e3)
    if r + 1 < len(seq["k_send"]):
        spans.append((seq["k_send"][r + 1][0] - s[0]) / 1e3)
    print(f"round {r}: k_send {sends[-1]:6.1f} us, gap {gaps[-1]:5.1f}, {merge} {merges[-1]:6.1f} us"
          + (f", next send after {spans[-1]:6.1f} us" if spans else ""))
print(f"median: k_send {statistics.median(sends):.1f} us, {merge} {statistics.median(merges):.1f} us, "
      f"send->merge gap {statistics.median(gaps):.1f} us, round start->start {statistics.median(spans[:-1] or spans):.1f} us")

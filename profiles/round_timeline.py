"""Per-round kernel timeline of the gossip path from a rocprofv3 kernel trace: for every round
(from k_owner, or from k_send when it runs the owner ticks itself), each kernel's duration and
the round's device span from the first dispatch's start to the last gossip kernel's end
(push-pull and storm kernels excluded).

  python profiles/round_timeline.py <run_kernel_trace.csv> [skip_rounds]
"""
import csv
import statistics
import sys

GOSSIP = ("k_owner", "k_scan", "k_bt_finish", "k_send", "k_merge_lean", "k_merge", "k_merge_seg")
rows = list(csv.DictReader(open(sys.argv[1])))
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 2
ks = []
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n))
ks.sort()
rounds, cur = [], None
for s, e, n in ks:
    # a round starts at k_owner, or at k_send when the owner ticks run inside it (fused launch)
    if n == "k_owner" or (n == "k_send" and (cur is None or any(x[2] in ("k_merge", "k_merge_lean", "k_merge_seg") for x in cur))):
        cur = []
        rounds.append(cur)
    if cur is not None and n in GOSSIP:
        cur.append((s, e, n))
rounds = [r for r in rounds if r][skip:]
per = {}
spans = []
for r in rounds:
    spans.append((r[-1][1] - r[0][0]) / 1e3)
    for s, e, n in r:
        per.setdefault(n, []).append((e - s) / 1e3)
print(f"{len(rounds)} rounds; device span per round: median {statistics.median(spans):.1f} us, "
      f"mean {statistics.mean(spans):.1f} us, min {min(spans):.1f} us")
for n in GOSSIP:
    if n in per:
        v = per[n]
        print(f"  {n:14s} {len(v):4d} launches  median {statistics.median(v):7.1f} us  mean {statistics.mean(v):7.1f} us")
busy = [sum(e - s for s, e, _ in r) / 1e3 for r in rounds]
print(f"  kernel-busy per round: median {statistics.median(busy):.1f} us (gaps = span - busy)")

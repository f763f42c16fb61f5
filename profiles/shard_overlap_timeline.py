"""Per-stream timeline of the push-pull rounds in a rocprofv3 kernel trace of shard_overlap.py:
for each push-pull round, the shard-local k_ae_plan dispatches on the engines' side streams and
the exchange-stage kernels on torch's stream that ran while they did.

  python profiles/shard_overlap_timeline.py <run_kernel_trace.csv>
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    r["n"] = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
rows.sort(key=lambda r: r["s"])
side = [r for r in rows if "ae_plan" in r["n"] and r["Stream_Id"] != "0"]
# side-stream dispatches of one push-pull round start within 1 ms of each other
rounds = []
for r in side:
    if rounds and r["s"] - rounds[-1][0]["s"] < 1_000_000:
        rounds[-1].append(r)
    else:
        rounds.append([r])
t0 = rows[0]["s"]
for g in rounds:
    lo, hi = min(r["s"] for r in g), max(r["e"] for r in g)
    main = [r for r in rows if r["Stream_Id"] == "0" and r["e"] > lo and r["s"] < hi]
    busy = sum(min(r["e"], hi) - max(r["s"], lo) for r in main)
    print(f"push-pull round at {(lo - t0) / 1e6:.3f} ms: side-stream local merges {len(g)} dispatches, "
          f"window {(hi - lo) / 1e3:.1f} us; torch-stream kernels inside it {len(main)}, busy {busy / 1e3:.1f} us "
          f"({100.0 * busy / (hi - lo):.0f}%)")
    for r in sorted(g + main, key=lambda r: r["s"]):
        print(f"   {(r['s'] - lo) / 1e3:9.1f} +{(r['e'] - r['s']) / 1e3:8.1f} us  stream {r['Stream_Id']}  {r['n']}")

"""Total and mean device time per kernel name in a rocprofv3 kernel trace (optionally only the
dispatches whose name contains a filter), sorted by total.

  python profiles/kernel_totals.py <run_kernel_trace.csv> [filter]
"""
import csv
import sys

flt = sys.argv[2] if len(sys.argv) > 2 else ""
tot = {}
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if flt not in n:
        continue
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    t = tot.setdefault(n, [0.0, 0])
    t[0] += d
    t[1] += 1
for n, (ms, k) in sorted(tot.items(), key=lambda x: -x[1][0])[:25]:
    print(f"{ms:10.3f} ms {k:6d} x {1e3 * ms / k:9.1f} us  {n}")

"""Per-launch duration and HBM traffic of the streaming kernels (k_ae, k_scan, k_storm*) from a
profiles/r03/stream_prof.sh run: kernel trace + FETCH_SIZE / WRITE_SIZE passes of the same bench.
traffic = 2 x FETCH + WRITE (gfx950 streaming correction, MI355X_MICROARCH.md §HBM).

  python profiles/r03/stream_summary.py gpurun_out/r03s cfg2 [cfg4 ...]
"""
import csv
import json
import sys

KS = ("k_ae", "k_scan", "k_storm_p2", "k_storm")


def name(r):
    return r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]


def seq(path, key):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r[key]))
    out = {}
    for r in rows:
        out.setdefault(name(r), []).append(r)
    return out


src = sys.argv[1]
res = {}
for cfg in sys.argv[2:]:
    tr = seq(f"{src}/{cfg}/trace/run_kernel_trace.csv", "Start_Timestamp")
    fe = seq(f"{src}/{cfg}/fetch/run_counter_collection.csv", "Dispatch_Id")
    wr = seq(f"{src}/{cfg}/write/run_counter_collection.csv", "Dispatch_Id")
    res[cfg] = {}
    for k in KS:
        if k not in tr:
            continue
        us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in tr[k]]
        f = [float(r["Counter_Value"]) * 1024 for r in fe.get(k, [])]
        w = [float(r["Counter_Value"]) * 1024 for r in wr.get(k, [])]
        n = min(len(us), len(f), len(w))
        tb = [(2 * f[i] + w[i]) for i in range(n)]
        res[cfg][k] = {"launches": len(us), "us": [round(x, 1) for x in us],
                       "traffic_GB": [round(x / 1e9, 3) for x in tb],
                       "write_GB": [round(x / 1e9, 3) for x in w[:n]],
                       "TBps_traffic": [round(tb[i] / (us[i] * 1e-6) / 1e12, 2) for i in range(n)],
                       "mean_us": round(sum(us) / len(us), 1),
                       "mean_TBps_traffic": round(sum(tb) / (sum(us[:n]) * 1e-6) / 1e12, 2) if n else None}
print(json.dumps(res, indent=1))

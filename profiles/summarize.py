"""Summarises a profiles/collect.sh run into profiles/<tag>/ and profiles/pmc_summary.json.

traffic (HBM bytes per launch) = (2 x FETCH_SIZE + WRITE_SIZE) x 1024: FETCH_SIZE reads half the
bytes of a wide coalesced stream on gfx950 (MI355X_MICROARCH.md §HBM); checked against the
anti-entropy kernel, whose doubled FETCH_SIZE equals its algorithmic read bytes (2 x 4 MB rows
per pair x 16384 pairs = 137.4 GB).
"""
import csv
import collections
import json
import os
import shutil
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = f"gpurun_out/prof_{tag}"
dst = f"profiles/{tag}"
os.makedirs(dst, exist_ok=True)
shutil.copy(f"{src}/trace/run_kernel_stats.csv", f"{dst}/cfg5_kernel_stats.csv")
shutil.copy(f"{src}/bench_trace.json", f"{dst}/cfg5_bench_under_rocprof.json")
agg = collections.defaultdict(dict)
for name, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
    rows = list(csv.DictReader(open(f"{src}/{name}/run_counter_collection.csv")))
    acc = collections.defaultdict(lambda: [0, 0.0])
    for r in rows:
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
        acc[k][0] += 1
        acc[k][1] += float(r["Counter_Value"])
    for k, (n, v) in acc.items():
        agg[k][ctr + "_KB_per_launch"] = v / n
        agg[k]["launches_" + name] = n
cls = {"k_ae": "ae", "k_ae_chunk": "ae", "k_scan": "scan", "k_merge": "merge", "k_merge_seg": "merge", "k_storm": "storm", "k_storm_p2": "storm", "k_send": "send",
       "k_owner": "owner"}
summary = {}
for k, v in agg.items():
    f, w = v.get("FETCH_SIZE_KB_per_launch"), v.get("WRITE_SIZE_KB_per_launch")
    if f is not None and w is not None:
        v["hbm_bytes_per_launch"] = int((2 * f + w) * 1024)
    for kk, c in cls.items():
        if k == kk:
            summary[c] = dict(v)
# the gossip merge class is two launches per round (k_merge_lean, then k_merge for the flagged
# receivers): its traffic per round is their sum (both launch once per round)
if "k_merge_lean" in agg and "merge" in summary:
    m, l = summary["merge"], agg["k_merge_lean"]
    for key in ("FETCH_SIZE_KB_per_launch", "WRITE_SIZE_KB_per_launch", "hbm_bytes_per_launch"):
        if key in m and key in l:
            m[key] = m[key] + l[key]
    m["kernels"] = ["k_merge_lean", "k_merge"]
json.dump(dict(agg), open(f"{dst}/cfg5_pmc.json", "w"), indent=1, sort_keys=True)
pmc = {}
if os.path.exists("profiles/pmc_summary.json"):
    pmc = json.load(open("profiles/pmc_summary.json"))
pmc["cfg5"] = summary
pmc["_note"] = ("hbm_bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE)*1024 from separate rocprofv3 --pmc "
                "passes of bench.py --config cfg5 --steps 100, the same launches as the default bench (profiles/collect.sh)")
json.dump(pmc, open("profiles/pmc_summary.json", "w"), indent=1, sort_keys=True)
print(json.dumps(summary, indent=1))

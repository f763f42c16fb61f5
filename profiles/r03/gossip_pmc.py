"""Per-round HBM traffic of the gossip kernels over one stretch of profiles/gossip_span.py, from
the FETCH_SIZE and WRITE_SIZE passes of profiles/r03/gossip_prof.sh.

Every round launches exactly one k_send and one merge kernel (k_merge_seg), so round r's launches
are the r-th of each in dispatch order; the stretch is rounds [r0, r0 + n). Reports, per kernel,
FETCH_SIZE and WRITE_SIZE per launch (KB from the counters x 1024) and the HBM bytes both ways:
raw (FETCH + WRITE) and with the gfx950 streaming correction (2 x FETCH + WRITE,
MI355X_MICROARCH.md §HBM), which applies to wide coalesced streams, not to the merge's 8-B gathers.

  python profiles/r03/gossip_pmc.py gpurun_out/r03g 51 [n=9]
"""
import csv
import json
import statistics
import sys

src, r0 = sys.argv[1], int(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 9
KERNELS = ("k_send", "k_merge_seg", "k_merge", "k_merge_lean", "k_wake")


def per_kernel(path):
    rows = list(csv.DictReader(open(path)))
    seq = {}
    for r in sorted(rows, key=lambda r: int(r["Dispatch_Id"])):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
        if k in KERNELS:
            seq.setdefault(k, []).append(float(r["Counter_Value"]) * 1024.0)
    return seq


fetch = per_kernel(f"{src}/fetch_{r0}/run_counter_collection.csv")
write = per_kernel(f"{src}/write_{r0}/run_counter_collection.csv")
out = {"rounds": [r0, r0 + n - 1]}
tot_raw = tot_corr = 0.0
for k in ("k_send", "k_merge_seg", "k_merge", "k_merge_lean"):
    if k not in fetch or len(fetch[k]) < r0 + n:
        continue
    f = fetch[k][r0:r0 + n]
    w = write[k][r0:r0 + n]
    fm, wm = statistics.mean(f), statistics.mean(w)
    out[k] = {"FETCH_bytes_per_launch": int(fm), "WRITE_bytes_per_launch": int(wm),
              "hbm_raw": int(fm + wm), "hbm_2fetch": int(2 * fm + wm)}
    tot_raw += fm + wm
    tot_corr += 2 * fm + wm
out["per_round_hbm_raw"] = int(tot_raw)
out["per_round_hbm_2fetch"] = int(tot_corr)
try:  # the span line printed by gossip_span.py under the trace run
    out["span_txt"] = open(f"{src}/span_{r0}.txt").read().strip().splitlines()
except OSError:
    pass
print(json.dumps(out, indent=1))

"""k_send's HBM traffic per launch in launch order (one launch per gossip round of the cfg 5 bench
window), from a profiles/collect.sh run: FETCH_SIZE and WRITE_SIZE rows of the two --pmc passes,
paired by launch index. bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (MI355X_MICROARCH.md gfx950
correction, as profiles/summarize.py).

    python profiles/r05/send_pmc_rounds.py gpurun_out/prof_<tag>
"""
import csv
import json
import sys

src = sys.argv[1]
KN = sys.argv[2] if len(sys.argv) > 2 else "k_send"


def rows(name, ctr):
    out = []
    for r in csv.DictReader(open(f"{src}/{name}/run_counter_collection.csv")):
        if r["Counter_Name"] == ctr and KN in r["Kernel_Name"]:
            out.append((int(r["Dispatch_Id"]), float(r["Counter_Value"]),
                        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    return [x for x in sorted(out)]


f, w = rows("fetch", "FETCH_SIZE"), rows("write", "WRITE_SIZE")
n = min(len(f), len(w))
# the bench runs the window more than once (warmup, timed): keep the last n_round launches
per = [{"i": i, "fetch_MB": round(f[i][1] / 1024, 2), "write_MB": round(w[i][1] / 1024, 2),
        "hbm_MB": round((2 * f[i][1] + w[i][1]) * 1024 / 1e6, 2), "us_fetch_pass": round(f[i][2], 1)}
       for i in range(n)]
for p in per:
    print(json.dumps(p))

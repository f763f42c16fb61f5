"""Summarize profiles/r05/shard_ab.sh: per build and lock model, the shard round (events) and the
kernels of the G = 8 shards' rounds (grid of one shard's hosts) from the kernel trace."""
import glob
import json
import os
import re
import sqlite3
import sys

D = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r05/sab"
rows = []
for js in sorted(glob.glob(os.path.join(D, "*.json"))):
    n = os.path.basename(js)[:-5]
    try:
        r = json.loads(open(js).read().strip().splitlines()[-1])
    except Exception:
        continue
    db = glob.glob(os.path.join(D, n, "*.db"))
    k = {}
    if db:
        c = sqlite3.connect(db[0])
        for name, gx, cnt, avg in c.execute(
                "select name, grid_x, count(*), avg(duration)/1000.0 from kernels where grid_x <= 4096*64 "
                "and name not like '%xplan%' group by name, grid_x order by sum(duration) desc limit 8"):
            k[re.sub(r"\(.*", "", name).replace("void ", "")[:48] + f"@{gx}"] = [cnt, round(avg, 2)]
    rows.append({"build": n, "per_shard_us_med": sorted(r["per_shard_us"])[len(r["per_shard_us"]) // 2],
                 "begin_us_med": sorted(r["per_shard_begin_us"])[len(r["per_shard_begin_us"]) // 2],
                 "end_us_med": sorted(r["per_shard_end_us"])[len(r["per_shard_end_us"]) // 2],
                 "unsharded_us_med": sorted(r["unsharded_us"])[len(r["unsharded_us"]) // 2],
                 "ratio": r["per_shard_over_unsharded_median"], "kernels": k})
for x in rows:
    print(json.dumps(x))

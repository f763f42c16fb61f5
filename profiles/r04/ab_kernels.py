"""A/B of per-kernel device time between engine builds, in ONE process: for each repetition and each
library (alternating, so the variants see the same GPU clocks), a fresh engine of the config runs
`--skip` rounds untimed, then `--rounds` rounds with the engine's launch timers on (gx_enable_timing:
HIP events around each phase's launches). Prints one JSON line per (rep, lib) with the ms and
launches per kernel class, and a summary line with the median ms per kernel class and library.

  python profiles/r04/ab_kernels.py --config cfg3 --skip 100 --rounds 30 --libs a.so b.so [--reps 3]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from sidecar_amd.abi import load_library  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg3")
ap.add_argument("--skip", type=int, default=100)
ap.add_argument("--rounds", type=int, default=30)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--libs", nargs="+", required=True)
ap.add_argument("--lock-model", type=int, default=1)
a = ap.parse_args()
libs = {os.path.basename(p): load_library(p) for p in a.libs}
res = {}
for rep in range(a.reps):
    for ln, lib in libs.items():
        e = bench.make_engine(lib, a.config, 0x5EED, 0, lock_model=a.lock_model)
        e.run_rounds(a.skip)
        e.enable_timing(True)
        t0 = e.timing()
        e.run_rounds(a.rounds)
        t1 = e.timing()
        st = e.stats()
        e.close()
        k = {n: {"ms": round(t1[n]["ms"] - t0[n]["ms"], 4), "launches": t1[n]["launches"] - t0[n]["launches"]}
             for n in t1 if t1[n]["launches"] > t0[n]["launches"]}
        for n, v in k.items():
            res.setdefault(n, {}).setdefault(ln, []).append(v["ms"])
        print(json.dumps({"rep": rep, "lib": ln, "config": a.config, "rounds": [a.skip, a.skip + a.rounds],
                          "kernels": k, "digest": int(st.get("round", 0))}), flush=True)
print(json.dumps({"summary_median_ms": {n: {ln: round(statistics.median(v), 4) for ln, v in d.items()}
                                        for n, d in res.items()}}), flush=True)

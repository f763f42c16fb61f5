"""A/B of the gossip round span in ONE process: for each variant (GX_AB_FLAGS value, read when an
engine is created) and repetition, a fresh cfg 5 engine runs to the stretch, runs the stretch
before it (queue set-up on a new stream), then the measured stretch of 9 gossip-only rounds between
two events on the engine's stream. Variants alternate, so they see the same GPU clocks.

  python profiles/r03/ab_span.py [--flags 0 2048] [--starts 21 51] [--reps 3] [--libs a.so b.so]

--libs: engine builds to compare (each loaded in this process; its own symbols), variant = (lib, flags).
"""
import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from sidecar_amd.abi import load_product  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--flags", type=int, nargs="+", default=[0, 2048])
ap.add_argument("--starts", type=int, nargs="+", default=[21, 51])
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--config", default="cfg5")
ap.add_argument("--libs", nargs="+", default=None)
a = ap.parse_args()
from sidecar_amd.abi import load_library  # noqa: E402
libs = {os.path.basename(p): load_library(p) for p in a.libs} if a.libs else {"libgx.so": load_product()}
res = {}
for st in a.starts:
    for rep in range(a.reps):
        for (ln, lib), fl in [(x, f) for x in libs.items() for f in a.flags]:
            os.environ["GX_AB_FLAGS"] = str(fl)
            e = bench.make_engine(lib, a.config, 0x5EED, 0)
            e.run_rounds(st - 10)
            s = torch.cuda.Stream()
            e.set_stream(s.cuda_stream, False)
            e.run_rounds(10)
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record(s)
            e.run_rounds(9)
            ev1.record(s)
            ev1.synchronize()
            us = 1e3 * ev0.elapsed_time(ev1) / 9
            e.set_stream(None, False)
            e.close()
            res.setdefault(f"start{st}_{ln}_ab{fl}", []).append(round(us, 2))
            print(json.dumps({"start": st, "rep": rep, "lib": ln, "ab": fl, "us_per_round": round(us, 2)}), flush=True)
print(json.dumps({k: {"median": statistics.median(v), "all": v} for k, v in res.items()}))

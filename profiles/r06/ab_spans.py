"""A/B of gossip stretch spans between engine builds in ONE process (bench.gossip_round_span: one
event pair around a stretch of gossip-only rounds), alternating the libraries each repetition so both
see the same GPU clocks. Stretches: cfg 5 lock off dead (21..29) and accepting (51..59), lock on
pipeline-fill (11..19) and full (21..29); one JSON line per measurement, medians at the end.
    python profiles/r06/ab_spans.py --libs a.so b.so [--reps 5] [--config cfg5]"""
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
ap.add_argument("--libs", nargs="+", required=True)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--config", default="cfg5")
a = ap.parse_args()
import torch  # noqa: E402
torch.cuda.init()
libs = [(os.path.basename(p), load_library(p)) for p in a.libs]
cases = [("off_dead", 0, 21), ("off_acc", 0, 51), ("on_fill", 1, 11), ("on_full", 1, 21), ("on_full51", 1, 51)]
res = {}
for rep in range(a.reps):
    for case, lm, start in cases:
        for ln, lib in (libs if rep % 2 == 0 else libs[::-1]):
            us, roof = bench.gossip_round_span(lib, a.config, 0x5EED, 0, start=start, lock_model=lm)
            res.setdefault(case, {}).setdefault(ln, []).append(us)
            print(json.dumps({"rep": rep, "case": case, "lib": ln, "us_per_round": us,
                              "merges_per_round": roof["merges_per_round"], "frac": roof["frac"]}), flush=True)
print(json.dumps({"median_us": {c: {ln: statistics.median(v) for ln, v in d.items()} for c, d in res.items()}}),
      flush=True)

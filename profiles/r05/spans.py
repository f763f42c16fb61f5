"""Gossip stretch spans as bench.py measures them (bench.gossip_round_span: one event pair around 9
gossip-only rounds), for cfg 5 and cfg5_defaults, both stretches, lock on and off. One JSON line each.

    python profiles/r05/spans.py [configs...]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from sidecar_amd.abi import load_product  # noqa: E402


def main():
    import torch
    torch.cuda.init()  # the HIP runtime through torch first (the engine library shares it)
    cfgs = sys.argv[1:] or ["cfg5", "cfg5_defaults"]
    lib = load_product()
    for cfg in cfgs:
        for lm in (1, 0):
            for acc in (False, True):
                start = bench.gossip_stretch_start(cfg, accepting=acc)
                if start is None:
                    continue
                us, roof = bench.gossip_round_span(lib, cfg, 0x5EED, 0, start=start, lock_model=lm)
                print(json.dumps({"config": cfg, "lock_model": lm, "stretch": roof["rounds"], "us_per_round": us,
                                  "merges_per_round": roof["merges_per_round"],
                                  "accepts_per_round": roof["accepts_per_round"],
                                  "line_frac": roof["line_ceiling"]["frac"], "hbm_frac": roof["frac"]}), flush=True)


if __name__ == "__main__":
    main()

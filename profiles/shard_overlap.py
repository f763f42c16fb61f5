"""Overlap of the shard-local push-pull merges with the exchange: G shards of the
cfg 5 schedule in one process on one GPU (LocalShards), timed with and without gx_ae_merge_local.
Run under rocprofv3 --kernel-trace to see the side-stream k_ae_plan dispatches beside the
exchange's kernels; this script reports the push-pull rounds' wall time both ways.

  python profiles/shard_overlap.py [G] [H]
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import sidecar_amd.dist as dist_mod  # noqa: E402
from sidecar_amd.abi import load_product  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 2
H = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
kw = dict(bench.CONFIGS["cfg5"]["p"], n_hosts=H)
lib = load_product()
res = {}
for mode in ("overlap", "serial"):
    orig = dist_mod.Engine.ae_merge_local
    if mode == "serial":  # gx_ae_merge then merges the local pairs too, on the engine's stream
        dist_mod.Engine.ae_merge_local = lambda self: None
    sh = dist_mod.LocalShards(lib, G, device="cuda:0", **kw)
    ae_ms = []
    for r in range(62):
        ae = sh.shards[0].e.is_ae_round()
        torch.cuda.synchronize()
        a = time.perf_counter()
        sh.run_rounds(1)
        torch.cuda.synchronize()
        if ae and r > 0:
            ae_ms.append(1e3 * (time.perf_counter() - a))
    dist_mod.Engine.ae_merge_local = orig
    res[mode] = {"push_pull_round_ms": [round(x, 3) for x in ae_ms], "sum_ms": round(sum(ae_ms), 3)}
    st = sh.stats()
    res[mode]["ae_merges"] = st["ae_merges"]
    for s in sh.shards:
        s.e.close()
print(json.dumps({"G": G, "H": H, **res}))

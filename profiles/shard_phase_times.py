"""Per-phase host time of a sharded round (LocalShards on one GPU, cfg 5 schedule at H = 16384):
where the per-round cost of the exchange layer goes, call by call (each call returns after its
device work). Gossip rounds only (no push-pull, no storm).

  python profiles/shard_phase_times.py [G] [H]
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from sidecar_amd.abi import load_product  # noqa: E402
from sidecar_amd.dist import LocalShards, _ptr  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 8
kw = dict(bench.CONFIGS["cfg5"]["p"])
kw["n_hosts"] = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
sh = LocalShards(load_product(), G, device="cuda:0", **kw)
sh.run_rounds(11)  # past the first push-pull round and the storm
T = {}


def timed(name, fn):
    a = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    T.setdefault(name, []).append(time.perf_counter() - a)
    return r


for _ in range(8):
    if sh.shards[0].e.is_ae_round():
        sh.run_rounds(1)
        continue
    for s in sh.shards:
        timed("round_send", s.e.round_send)
    sizes = [timed("outbox_bytes", s.e.outbox_bytes) for s in sh.shards]
    bufs = []
    for s, sz in zip(sh.shards, sizes):
        buf = torch.empty(int(sz.sum()), dtype=torch.uint8, device="cuda:0")
        timed("outbox_pack", lambda: s.e.outbox_pack(_ptr(buf), buf.numel()))
        bufs.append((buf, sz))
    for dst, s in enumerate(sh.shards):
        parts = [b[int(sz[:dst].sum()):int(sz[:dst].sum()) + int(sz[dst])] for b, sz in bufs]
        x = timed("inbox_concat", lambda: torch.cat(parts))
        timed("inbox_unpack", lambda: s.e.inbox_unpack(_ptr(x), x.numel()))
    for s in sh.shards:
        timed("round_merge", s.e.round_merge)
    for s in sh.shards:
        timed("round_end", s.e.round_end)
out = {k: round(1e6 * float(np.mean(v)), 1) for k, v in T.items()}
# push-pull rounds: whole-round wall time per shard through LocalShards, then its phases
while not sh.shards[0].e.is_ae_round():
    sh.run_rounds(1)
import sidecar_amd.dist as dist_mod  # noqa: E402
orig = {n: getattr(dist_mod.Engine, n) for n in ("ae_bytes", "ae_pack", "ae_merge_local", "ae_delta_bytes",
                                                 "ae_delta_pack", "ae_return_bytes", "ae_return_pack", "ae_merge")}
TA = {}
for n, f in orig.items():
    def wrap(self, *a, _f=f, _n=n):
        t0 = time.perf_counter()
        r = _f(self, *a)
        torch.cuda.synchronize()
        TA.setdefault(_n, []).append(time.perf_counter() - t0)
        return r
    setattr(dist_mod.Engine, n, wrap)
a = time.perf_counter()
sh.run_rounds(1)
torch.cuda.synchronize()
ae_wall = time.perf_counter() - a
for n, f in orig.items():
    setattr(dist_mod.Engine, n, f)
ae = {k: round(1e3 * float(np.sum(v)) / G, 3) for k, v in TA.items()}
print(json.dumps({"G": G, "H": kw["n_hosts"], "us_per_call": out,
                  "us_per_shard_round": round(sum(out.values()), 1),
                  "push_pull_round": {"round": sh.shards[0].e.round - 1, "wall_ms_all_shards": round(1e3 * ae_wall, 2),
                                      "ms_per_shard_by_call": ae}}), flush=True)

"""Sharded rounds on one GPU (LocalShards, cfg 5 schedule at full size): per-round host wall time
beside device time (HIP events on the stream every shard's engine queues on), for the gossip-only
rounds 51..59 and the post-heal push-pull round 60, against the unsharded engine's same rounds.
The shards run one after another on the one GPU, so a sharded round's device time is the sum over
shards; per shard = / G.

  [GX_LIB=<build>] python profiles/r05/shard_ae_g8.py [G=8] [H=32768]   (lock on, the default)
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from sidecar_amd.abi import Engine, default_params, load_library, load_product  # noqa: E402
from sidecar_amd.dist import LocalShards  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 8
H = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
kw = dict(bench.CONFIGS["cfg5"]["p"])
kw["n_hosts"] = H
lib = load_library(os.environ["GX_LIB"]) if os.environ.get("GX_LIB") else load_product()


def timed_round(run, stream):
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    a.record(stream)
    run()
    b.record(stream)
    t1 = time.perf_counter()  # host time to issue the round (returns once queued or waited)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return {"host_ms": round((t1 - t0) * 1e3, 3), "wall_ms": round((t2 - t0) * 1e3, 3),
            "device_ms": round(a.elapsed_time(b), 3)}


out = {"G": G, "H": H}
# unsharded: its own stream, the same rounds
s = torch.cuda.Stream()
e = Engine(default_params(lib, **kw), lib=lib)
e.set_stream(s.cuda_stream, False)
e.run_rounds(51)
out["unsharded"] = {r: timed_round(lambda: e.run_rounds(1), s) for r in range(51, 61)}
e.close()
del e
torch.cuda.synchronize()
sh = LocalShards(lib, G, device="cuda:0", **kw)
sh.run_rounds(51)
cs = torch.cuda.current_stream()
out["sharded"] = {r: timed_round(lambda: sh.run_rounds(1), cs) for r in range(51, 61)}
for k in ("unsharded", "sharded"):
    g = [v for r, v in out[k].items() if r < 60]
    out[k + "_gossip_median"] = {f: sorted(x[f] for x in g)[len(g) // 2] for f in ("host_ms", "wall_ms", "device_ms")}
out["ae_round60_device_per_shard_over_unsharded"] = round(out["sharded"][60]["device_ms"] / G /
                                                            out["unsharded"][60]["device_ms"], 3)
print(json.dumps(out), flush=True)

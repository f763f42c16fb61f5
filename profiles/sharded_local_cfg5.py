"""Full-size check of the sharded protocol on ONE GPU: cfg 5 (32768 x 16) split into G shards
driven in one process (sidecar_amd.dist.LocalShards: the same C-ABI phases and wire formats the
RCCL path moves between GPUs, exchanged here by device copies), against the unsharded engine:
identical counters, host queue digests and per-record min/max words after R rounds (storm, heal,
post-heal push-pull rounds). Reports the exchange volumes per kind. Wall times are NOT a scaling
measurement (the G shards share one GPU and run one after another).

  python profiles/sharded_local_cfg5.py [G] [ROUNDS] [H] [CHECKPOINTS]

CHECKPOINTS (comma-separated rounds, e.g. 51,61,91) adds the counter and min/max comparison after
each of those rounds; ROUNDS is then their maximum. Round 3 ran G = 8 at the full H = 32768 with
checkpoints 51, 61, 91 (profiles/r03/sharded_g8_h32768.json).

At H = 32768 and G = 2 the first push-pull round after the heal ships every cross pair's whole
row (32 GB per shard and direction): more than one GPU can hold twice next to the views, so the
one-GPU check runs the cfg 5 schedule at H = 16384 by default.
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
from sidecar_amd.abi import Engine, default_params, load_product  # noqa: E402
from sidecar_amd.dist import LocalShards  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 2
ROUNDS = int(sys.argv[2]) if len(sys.argv) > 2 else 61
kw = dict(bench.CONFIGS["cfg5"]["p"])
kw["n_hosts"] = int(sys.argv[3]) if len(sys.argv) > 3 else 16384
CHECK = sorted(int(x) for x in sys.argv[4].split(",")) if len(sys.argv) > 4 else []
if CHECK:
    ROUNDS = max(CHECK)
lib = load_product()
R = kw["n_hosts"] * kw["n_services"]


def minmax(engines):
    mn = torch.empty(R, dtype=torch.int64, device="cuda:0")
    mx = torch.empty(R, dtype=torch.int64, device="cuda:0")
    gmn = gmx = None
    for e in engines:
        e.view_minmax(mn.data_ptr(), mx.data_ptr())
        gmn = mn.clone() if gmn is None else torch.minimum(gmn, mn)
        gmx = mx.clone() if gmx is None else torch.maximum(gmx, mx)
    return gmn.cpu().numpy(), gmx.cpu().numpy()


ref_ck, got_ck = {}, {}
t0 = time.perf_counter()
w = Engine(default_params(lib, **kw), lib=lib)
whole_round = []
for r in range(ROUNDS):
    a = time.perf_counter()
    w.run_rounds(1)
    torch.cuda.synchronize()
    whole_round.append(time.perf_counter() - a)
    if r + 1 in CHECK:
        ref_ck[r + 1] = (w.stats(), *minmax([w]))
ref = (w.stats(), w.digests(), *minmax([w]))
t_whole = time.perf_counter() - t0
w.close()
del w
torch.cuda.empty_cache()

t0 = time.perf_counter()
sh = LocalShards(lib, G, device="cuda:0", **kw)
per_round = []
for r in range(ROUNDS):
    a = time.perf_counter()
    sh.run_rounds(1)
    torch.cuda.synchronize()
    per_round.append(time.perf_counter() - a)
    if r + 1 in CHECK:
        got_ck[r + 1] = (sh.stats(), *minmax(sh.engines), dict(sh.wire.as_dict()))
got = (sh.stats(), np.concatenate([e.digests() for e in sh.engines]), *minmax(sh.engines))
t_sharded = time.perf_counter() - t0
ok = {
    "stats": got[0] == ref[0],
    "host_digests": bool(np.array_equal(got[1], ref[1])),
    "record_minmax": bool(np.array_equal(got[2], ref[2]) and np.array_equal(got[3], ref[3])),
}
checkpoints = {}
for r in CHECK:
    a, b = ref_ck[r], got_ck[r]
    checkpoints[r] = {"stats": a[0] == b[0],
                      "record_minmax": bool(np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])),
                      "records_disagreeing": int((a[1] != a[2]).sum()),
                      "wire_bytes_so_far": b[3]}
    ok[f"round_{r}"] = checkpoints[r]["stats"] and checkpoints[r]["record_minmax"]
out = {"config": f"cfg5 schedule at H={kw['n_hosts']}", "G": G, "rounds": ROUNDS, "identical": ok, "checkpoints": checkpoints, "wire_bytes": sh.wire.as_dict(),
       "wall_s": {"unsharded": round(t_whole, 2), "sharded_on_one_gpu": round(t_sharded, 2)},
       "slowest_rounds": sorted(((round(x * 1e3, 1), i) for i, x in enumerate(per_round)), reverse=True)[:6],
       # rounds without push-pull or storm: host-side cost of the phase calls (G shards in turn)
       "median_gossip_round_ms": {"unsharded": round(1e3 * float(np.median([x for i, x in enumerate(whole_round) if i % 10 and i != 5])), 3),
                                  "sharded_on_one_gpu": round(1e3 * float(np.median([x for i, x in enumerate(per_round) if i % 10 and i != 5])), 3)}}
print(json.dumps(out), flush=True)
assert all(ok.values()), ok

"""Membership reconvergence of cfg5fd: the 2-way partition of rounds [0, pe)
with memberlist's detector, then the heal. Prints, every `step` rounds, the member-list entries
that disagree with the truth (gx_fd_converged), the deaths / refutations so far, and the
catalogs' disagreeing records.

  python profiles/fd_reconverge.py [H] [rounds] [partition_end] [step] [oracle|gpu] [gossip_messages]

gossip_messages 15 is Sidecar's default (config/config.go:46); the bench's cfg5fd runs 1.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from sidecar_amd.abi import Engine, default_params, load_product  # noqa: E402

H = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 1500
pe = int(sys.argv[3]) if len(sys.argv) > 3 else 50
step = int(sys.argv[4]) if len(sys.argv) > 4 else 50
if len(sys.argv) > 5 and sys.argv[5] == "oracle":
    from tests.oracle_lib import load_oracle
    lib = load_oracle()
else:
    lib = load_product()
kw = dict(bench.CONFIGS["cfg5fd"]["p"], n_hosts=H, partition_end=pe)
if len(sys.argv) > 6:
    kw["gossip_messages"] = int(sys.argv[6])
e = Engine(default_params(lib, **kw), lib=lib)
p = e.params
print(json.dumps({"H": H, "partition_end": pe, "gossip_messages": kw.get("gossip_messages", 1), "suspicion_rounds": list(p.fd_suspicion_rounds[:p.fd_suspicion_k + 1]),
                  "retransmit_limit": p.fd_retransmit_limit, "gossip_dead_rounds": p.fd_gossip_dead_rounds}),
      flush=True)
t = time.time()
for r in range(step, rounds + 1, step):
    e.run_rounds(step)
    ok, bad = e.fd_converged()
    cat_ok, cat_bad = e.converged()
    st = e.stats()
    print(json.dumps({"round": r, "member_disagree": int(bad), "catalog_disagree": int(cat_bad),
                      "fd_deaths": st["fd_deaths"], "fd_refutes": st["fd_refutes"],
                      "fd_suspicions": st["fd_suspicions"], "wall_s": round(time.time() - t, 1)}), flush=True)

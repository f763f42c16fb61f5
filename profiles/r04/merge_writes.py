"""cfg 5 rounds 51..55 (accepting, after the heal), one round per call: per-round gossip accepts,
retransmits and deferred jobs, for comparing the gossip merge's PMC WRITE_SIZE per launch with its
algorithmic writes (8 B per accepted slot + 16 B per stored retransmit + 8 B per server-time field).

  rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_merge_seg -d ... -- python3 profiles/r04/merge_writes.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from sidecar_amd.abi import load_product  # noqa: E402

lib = load_product()
e = bench.make_engine(lib, "cfg5", 0x5EED, 0)
e.run_rounds(51)
for r in range(51, 56):
    s0 = e.stats()
    e.run_rounds(1)
    s1 = e.stats()
    d = {k: s1[k] - s0[k] for k in ("gossip_merges", "gossip_accepts", "retransmits", "queue_deferred", "changes")
         if k in s1}
    d["stored_retransmits"] = d["retransmits"] - d["queue_deferred"]
    print(json.dumps({"round": r, **d}), flush=True)
e.close()

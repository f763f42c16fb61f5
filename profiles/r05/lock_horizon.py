"""How long the ServicesState lock holds a configuration (gx.h lock_model).

Runs one bench.py configuration on the HIP engine with the lock modelled and prints one JSON line
every --every rounds: hosts locked, records held in pipelines, the deepest broadcast FIFO, records
on which the views disagree, and the lock / queue counters. Usage:
    python profiles/r05/lock_horizon.py cfg5 --rounds 12000 --every 500 [--hosts H] [--lock-model 0]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from sidecar_amd.abi import load_product  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("--rounds", type=int, default=12000)
    ap.add_argument("--every", type=int, default=500)
    ap.add_argument("--hosts", type=int, default=0)
    ap.add_argument("--lock-model", type=int, default=1)
    ap.add_argument("--seed", type=int, default=0x5EED)
    a = ap.parse_args()
    over = dict(lock_model=a.lock_model)
    if a.hosts:
        over["n_hosts"] = a.hosts
    lib = load_product()
    e = bench.make_engine(lib, a.config, a.seed, 0, **over)
    t0 = time.time()
    first_conv = None
    while e.round < a.rounds:
        e.run_rounds(min(a.every, a.rounds - e.round))
        st = e.stats()
        hs = e.hosts()
        rnd = e.round
        ok, n = e.converged()
        if ok and first_conv is None:
            first_conv = rnd
        depth = max(h.fifo_tail - h.fifo_head for h in hs)
        print(json.dumps({
            "round": rnd, "wall_s": round(time.time() - t0, 2), "converged": ok, "disagreeing": n,
            "hosts_locked": sum(h.locked_at(rnd) for h in hs),
            "bs_blocked": sum(h.flags & 1 for h in hs), "bt_blocked": sum((h.flags >> 1) & 1 for h in hs),
            "records_held": sum(h.lock_buffered for h in hs), "max_fifo_depth": depth,
            **{k: st[k] for k in ("gossip_accepts", "ae_accepts", "ae_exchanges", "ae_locked", "lock_buffered",
                                  "lock_drops", "lock_drained", "expire_deferred", "queue_drops",
                                  "queue_deferred", "first_locked_round", "retransmits")}}), flush=True)
    print(json.dumps({"config": a.config, "lock_model": a.lock_model, "rounds": a.rounds,
                      "first_converged_sample": first_conv}), flush=True)
    e.close()


if __name__ == "__main__":
    main()

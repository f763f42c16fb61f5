"""Long faithful runs of a bench configuration: the HIP engine with the lock
modelled and a stored FIFO window large enough that no job is LOST (queue_drops stays 0, so every
round is the reference's unbounded queue), run to catalog agreement or far enough to show the
pattern it repeats. One JSON line every --every rounds: agreement (records some live view disagrees
on), hosts locked, looper states, records held in pipelines, the deepest FIFO, false expiries
(gx.h false_expiries) and the queue counters; a summary line at the end.
    python profiles/r06/converge_long.py cfg2 --rounds 100000 --every 500 --queue-cap 1048576 [--set k=v ...]
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

KEYS = ("gossip_accepts", "ae_accepts", "ae_exchanges", "ae_locked", "lock_buffered", "lock_drops", "lock_drained",
        "expired", "false_expiries", "queue_drops", "queue_deferred", "retransmits", "dequeues", "first_locked_round",
        "first_drop_round", "nil_batches", "send_jobs")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("--rounds", type=int, default=100000)
    ap.add_argument("--every", type=int, default=500)
    ap.add_argument("--queue-cap", type=int, default=0)
    ap.add_argument("--seed", type=int, default=0x5EED)
    ap.add_argument("--set", action="append", default=[], help="param=value overrides")
    ap.add_argument("--stop-on-converge", type=int, default=1)
    a = ap.parse_args()
    over = {}
    if a.queue_cap:
        over["queue_cap"] = a.queue_cap
    for kv in a.set:
        k, v = kv.split("=")
        over[k] = int(v)
    lib = load_product()
    e = bench.make_engine(lib, a.config, a.seed, 0, **over)
    t0 = time.time()
    first_conv, min_bad, samples = None, None, []
    run_s = 0.0
    while e.round < a.rounds:
        t1 = time.time()
        e.run_rounds(min(a.every, a.rounds - e.round))
        st = e.stats()  # waits for the device
        run_s += time.time() - t1
        hs = e.hosts()
        rnd = e.round
        ok, n = e.converged()
        min_bad = n if min_bad is None else min(min_bad, n)
        if ok and first_conv is None:
            first_conv = st["last_change_round"] + 1
        row = {"round": rnd, "wall_s": round(time.time() - t0, 2), "engine_s": round(run_s, 3), "converged": ok,
               "disagreeing": n, "hosts_locked": sum(h.locked_at(rnd) for h in hs),
               "bs_blocked": sum(h.flags & 1 for h in hs), "bt_blocked": sum((h.flags >> 1) & 1 for h in hs),
               "records_held": sum(h.lock_buffered for h in hs),
               "max_fifo_depth": max(h.fifo_tail - h.fifo_head for h in hs),
               "mean_fifo_depth": round(sum(h.fifo_tail - h.fifo_head for h in hs) / len(hs), 1),
               **{k: st[k] for k in KEYS}}
        samples.append(row)
        print(json.dumps(row), flush=True)
        if ok and a.stop_on_converge:
            break
    st = e.stats()
    print(json.dumps({"summary": True, "config": a.config, "overrides": over, "rounds_run": e.round,
                      "rounds_to_converge": first_conv, "min_disagreeing": min_bad,
                      "lossless": st["queue_drops"] == 0, "queue_drops": st["queue_drops"],
                      "false_expiries": st["false_expiries"], "expired": st["expired"],
                      "engine_s": round(run_s, 3)}), flush=True)
    e.close()


if __name__ == "__main__":
    main()

"""Per-round device time of a gossip stretch, split by kernel class (gx_timing, HIP events around
every launch) and unsplit (one event pair per round on the engine's stream).

    python profiles/r05/stretch.py cfg5 --start 21 --rounds 9 [--lock-model 0] [--hosts H]

Prints one JSON line per round and a summary line.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from sidecar_amd.abi import load_product  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("--start", type=int, default=21)
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--lock-model", type=int, default=1)
    ap.add_argument("--hosts", type=int, default=0)
    ap.add_argument("--seed", type=int, default=0x5EED)
    a = ap.parse_args()
    import torch
    over = dict(lock_model=a.lock_model)
    if a.hosts:
        over["n_hosts"] = a.hosts
    lib = load_product()
    e = bench.make_engine(lib, a.config, a.seed, 0, **over)
    e.run_rounds(a.start - 1)
    st = torch.cuda.Stream()
    e.set_stream(st.cuda_stream, False)
    e.run_rounds(1)  # queue set-up on the new stream
    plain = []
    for _ in range(a.rounds):  # unsplit: one event pair per round
        x, y = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0 = e.stats()
        x.record(st)
        e.run_rounds(1)
        y.record(st)
        y.synchronize()
        s1 = e.stats()
        plain.append((e.round - 1, 1e3 * x.elapsed_time(y), {k: s1[k] - s0[k] for k in (
            "gossip_merges", "gossip_accepts", "records_sent", "packets", "lock_buffered", "lock_drops",
            "lock_drained", "dequeues", "retransmits")}))
    e.enable_timing(True)
    split = []
    for _ in range(a.rounds):  # the same number of following rounds, split by class
        t0 = e.timing()
        e.run_rounds(1)
        torch.cuda.synchronize()
        t1 = e.timing()
        split.append({c: round(1e3 * (t1[c]["ms"] - t0[c]["ms"]), 2) for c in t1
                      if t1[c]["launches"] != t0[c]["launches"]})
    for (rnd, us, d), sp in zip(plain, split):
        print(json.dumps({"round": rnd, "us": round(us, 2), **d, "next_round_split_us": sp}), flush=True)
    us = [p[1] for p in plain]
    print(json.dumps({"config": a.config, "lock_model": a.lock_model, "start": a.start, "rounds": a.rounds,
                      "mean_us": round(sum(us) / len(us), 2), "min_us": round(min(us), 2)}), flush=True)
    e.set_stream(None, False)
    e.close()


if __name__ == "__main__":
    main()

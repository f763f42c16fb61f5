"""Device time of one shard's planned gossip round (gx_round_gossip_begin: k_send packing the send
buffer; gx_round_gossip_end: unpack, merge, round end) at G shards of the cfg 5 schedule, against
the unsharded engine's whole round. LocalShards runs the G shards one after another on the one GPU;
HIP events bracket each shard's two calls (the in-process exchange between them, torch.cat copies
standing in for the all-to-all, is not counted). Launch counts from the engine's kernel timing.

    python profiles/r05/shard_round.py [--G 8] [--config cfg5] [--start 51] [--rounds 9] [--lock-model 1]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--G", type=int, default=8)
    ap.add_argument("--config", default="cfg5")
    ap.add_argument("--start", type=int, default=51)
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--lock-model", type=int, default=1)
    ap.add_argument("--lib", default=None, help="another build of the engine (A/B)")
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    import bench
    from sidecar_amd.abi import Engine, default_params, load_library, load_product
    from sidecar_amd.dist import LocalShards, _ptr
    lib = load_library(a.lib) if a.lib else load_product()
    kw = dict(bench.CONFIGS[a.config]["p"], seed=0x5EED, lock_model=a.lock_model)
    stream = torch.cuda.current_stream()
    out = {"config": a.config, "G": a.G, "lock_model": a.lock_model, "rounds": [a.start, a.start + a.rounds - 1]}

    # unsharded: one event pair per round on the engine's stream
    e = Engine(default_params(lib, **kw), lib=lib)
    e.set_stream(stream.cuda_stream, True)
    e.run_rounds(a.start)
    per = []
    for _ in range(a.rounds):
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record(stream)
        e.run_rounds(1)
        t1.record(stream)
        torch.cuda.synchronize()
        per.append(1e3 * t0.elapsed_time(t1))
    out["unsharded_us"] = [round(x, 1) for x in per]
    e.close()
    del e
    torch.cuda.synchronize()

    sh = LocalShards(lib, a.G, device="cuda:0", **kw)
    sh.run_rounds(a.start)
    torch.cuda.synchronize()
    G = a.G
    bufs = sh._planned_bufs()
    send_us, end_us, slots, host_us = [], [], [], []
    for _ in range(a.rounds):
        plan = np.zeros(G * G, dtype=np.uint64)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(2 * G)]
        th = 0.0  # host time to issue the shards' calls (they return once queued)
        for g, (s, b) in enumerate(zip(sh.shards, bufs)):
            ev[g][0].record(stream)
            h0 = time.perf_counter()
            s.e.round_gossip_begin(plan, _ptr(b), b.numel())
            th += time.perf_counter() - h0
            ev[g][1].record(stream)
        m = plan.reshape(G, G)
        slots.append(int(m.sum()) // (16 + 16 * sh.shards[0].e.params.packet_cap))
        ae = False
        for dst, s in enumerate(sh.shards):
            x = torch.cat([bufs[src][int(m[src][:dst].sum()):int(m[src][:dst + 1].sum())] for src in range(G)])
            ev[G + dst][0].record(stream)
            h0 = time.perf_counter()
            ae = s.e.round_gossip_end(_ptr(x), x.numel())
            th += time.perf_counter() - h0
            ev[G + dst][1].record(stream)
        if ae:
            raise SystemExit("a push-pull round in the stretch: pick gossip-only rounds")
        torch.cuda.synchronize()
        host_us.append(1e6 * th / G)
        send_us.append([1e3 * p.elapsed_time(q) for p, q in ev[:G]])
        end_us.append([1e3 * p.elapsed_time(q) for p, q in ev[G:]])
    S, E = np.array(send_us), np.array(end_us)
    per_shard = (S + E).mean(axis=1)  # mean over shards, per round
    out["per_shard_begin_us"] = [round(float(x), 1) for x in S.mean(axis=1)]
    out["per_shard_end_us"] = [round(float(x), 1) for x in E.mean(axis=1)]
    out["per_shard_us"] = [round(float(x), 1) for x in per_shard]
    out["per_shard_over_unsharded_median"] = round(float(np.median(per_shard / np.array(per))), 3)
    out["slots_per_round"] = slots
    out["per_shard_host_issue_us"] = [round(x, 1) for x in host_us]  # the two engine calls (ctypes included)
    for s in sh.shards:
        s.e.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

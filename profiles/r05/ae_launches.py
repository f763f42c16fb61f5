"""Per-launch device time and algorithmic bytes of the push-pull kernel class (gx_timing, HIP
events around its launches) for every push-pull round of a configuration, with the round's accepts
and retransmits: where a push-pull launch falls below the HBM roofline and why.

    python profiles/r05/ae_launches.py cfg2 [--rounds 100] [--lock-model 0]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("--rounds", type=int, default=100)
    ap.add_argument("--lock-model", type=int, default=0)
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    import bench
    from sidecar_amd.abi import load_product
    lib = load_product()
    e = bench.make_engine(lib, a.config, 0x5EED, 0, lock_model=a.lock_model)
    e.enable_timing(True)
    p = e.params
    while e.round < a.rounds:
        r = e.round
        ae = p.ae_period_rounds and r % p.ae_period_rounds == p.ae_phase
        t0, s0 = e.timing(), e.stats()
        e.run_rounds(1)
        torch.cuda.synchronize()
        t1, s1 = e.timing(), e.stats()
        if not ae:
            continue
        ms = t1["ae"]["ms"] - t0["ae"]["ms"]
        b = t1["ae"]["bytes"] - t0["ae"]["bytes"]
        d = {k: s1[k] - s0[k] for k in ("ae_merges", "ae_accepts", "retransmits", "queue_deferred", "ae_exchanges",
                                        "ae_locked")}
        print(json.dumps({"config": a.config, "lock_model": a.lock_model, "round": r, "ms": round(ms, 3),
                          "GB": round(b / 1e9, 3), "TBps": round(b / (ms * 1e9), 3) if ms else None,
                          "frac": round(b / (ms * 1e9) / 8.0, 3) if ms else None, **d}), flush=True)
    e.close()


if __name__ == "__main__":
    main()

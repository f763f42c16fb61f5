"""Where a send team's time goes in the planned GetBroadcasts loop (engine built with
-DGX_SEND_SPLIT, GX_KPROF set): per wave, the lane-0 team's time in the plan, record, header and
ring-write parts summed over its chunks, and its chunk and refill counts; p50 / p90 over waves.

    GX_KPROF=1 python profiles/r05/split.py --lib profiles/r05/lib/libgx_split.so --config cfg5_defaults \\
        --rounds 21 51 [--lock-model 0]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "profiles"))
os.environ.setdefault("GX_KPROF", "1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--config", default="cfg5_defaults")
    ap.add_argument("--rounds", type=int, nargs="+", default=[21, 51])
    ap.add_argument("--lock-model", type=int, default=1)
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    import bench
    import kprof
    from sidecar_amd.abi import load_library
    lib = load_library(a.lib)
    lib.gx_kprof_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
    e = bench.make_engine(lib, a.config, 0x5EED, 0, lock_model=a.lock_model)
    names = ["plan_us", "records_us", "headers_us", "ring_sync_us", "chunks", "refills"]
    for r in a.rounds:
        e.run_rounds(r - e.round)
        e.run_rounds(1)
        wm, _, _, _ = kprof.marks(e, lib)
        wm = wm[wm[:, 0] > 0]
        out = {"config": a.config, "lock_model": a.lock_model, "round": r, "waves": int(wm.shape[0]),
               "kernel_us": round(float(wm[:, 7].max() - wm[:, 0].min()) / 100.0, 2)}
        for i, n in enumerate(names):
            col = wm[:, 1 + i].astype(np.float64) / (100.0 if n.endswith("_us") else 1.0)
            out[n] = {"p50": round(float(np.percentile(col, 50)), 2), "p90": round(float(np.percentile(col, 90)), 2)}
        print(json.dumps(out), flush=True)
    e.close()


if __name__ == "__main__":
    main()

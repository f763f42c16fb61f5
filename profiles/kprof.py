"""k_send phase marks (diagnostics): wall-clock (100 MHz) marks per wave of one k_send launch,
read through gx_kprof_read (engine created with GX_KPROF set). Prints, per mark, the spread over
waves relative to the launch's first start mark: how long the owner ticks, the block barrier, the
plan and the record phase take, and which waves finish last.

  GX_KPROF=1 python profiles/kprof.py [--config cfg5] [--rounds 21 51]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("GX_KPROF", "1")

MERGE_N = 64  # GX_KPROF_MERGE_N: the merge path counters after the per-wave marks
MERGE_NAMES = ["receivers", "seg16", "seg32", "wave", "fallback_wave", "live_records"]
NAMES = ["start", "ticks_done", "barrier", "sends_begin", "send_host", "chunk_planned", "chunk_stored", "sends_done"]


def marks(e, lib):
    n = ctypes.c_uint64(0)
    lib.gx_kprof_read(e.h, None, ctypes.c_uint64(0), ctypes.byref(n))
    buf = (ctypes.c_uint64 * n.value)()
    assert lib.gx_kprof_read(e.h, buf, ctypes.c_uint64(n.value), ctypes.byref(n)) == 0
    a = np.frombuffer(buf, dtype=np.uint64).astype(np.int64)
    return a[:-MERGE_N].reshape(-1, 8), a[-MERGE_N:]


def summarize(m):
    live = m[:, 0] > 0
    m = m[live]
    t0 = m[:, 0].min()
    out = {"waves": int(m.shape[0]), "span_us": round(float(m.max() - t0) / 100.0, 2)}
    for k, name in enumerate(NAMES):
        col = m[:, k]
        col = col[col > 0]
        if not col.size:
            continue
        rel = (col - t0) / 100.0  # us
        out[name] = {"p10": round(float(np.percentile(rel, 10)), 2), "p50": round(float(np.percentile(rel, 50)), 2),
                     "p90": round(float(np.percentile(rel, 90)), 2), "max": round(float(rel.max()), 2)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg5")
    ap.add_argument("--rounds", type=int, nargs="+", default=[21, 51])
    a = ap.parse_args()
    import bench
    from sidecar_amd.abi import load_product
    lib = load_product()
    lib.gx_kprof_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
    e = bench.make_engine(lib, a.config, 0x5EED, 0)
    res = {}
    for r in sorted(a.rounds):
        e.run_rounds(r - e.round)
        _, m0 = marks(e, lib)
        e.run_rounds(1)  # round r: its k_send's marks, its merge's path counts
        wm, m1 = marks(e, lib)
        res[r] = summarize(wm)
        res[r]["merge_paths"] = {k: int(m1[i] - m0[i]) for i, k in enumerate(MERGE_NAMES)}
        print(json.dumps({"config": a.config, "round": r, **res[r]}), flush=True)
    e.close()


if __name__ == "__main__":
    main()

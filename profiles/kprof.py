"""k_send phase marks (diagnostics): wall-clock (100 MHz) marks per wave of one k_send launch,
read through gx_kprof_read (engine created with GX_KPROF set). Prints, per mark, the spread over
waves relative to the launch's first start mark: how long the owner ticks, the block barrier, the
plan and the record phase take, and which waves finish last.

  GX_KPROF=1 python profiles/kprof.py [--config cfg5] [--rounds 21 51] [--ae-rounds 10 20]

With --ae-rounds: the push-pull launch of each such round, per block (start, end, CU): the block
durations, how busy the CUs' slots were over the launch, and the launch's tail (when the CUs ran
out of blocks).
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
MERGE_NAMES = ["receivers", "seg16", "seg32", "wave", "fallback_wave", "live_records", "", "",
               "wave_tile_cyc_loads", "wave_tile_cyc_sort", "wave_tile_cyc_fold", "wave_tile_cyc_rest", "wave_tiles"]
NAMES = ["start", "ticks_done", "barrier", "sends_begin", "send_host", "chunk_planned", "chunk_stored", "sends_done"]


def marks(e, lib):
    n = ctypes.c_uint64(0)
    lib.gx_kprof_read(e.h, None, ctypes.c_uint64(0), ctypes.byref(n))
    buf = (ctypes.c_uint64 * n.value)()
    assert lib.gx_kprof_read(e.h, buf, ctypes.c_uint64(n.value), ctypes.byref(n)) == 0
    a = np.frombuffer(buf, dtype=np.uint64).astype(np.int64)
    ns = a.size - MERGE_N - 3 * e.H  # layout: k_send marks, merge counters, push-pull block marks, scans
    return a[:ns].reshape(-1, 8), a[ns:ns + MERGE_N], a[ns + MERGE_N:ns + MERGE_N + e.H].reshape(-1, 2), \
        a[ns + MERGE_N + e.H:].reshape(-1, 2)


def summarize_ae(m):
    m = m[m[:, 0] > 0]
    start = m[:, 0] & ((1 << 48) - 1)
    cu = m[:, 0] >> 48
    end = m[:, 1]
    t0 = start.min()
    span = float(end.max() - t0)
    dur = (end - start) / 100.0
    out = {"blocks": int(m.shape[0]), "span_us": round(span / 100.0, 1),
           "block_us": {q: round(float(np.percentile(dur, q)), 1) for q in (1, 10, 50, 90, 99)},
           "block_us_max": round(float(dur.max()), 1)}
    cus = np.unique(cu)
    last = np.array([end[cu == c].max() - t0 for c in cus]) / 100.0
    first = np.array([start[cu == c].min() - t0 for c in cus]) / 100.0
    busy = np.array([dur[cu == c].sum() for c in cus])
    nb = np.array([(cu == c).sum() for c in cus])
    out["cus"] = int(cus.size)
    out["blocks_per_cu"] = {"min": int(nb.min()), "max": int(nb.max())}
    out["cu_first_start_us"] = {"p50": round(float(np.median(first)), 1), "max": round(float(first.max()), 1)}
    out["cu_last_end_us"] = {"min": round(float(last.min()), 1), "p50": round(float(np.median(last)), 1),
                             "max": round(float(last.max()), 1)}
    # mean blocks resident per CU over the launch (sum of block durations / span)
    out["resident_blocks_per_cu"] = round(float(busy.mean() / (span / 100.0)), 2)
    return out


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
    ap.add_argument("--rounds", type=int, nargs="*", default=[21, 51])
    ap.add_argument("--ae-rounds", type=int, nargs="*", default=[])
    ap.add_argument("--scan-rounds", type=int, nargs="*", default=[])
    ap.add_argument("--lock-model", type=int, default=1)
    a = ap.parse_args()
    import bench
    from sidecar_amd.abi import load_product
    lib = load_product()
    lib.gx_kprof_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
    e = bench.make_engine(lib, a.config, 0x5EED, 0, lock_model=a.lock_model)
    res = {}
    for r in sorted(set(a.rounds) | set(a.ae_rounds) | set(a.scan_rounds)):
        e.run_rounds(r - e.round)
        _, m0, _, sm0 = marks(e, lib)
        e.run_rounds(1)  # round r: its k_send's marks, its merge's path counts, its push-pull blocks
        wm, m1, am, sm = marks(e, lib)
        if r in a.rounds:
            res[r] = summarize(wm)
            res[r]["merge_paths"] = {k: int(m1[i] - m0[i]) for i, k in enumerate(MERGE_NAMES) if k}
            print(json.dumps({"config": a.config, "lock_model": a.lock_model, "round": r, **res[r]}), flush=True)
        if r in a.ae_rounds:
            print(json.dumps({"config": a.config, "round": r, "push_pull": summarize_ae(am)}), flush=True)
        if r in a.scan_rounds:
            fresh = sm[:, 0] != sm0[:, 0]  # views this round's launch scanned (the region keeps older marks)
            print(json.dumps({"config": a.config, "round": r, "scan": summarize_ae(sm[fresh])}), flush=True)
    e.close()


if __name__ == "__main__":
    main()

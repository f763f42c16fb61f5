"""Full-state JSON codec throughput on one MI355X, plus the CPU oracle beside it.

A LocalState of one view of the cfg 5 catalog (H=32768 hosts x S=16 services, every record
present) is encoded, decoded and merged back (MergeRemoteState) several times. Device time per
direction comes from HIP events on the engine's stream (gx_timing classes encode / decode); the
wall time also includes the PCIe copy of the document (host buffers cross the C-ABI).

  python profiles/codec_bench.py [--hosts 32768 --services 16 --reps 5]
Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from sidecar_amd.abi import INIT_WARM, Engine, default_params, load_product  # noqa: E402
from sidecar_amd.codec import synthetic_names  # noqa: E402

HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hosts", type=int, default=32768)
    ap.add_argument("--services", type=int, default=16)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cpu-hosts", type=int, default=2048)
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    H, S = a.hosts, a.services
    t0 = time.perf_counter()
    names = synthetic_names(H, S, seed=11)
    t_names = time.perf_counter() - t0
    lib = load_product()
    e = Engine(default_params(lib, n_hosts=H, n_services=S, init_mode=INIT_WARM, queue_cap=4096, ae_period_rounds=0),
               lib=lib)
    e.run_rounds(2)
    e.set_names(names)
    e.enable_timing(True)
    doc = e.local_state_json(0)  # warm-up (buffers)
    e.decode_state_json(doc)
    import ctypes as C
    buf = C.create_string_buffer(len(doc) + 4096)  # the caller's buffer, allocated once
    n_out = C.c_uint64()
    tm0 = e.timing()
    t0 = time.perf_counter()
    for _ in range(a.reps):  # the ABI call alone: size + fill in one call (the buffer is large enough)
        assert lib.gx_local_state_json(e.h, 0, buf, len(buf), C.byref(n_out)) == 0
    t_enc = (time.perf_counter() - t0) / a.reps
    assert buf.raw[:n_out.value] == doc
    tm1 = e.timing()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        rc, recs, ds = e.decode_state_json(doc, cap=1)
        assert rc == 0 and ds["records"] == H * S, ds
    t_dec = (time.perf_counter() - t0) / a.reps
    tm2 = e.timing()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        rc, ds = e.merge_remote_state_json(1, doc)
        assert rc == 0
    t_mrg = (time.perf_counter() - t0) / a.reps
    n = len(doc)
    enc_ms = (tm1["encode"]["ms"] - tm0["encode"]["ms"]) / a.reps
    enc_b = (tm1["encode"]["bytes"] - tm0["encode"]["bytes"]) / a.reps
    dec_ms = (tm2["decode"]["ms"] - tm1["decode"]["ms"]) / a.reps
    out = {
        "workload": f"LocalState JSON of one view, {H} hosts x {S} services (all present), synthetic names",
        "doc_bytes": n, "records": H * S, "tokens": ds["tokens"], "names_setup_s": round(t_names, 2),
        "encode": {"device_ms": round(enc_ms, 3), "wall_ms": round(t_enc * 1e3, 3),
                   "doc_GBps": round(n / (enc_ms * 1e6), 1), "records_per_s": H * S / (enc_ms * 1e-3),
                   "algorithmic_bytes": int(enc_b), "achieved_GBps": round(enc_b / (enc_ms * 1e6), 1),
                   "roofline_frac": round(enc_b / (enc_ms * 1e6) / HBM_PEAK_GBS, 4)},
        "decode": {"device_ms": round(dec_ms, 3), "wall_ms": round(t_dec * 1e3, 3),
                   "doc_GBps": round(n / (dec_ms * 1e6), 1), "records_per_s": H * S / (dec_ms * 1e-3)},
        "merge_remote_state_wall_ms": round(t_mrg * 1e3, 3),
    }
    e.close()
    if not a.no_cpu:
        from tests.oracle_lib import load_oracle
        orc = load_oracle()
        hc = min(H, a.cpu_hosts)
        o = Engine(default_params(orc, n_hosts=hc, n_services=S, init_mode=INIT_WARM, queue_cap=4096), lib=orc)
        o.run_rounds(2)
        o.set_names(synthetic_names(hc, S, seed=11))
        t0 = time.perf_counter()
        cdoc = o.local_state_json(0)
        te = time.perf_counter() - t0
        t0 = time.perf_counter()
        rc, _, _ = o.decode_state_json(cdoc, cap=1)
        td = time.perf_counter() - t0
        out["cpu_oracle"] = {"hosts": hc, "doc_bytes": len(cdoc), "encode_MBps": round(len(cdoc) / te / 1e6, 1),
                             "decode_MBps": round(len(cdoc) / td / 1e6, 1), "cores": 1}
        o.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

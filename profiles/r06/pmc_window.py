"""The bench window's own launches, delimited for a rocprofv3 --pmc pass: builds
the bench's engine for a config, runs the warmup rounds, launches one k_view_minmax as a marker, runs
the timed window's rounds, and a second marker. `summarize` then keeps the dispatches between the two
markers and gives each kernel class's HBM bytes per launch, (2 * FETCH_SIZE + WRITE_SIZE) * 1024
(MI355X_MICROARCH.md, the gfx950 FETCH correction for 16-B streams), from the two --pmc passes.
    rocprofv3 --pmc FETCH_SIZE --output-format csv -d D/fetch -o run -- python3 profiles/r06/pmc_window.py run cfg5 5 20
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d D/write -o run -- python3 profiles/r06/pmc_window.py run cfg5 5 20
    python3 profiles/r06/pmc_window.py summarize D cfg5 [out.json]
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

CLASSES = (("k_storm", "storm"), ("k_ae", "ae"), ("k_probe", "send"), ("k_send", "send"), ("k_merge", "merge"), ("k_lock_append", "merge"),
           ("k_owner", "owner"), ("k_scan", "scan"), ("k_bt_finish", "scan"), ("k_wake", "wake"))
PRIMARY = {"merge": "k_merge_seg", "scan": "k_scan_split", "send": "k_send"}


def run(cfg, warmup, steps):
    import torch
    import bench
    from sidecar_amd.abi import load_product
    lib = load_product()
    e = bench.make_engine(lib, cfg, 0x5EED, 0)
    R = e.H * e.S
    mn = torch.empty(R, dtype=torch.int64, device="cuda:0")
    mx = torch.empty(R, dtype=torch.int64, device="cuda:0")
    e.run_rounds(warmup)
    e.view_minmax(mn.data_ptr(), mx.data_ptr())  # marker
    e.run_rounds(steps)
    e.view_minmax(mn.data_ptr(), mx.data_ptr())  # marker
    torch.cuda.synchronize()
    e.close()


def window_rows(path, counter):
    rows = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"]),
                         (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    rows.sort()
    marks = [i for i, x in enumerate(rows) if "k_view_minmax" in x[1]]
    assert len(marks) >= 2, "markers not found"
    return rows[marks[-2] + 1:marks[-1]]


def find_csv(d):
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                return os.path.join(root, f)
    raise FileNotFoundError(d)


def summarize(d, cfg, out=None):
    f = window_rows(find_csv(os.path.join(d, "fetch")), "FETCH_SIZE")
    w = window_rows(find_csv(os.path.join(d, "write")), "WRITE_SIZE")
    assert [x[1] for x in f] == [x[1] for x in w], "the two passes launched different kernels"
    res = {}
    for (_, name, fk, us), (_, _, wk, _) in zip(f, w):
        cls = next((c for p, c in CLASSES if p in name), "other")
        r = res.setdefault(cls, {"launches": 0, "FETCH_SIZE_KB": 0.0, "WRITE_SIZE_KB": 0.0, "us": 0.0})
        r["launches"] += 1
        r["FETCH_SIZE_KB"] += fk
        r["WRITE_SIZE_KB"] += wk
        r["us"] += us
    # a class's "launch" is one engine-timer scope (bench.py's per-launch averages): count the scope's
    # primary kernel when the class has one in the window (k_lock_append runs ahead of k_merge_seg,
    # k_scan_join after k_scan_split), else every kernel of the class
    names = [x[1] for x in f]
    for cls, prim in PRIMARY.items():
        if cls in res:
            n = sum(1 for x in names if prim in x and next((c for p, c in CLASSES if p in x), "other") == cls)
            if n:
                res[cls]["launches"] = n
    for r in res.values():
        r["hbm_bytes_per_launch"] = int((2 * r["FETCH_SIZE_KB"] + r["WRITE_SIZE_KB"]) * 1024 / r["launches"])
        r["us_per_launch_pmc_pass"] = round(r["us"] / r["launches"], 2)
    doc = {}
    if out and os.path.exists(out):
        doc = json.load(open(out))
    doc["_note"] = ("per kernel class, the launches of the bench window only (between two k_view_minmax "
                    "markers, profiles/r06/pmc_window.py): HBM bytes per launch = (2 * FETCH_SIZE + "
                    "WRITE_SIZE) * 1024, from separate --pmc passes")
    doc[cfg] = res
    s = json.dumps(doc, indent=1)
    if out:
        open(out, "w").write(s)
    print(s)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
    else:
        summarize(sys.argv[2], sys.argv[3], sys.argv[4] if len(sys.argv) > 4 else None)

"""Summarize bench lines: python profiles/r05/summarize.py gpurun_out/r05/<tag>/bench_*.json"""
import json
import sys


def rf(r):
    return None if not r else (r["kernel"], r["frac"], r.get("us_per_launch"))


for f in sys.argv[1:]:
    d = json.load(open(f))
    g = d.get("gossip") or {}
    lo = g.get("lock_off") or {}
    print(f.split("/")[-1], "value %.3g" % d["value"], "ms/step %.3f" % d["ms_per_step"], "roof", rf(d["roofline"]))
    print("   gossip span lock-on", g.get("round_span_us"), g.get("round_span_us_accepting"),
          "| lock-off", lo.get("round_span_us"), lo.get("round_span_us_accepting"))
    for k in ("roofline", "roofline_accepting"):
        for src, name in ((g, "on"), (lo, "off")):
            r = src.get(k)
            if r:
                print("     %s %s frac %s lines %s line_frac %s merges %s" % (
                    name, k, r["frac"], r["line_ceiling"]["view_lines_per_round"], r["line_ceiling"]["frac"],
                    r["merges_per_round"]))
    ro = d.get("roofline_lock_off") or {}
    print("   lock-off rooflines", {k: rf(v) for k, v in ro.items() if k != "note"})
    cv = d.get("converge") or {}
    print("   converge", cv.get("rounds_to_converge"), (cv.get("lock") or {}).get("hosts_locked_at_end"),
          "lock-off", (d.get("converge_lock_off") or {}).get("rounds_to_converge"),
          "ref", (d.get("converge_ref_cadence") or {}).get("rounds_to_converge"))
    print("   kernels", {k: (v["ms"], v["launches"], v["GBps"]) for k, v in d["kernels"].items()})
    if d.get("kernels_lock_off"):
        print("   kernels_off", {k: (v["ms"], v["launches"], v["GBps"]) for k, v in d["kernels_lock_off"].items()})

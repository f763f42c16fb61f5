"""Per-dispatch durations of the push-pull and storm kernels from a rocprofv3 kernel trace
(usage: python profiles/trace_dispatch.py <run_kernel_trace.csv>)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Kernel_Name"]
    if any(k in n for k in ("k_ae", "k_storm", "k_json", "k_codec")):
        ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        print(f"{n.split('(')[0]:40s} {ms:9.3f} ms  vgpr={r['VGPR_Count']} lds={r['LDS_Block_Size']}")

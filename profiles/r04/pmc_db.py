"""Per-dispatch counter sums from a rocprofv3 SQLite output (rocpd tables): one line per dispatch
with the kernel name, duration and each counter summed over its instances.

  python profiles/r04/pmc_db.py gpurun_out/r04/ae_pmc/eng/pmc_results.db [name-substring]
"""
import json
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
sub = sys.argv[2] if len(sys.argv) > 2 else ""
q = """select d.id, s.kernel_name, d.end - d.start, p.name, sum(e.value)
       from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on s.id = d.kernel_id
       join rocpd_pmc_event e on e.event_id = d.event_id join rocpd_info_pmc p on p.id = e.pmc_id
       group by d.id, p.name order by d.id"""
rows = {}
for did, kn, dur, pn, v in db.execute(q):
    if sub not in kn:
        continue
    r = rows.setdefault(did, {"kernel": kn[:60], "ns": dur})
    r[pn] = v
for r in rows.values():
    print(json.dumps(r))

"""Debug: the worklist merge against the oracle on one scenario, round by round (views that differ)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from sidecar_amd.abi import Engine, default_params, load_product  # noqa: E402
from tests.oracle_lib import load_oracle  # noqa: E402
from tests.test_gpu_parity import SCENARIOS  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "cfg1_churn_aged"
gx, orc = load_product(), load_oracle()
kw = SCENARIOS[name]
g = Engine(default_params(gx, **kw), lib=gx)
o = Engine(default_params(orc, **kw), lib=orc)
for r in range(3):
    g.run_rounds(1)
    o.run_rounds(1)
    vg, vo = g.read_views(), o.read_views()
    bad = np.argwhere(vg != vo)
    sg, so = g.stats(), o.stats()
    print(f"round {r}: stats diff {[(k, sg[k], so[k]) for k in sg if sg[k] != so[k]]}")
    views = sorted(set(int(x) for x in bad[:, 0])) if len(bad) else []
    print(f"  views differing: {views}")
    for v in views[:4]:
        cols = np.nonzero(vg[v] != vo[v])[0]
        print(f"   view {v}: keys {cols.tolist()[:20]} gpu {[hex(int(x)) for x in vg[v][cols[:4]]]} orc {[hex(int(x)) for x in vo[v][cols[:4]]]}")

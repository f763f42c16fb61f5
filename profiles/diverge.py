"""First round where the HIP engine and the oracle differ on a golden case (stats, views)."""
import sys
import numpy as np
sys.path.insert(0, ".")
from sidecar_amd.abi import Engine, default_params, load_product
from tests.oracle_lib import load_oracle
from tests.golden.make_golden import CASES

name = sys.argv[1] if len(sys.argv) > 1 else "cfg1_churn_500"
kw, rounds = CASES[name]
g = Engine(default_params(load_product(), **kw), lib=load_product())
o = Engine(default_params(load_oracle(), **kw), lib=load_oracle())
for r in range(rounds):
    g.run_rounds(1)
    o.run_rounds(1)
    sg, so = g.stats(), o.stats()
    vg, vo = g.read_views(), o.read_views()
    if sg != so or not np.array_equal(vg, vo) or not np.array_equal(g.digests(), o.digests()):
        print("round", r, {k: (sg[k], so[k]) for k in sg if sg[k] != so.get(k)})
        d = np.argwhere(vg != vo)
        print("view diffs", len(d), d[:10].tolist())
        for v, k in d[:5]:
            print(v, k, hex(int(vg[v, k])), hex(int(vo[v, k])))
        break
else:
    print("no divergence in", rounds, "rounds")

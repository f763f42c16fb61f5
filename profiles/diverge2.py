"""Round 120 of cfg1_churn_500 slot by slot: the pre-round words of the diverging slots."""
import sys
import numpy as np
sys.path.insert(0, ".")
from sidecar_amd.abi import Engine, default_params, load_product
from tests.oracle_lib import load_oracle
from tests.golden.make_golden import CASES

kw, rounds = CASES["cfg1_churn_500"]
g = Engine(default_params(load_product(), **kw), lib=load_product())
o = Engine(default_params(load_oracle(), **kw), lib=load_oracle())
g.run_rounds(120)
o.run_rounds(120)
vg, vo = g.read_views(), o.read_views()
print("pre equal", np.array_equal(vg, vo), "round", g.stats()["round"])
for v in (18, 37):
    print("pre", v, hex(int(vg[v, 327])), hex(int(vo[v, 327])))
g.run_rounds(1)
o.run_rounds(1)
vg, vo = g.read_views(), o.read_views()
for v in (18, 37):
    print("post", v, hex(int(vg[v, 327])), hex(int(vo[v, 327])))
print("all views holding key 327, post oracle:", sorted(set(hex(int(x)) for x in vo[:, 327])))
print("all views holding key 327, post gpu:", sorted(set(hex(int(x)) for x in vg[:, 327])))

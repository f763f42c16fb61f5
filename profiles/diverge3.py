"""cfg1_churn_500: does either engine's state at round 121 depend on how rounds are split into calls?"""
import sys
import numpy as np
sys.path.insert(0, ".")
from sidecar_amd.abi import Engine, default_params, load_product
from tests.oracle_lib import load_oracle
from tests.golden.make_golden import CASES

kw, rounds = CASES["cfg1_churn_500"]
N = int(sys.argv[1]) if len(sys.argv) > 1 else 121
res = {}
for name, lib in (("gpu", load_product()), ("oracle", load_oracle())):
    a = Engine(default_params(lib, **kw), lib=lib)
    for _ in range(N):
        a.run_rounds(1)
    b = Engine(default_params(lib, **kw), lib=lib)
    b.run_rounds(N)
    res[name] = (a.read_views(), b.read_views(), a.stats(), b.stats())
    print(name, "per-round == one call:", np.array_equal(res[name][0], res[name][1]), res[name][2] == res[name][3])
print("gpu/oracle per-round equal:", np.array_equal(res["gpu"][0], res["oracle"][0]))
print("gpu/oracle one-call equal:", np.array_equal(res["gpu"][1], res["oracle"][1]))

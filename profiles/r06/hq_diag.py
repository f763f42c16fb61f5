"""First round where the HIP engine and the oracle diverge on an fd_handoff_shared scenario
(diagnostic for tests/test_gpu_fd_handoff.py)."""
import sys
sys.path.insert(0, '.')
from sidecar_amd.abi import Engine, default_params
from tests.oracle_lib import load_oracle
from sidecar_amd.abi import load_product
from tests.test_gpu_fd_handoff import BASE, SCENARIOS
from tests.parity import snapshot
from tests.fd_parity import fd_snapshot

name = sys.argv[1]
kw = dict(BASE); kw.update(SCENARIOS[name])
gl, ol = load_product(), load_oracle()
g = Engine(default_params(gl, **kw), lib=gl)
o = Engine(default_params(ol, **kw), lib=ol)
for r in range(200):
    g.run_rounds(1); o.run_rounds(1)
    sg, so = g.stats(), o.stats()
    fg, fo = fd_snapshot(g), fd_snapshot(o)
    hg, ho = snapshot(g)["hosts"], snapshot(o)["hosts"]
    if sg != so or fg["hosts"] != fo["hosts"] or hg != ho or fg["members"] != fo["members"]:
        print("diverge at round", g.round)
        print({k: (sg[k], so[k]) for k in sg if sg[k] != so[k]})
        for v in range(len(hg)):
            if hg[v] != ho[v]:
                print("host", v, hg[v], ho[v])
        gh, oh = g.fd_hosts(), o.fd_hosts()
        for v in range(len(gh)):
            if bytes(gh[v]) != bytes(oh[v]):
                print("fdhost", v, gh[v].hq_len, oh[v].hq_len, gh[v].q_len, oh[v].q_len)
        for v in range(len(fg["members"])):
            if fg["members"][v] != fo["members"][v]:
                print("members of", v, "differ")
                break
        break
else:
    print("no divergence in 200 rounds")

"""Timeline of one record's versions on the CPU oracle: for record `rec`, every
round in which some view's word for it changes, with the view, the new (Updated, status), how it got
there (owner restamp, gossip packet, push-pull round, or the view's own alive-lifespan expiry) and the
owner's own word. Sidecar's cadences by default (GossipMessages 15, per-node push-pull every 20 s).
    python profiles/r06/trace_record.py H S rounds rec [json overrides]"""
import json
import sys

import numpy as np

sys.path.insert(0, ".")
from sidecar_amd.abi import Engine, default_params  # noqa: E402
from tests.oracle_lib import load_oracle  # noqa: E402

ST = {0: "ALIVE", 1: "TOMB", 2: "UNHEALTHY", 3: "UNKNOWN", 4: "DRAINING", 7: "-"}


def main():
    H, S, rounds, rec = (int(x) for x in sys.argv[1:5])
    over = json.loads(sys.argv[5]) if len(sys.argv) > 5 else {}
    kw = dict(n_hosts=H, n_services=S, fanout=3, packet_cap=32, queue_cap=1 << 16, list_slots=64, init_mode=2,
              ae_period_rounds=100, push_pull_mode=1, gossip_messages=15)
    kw.update(over)
    lib = load_oracle()
    p = default_params(lib, **kw)
    p.seed = 7
    e = Engine(p, lib=lib)
    o = rec // S
    sec = 10**9
    prev = e.read_views().reshape(H, H * S)[:, rec].copy()
    t_base = None
    ae_prev = 0
    for n in range(rounds):
        e.run_rounds(1)
        st = e.stats()
        ae = st["ae_exchanges"] != ae_prev
        ae_prev = st["ae_exchanges"]
        cur = e.read_views().reshape(H, H * S)[:, rec].copy()
        for v in np.nonzero(cur != prev)[0].tolist():
            w0, w1 = int(prev[v]), int(cur[v])
            t1 = e.word_time(w1) if (w1 & 7) != 7 else None
            if t_base is None:
                t_base = e.now(0)
            how = ("owner restamp" if v == o else
                   "expiry (own scan)" if (w1 & 7) == 1 and (w0 & 7) != 1 and (w1 >> 3) == (w0 >> 3) + sec else
                   "push-pull" if ae else "gossip")
            ow = int(cur[o])
            print(f"round {n:5d} t={(e.now(n) - t_base) / sec:7.1f}s view {v:3d} <- "
                  f"{ST[w1 & 7]:9s} Updated t={(t1 - t_base) / sec if t1 is not None else float('nan'):8.3f}s"
                  f"  [{how}]  owner holds t={(e.word_time(ow) - t_base) / sec:8.3f}s")
        prev = cur


if __name__ == "__main__":
    main()

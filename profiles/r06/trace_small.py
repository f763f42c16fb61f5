"""Per-record trace of the small-cluster flapping, on the CPU oracle.

Runs H hosts x S services from a warm catalog under Sidecar's cadences and, every round, diffs all
views to find each alive-lifespan expiry (services_state.go:655-679: a non-tombstone at Updated T
becomes TOMBSTONE at T + 1 s) of a record whose owner is live. For each such false expiry it records
whether the owner had a newer version at that moment (the refresh did not reach the view in time) or
not (the owner itself had not restamped for 80 s), and for every refresh version the rounds until
k views hold it, split by the path that delivered it (gossip packet vs push-pull).

usage: python profiles/r06/trace_small.py H S rounds [lock] [gm] [pp_period] [probe]"""
import json
import sys

import numpy as np

sys.path.insert(0, ".")
from sidecar_amd.abi import Engine, default_params  # noqa: E402
from tests.oracle_lib import load_oracle  # noqa: E402


def main():
    H, S, rounds = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    lock = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    gm = int(sys.argv[5]) if len(sys.argv) > 5 else 15
    pp = int(sys.argv[6]) if len(sys.argv) > 6 else 100
    extra = json.loads(sys.argv[7]) if len(sys.argv) > 7 else {}
    lib = load_oracle()
    p = default_params(lib, n_hosts=H, n_services=S, fanout=3, packet_cap=32, queue_cap=1 << 16,
                       list_slots=64, init_mode=2, ae_period_rounds=pp, push_pull_mode=1 if pp else 0,
                       gossip_messages=gm, lock_model=lock, **extra)
    p.seed = 7
    e = Engine(p, lib=lib)
    R = H * S
    sec = 1_000_000_000
    prev = e.read_views().reshape(H, R).copy()
    own = np.array([prev[r // S, r] for r in range(R)], dtype=np.uint64)
    birth = {}  # (r, ts) -> round the owner's own view got it
    reach = {}  # (r, ts) -> rounds at which each view got it
    false_exp = []
    st_prev = e.stats()
    ae_rounds = set()
    blocked_bs = 0
    maxdepth = 0
    for n in range(rounds):
        e.run_rounds(1)
        st = e.stats()
        if st["ae_exchanges"] != st_prev["ae_exchanges"]:
            ae_rounds.add(n)
        st_prev = st
        cur = e.read_views().reshape(H, R)
        hs = e.hosts()
        blocked_bs += sum(1 for h in hs if h.flags & 1)
        maxdepth = max(maxdepth, max(h.fifo_tail - h.fifo_head for h in hs))
        ch = np.nonzero(cur != prev)
        for v, r in zip(ch[0].tolist(), ch[1].tolist()):
            o, w0, w1 = r // S, int(prev[v, r]), int(cur[v, r])
            t0, s0, t1, s1 = w0 >> 3, w0 & 7, w1 >> 3, w1 & 7
            if v == o:
                birth.setdefault((r, t1), n)
            if s0 not in (1, 7) and s1 == 1 and t1 == t0 + sec:  # alive-lifespan expiry
                ow = int(cur[o, r])
                false_exp.append(dict(round=n, view=v, rec=r, age_s=(e.now(n) - e.word_time(w0)) / sec,
                                      owner_newer=(ow >> 3) > t0 and (ow & 7) != 1,
                                      owner_age_s=(e.now(n) - e.word_time(ow)) / sec))
            elif v != o and s1 != 1 and t1 > t0:
                reach.setdefault((r, t1), []).append((n, n in ae_rounds))
        prev = cur.copy()
    # spread of each refresh version born after round 0 on the owner
    spread = []
    for (r, t), b in birth.items():
        got = reach.get((r, t), [])
        if b < 10 or b > rounds - 600:
            continue
        via_pp = sum(1 for (_, a) in got if a)
        first = {}
        for x, a in got:
            first.setdefault(x, a)
        spread.append(dict(rec=r, born=b, views=len(got) + 1, via_pp=via_pp,
                           all_at=(max(x for x, _ in got) - b) if len(got) + 1 >= H else None,
                           gossip_views_first_100=sum(1 for (x, a) in got if not a and x - b < 100)))
    n_exp = len(false_exp)
    out = dict(H=H, S=S, rounds=rounds, lock=lock, gm=gm, pp=pp, extra=extra, false_expiries=n_exp,
               false_expiries_owner_had_newer=sum(1 for f in false_exp if f["owner_newer"]),
               false_expiries_owner_stale=sum(1 for f in false_exp if not f["owner_newer"]),
               mean_owner_age_at_expiry_s=float(np.mean([f["owner_age_s"] for f in false_exp])) if n_exp else None,
               versions=len(spread),
               versions_reaching_all=sum(1 for s in spread if s["all_at"] is not None),
               views_reached_p50=float(np.median([s["views"] for s in spread])) if spread else None,
               gossip_views_in_100_rounds_p50=float(np.median([s["gossip_views_first_100"] for s in spread]))
               if spread else None,
               all_reached_rounds_p50=float(np.median([s["all_at"] for s in spread if s["all_at"] is not None]))
               if any(s["all_at"] is not None for s in spread) else None,
               bs_blocked_host_rounds=blocked_bs, max_fifo_depth=int(maxdepth),
               stats={k: st[k] for k in ("gossip_accepts", "ae_accepts", "retransmits", "dequeues", "expired",
                                         "ae_exchanges", "ae_locked", "lock_drops", "false_expiries")})
    print(json.dumps(out))


if __name__ == "__main__":
    main()

"""Generates the committed golden round-model fixtures (tests/golden/*.npz) from the CPU oracle.

Inputs are the seeded cfg-1 schedules below (64 hosts x 8 services, fanout 3); outputs are the
final views, per-host queue digests, host bookkeeping and counters after `rounds` rounds.
The oracle is pinned to the reference by tests/kat_cases.py; these fixtures pin the oracle (and
the HIP engine) against regressions of the round model itself.

    python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from sidecar_amd.abi import Engine, default_params  # noqa: E402
from tests.oracle_lib import load_oracle  # noqa: E402

CASES = {
    "cfg1_empty_300": (dict(n_hosts=64, n_services=8, fanout=3, init_mode=0, queue_cap=4096), 300),
    "cfg1_own_ae10_200": (dict(n_hosts=64, n_services=8, fanout=3, init_mode=1, ae_period_rounds=10,
                               queue_cap=4096), 200),
    "cfg1_storm_150": (dict(n_hosts=64, n_services=8, fanout=3, init_mode=2, ae_period_rounds=10,
                            partition_start=0, partition_end=50, storm_round=5, queue_cap=4096), 150),
    "cfg1_churn_500": (dict(n_hosts=64, n_services=8, fanout=3, init_mode=1, churn_ppm=50000,
                            aged_ppm=50000, ae_period_rounds=20, queue_cap=256, list_slots=4), 500),
}


def run(lib, kw, rounds):
    e = Engine(default_params(lib, **kw), lib=lib)
    e.run_rounds(rounds)
    hosts = np.array([[getattr(h, f) & 0xFFFFFFFFFFFFFFFF for f, _ in h._fields_] for h in e.hosts()],
                     dtype=np.uint64)
    return dict(views=e.read_views(), digests=e.digests(), hosts=hosts,
                stats=json.dumps(e.stats(), sort_keys=True))


def main():
    lib = load_oracle()
    for name, (kw, rounds) in CASES.items():
        out = run(lib, kw, rounds)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), params=json.dumps(kw), rounds=rounds, **out)
        print(name, json.loads(out["stats"])["gossip_merges"])


if __name__ == "__main__":
    main()

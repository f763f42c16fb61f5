"""How often the lock model's one known restatement gap matters (VERDICT r05 Missing 3): push-pull
exchanges the model fails (gx_stats.ae_locked) although every locked side held only
BroadcastServices' read lock with no writer waiting, which Go's RWMutex would let run
(gx_oracle_ro_runnable, an oracle-only diagnostic). One JSON line per schedule.
    python profiles/r06/ro_runnable.py"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from sidecar_amd.abi import Engine, default_params  # noqa: E402
from tests.oracle_lib import load_oracle  # noqa: E402

CASES = [  # (name, config, host override, rounds, extra)
    ("cfg1_defaults_64", None, 64, 3000, dict(n_services=8, init_mode=2, ae_period_rounds=100, push_pull_mode=1,
                                             gossip_messages=15, queue_cap=1 << 16, list_slots=64)),
    ("cfg1_defaults_64_stagger", None, 64, 3000, dict(n_services=8, init_mode=2, ae_period_rounds=100,
                                                     push_pull_mode=1, push_pull_stagger=1, gossip_messages=15,
                                                     queue_cap=1 << 16, list_slots=64)),
    ("cfg5_h2048", "cfg5", 2048, 600, {}),
    ("cfg2_h1024", "cfg2", 1024, 2000, {}),
    ("cfg3_h1024", "cfg3", 1024, 600, {}),
    ("cfg4_h512", "cfg4", 512, 1000, {}),
    ("cfg5_defaults_h1024", "cfg5_defaults", 1024, 1000, {}),
]


def main():
    lib = load_oracle(omp=True)
    lib.gx_oracle_ro_runnable.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
    for name, cfg, h, rounds, extra in CASES:
        kw = dict(bench.CONFIGS[cfg]["p"]) if cfg else {}
        kw.update(extra)
        kw["n_hosts"] = h
        e = Engine(default_params(lib, **kw), lib=lib)
        e.run_rounds(rounds)
        n = C.c_uint64(0)
        lib.gx_oracle_ro_runnable(e.h, C.byref(n))
        st = e.stats()
        print(json.dumps({"case": name, "rounds": rounds, "ae_exchanges": st["ae_exchanges"],
                          "ae_locked": st["ae_locked"], "ro_runnable": n.value}), flush=True)
        e.close()


if __name__ == "__main__":
    main()

"""The multi-threaded oracle build (oracle/liboracle_gx_omp.so, bench.py's cpu_baseline) must equal
the serial checker bit for bit: views, host bookkeeping, queue digests, server times and counters.
Its per-host phase loops run on OpenMP threads with private counters (oracle/gx_oracle.c
for_hosts), so any cross-host write in a phase would show up here as a difference."""
import pytest

from sidecar_amd.abi import INIT_WARM, Engine, default_params
from tests.oracle_lib import load_oracle
from tests.parity import assert_same
from tests.test_gpu_parity import SCENARIOS

CASES = dict(SCENARIOS)
# a scaled cfg 5: partition + ExpireServer storm + heal, push-pull every 10 rounds
CASES["cfg5_h512"] = dict(n_hosts=512, n_services=16, init_mode=INIT_WARM, partition_start=0,
                          partition_end=50, storm_round=5, ae_period_rounds=10, queue_cap=20480)


@pytest.mark.parametrize("name", sorted(CASES))
def test_omp_oracle_equals_serial(oracle_lib, name):
    omp = load_oracle(omp=True)
    kw = CASES[name]
    a = Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    b = Engine(default_params(omp, **kw), lib=omp)
    rounds = 120 if name == "cfg5_h512" else 250
    done = 0
    for chunk in (1, 9, 40, 70, 130):
        n = min(chunk, rounds - done)
        if n <= 0:
            break
        a.run_rounds(n)
        b.run_rounds(n)
        done += n
        assert_same(a, b, f"{name} round {a.round}")
    a.close()
    b.close()

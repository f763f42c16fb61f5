"""The ServicesState lock held by a blocked looper (gx.h lock_model) on the HIP
engine: the known-answer cases of tests/lock_cases.py, each compared bit for bit with the oracle,
and round-model scenarios with the lock on and off (cfg 1 and cfg 5's schedule at H = 2048)."""
import pytest

from sidecar_amd.abi import INIT_OWN, INIT_WARM, Engine, default_params
from tests import lock_cases
from tests.oracle_lib import load_oracle
from tests.parity import assert_same

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", sorted(lock_cases.CASES))
def test_lock_case_gpu(oracle_lib, gx_lib, name):
    g = lock_cases.CASES[name](gx_lib)
    o = lock_cases.CASES[name](oracle_lib)
    assert_same(g, o, name)


SCENARIOS = {
    # cfg 1 with the storm: every host blocks behind the storm's ExpireServer jobs
    "cfg1_storm_lock": dict(n_hosts=64, n_services=8, init_mode=INIT_WARM, ae_period_rounds=10, partition_start=0,
                            partition_end=50, storm_round=5, queue_cap=4096),
    "cfg1_storm_lock_off": dict(n_hosts=64, n_services=8, init_mode=INIT_WARM, ae_period_rounds=10, partition_start=0,
                                partition_end=50, storm_round=5, queue_cap=4096, lock_model=0),
    # small pipelines overflow (memberlist's handoff queue drops)
    "cfg1_storm_pipeline8": dict(n_hosts=64, n_services=8, init_mode=INIT_WARM, ae_period_rounds=10, partition_start=0,
                                 partition_end=30, storm_round=3, queue_cap=4096, lock_buffer=8),
    # the storm lands on hosts already blocked (short looper intervals, deep queues): deferred ExpireServer
    "storm_on_locked_hosts": dict(n_hosts=96, n_services=4, init_mode=INIT_OWN, ae_period_rounds=5,
                                  alive_interval_rounds=2, tombstone_interval_rounds=3, churn_ppm=100000,
                                  storm_round=12, queue_cap=2048),
    "gm4_lock": dict(n_hosts=96, n_services=4, init_mode=INIT_WARM, gossip_messages=4, ae_period_rounds=10,
                     partition_start=0, partition_end=20, storm_round=4, queue_cap=4096),
    "pp_initiate_lock": dict(n_hosts=64, n_services=8, init_mode=INIT_WARM, push_pull_mode=1, ae_period_rounds=5,
                             storm_round=3, partition_start=0, partition_end=15, queue_cap=4096),
    "bytes_lock": dict(n_hosts=64, n_services=8, init_mode=INIT_WARM, limit_bytes=1398, overhead_bytes=3,
                       ae_period_rounds=10, storm_round=4, partition_start=0, partition_end=20, queue_cap=4096),
    "fd_depart_lock": dict(n_hosts=64, n_services=8, init_mode=INIT_WARM, fd_enable=1, depart_round=3,
                           depart_ppm=100000, ae_period_rounds=10, queue_cap=4096),
}


@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_lock_round_model_parity(oracle_lib, gx_lib, name):
    kw = SCENARIOS[name]
    g = Engine(default_params(gx_lib, **kw), lib=gx_lib)
    o = Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    for chunk in (1, 4, 10, 35, 50, 150):
        g.run_rounds(chunk)
        o.run_rounds(chunk)
        assert_same(g, o, f"{name} round {g.round}")
    st = g.stats()
    assert st["first_locked_round"] >= 0
    if kw.get("lock_model", 1):
        assert st["locked_merges"] == 0 and st["lock_buffered"] + st["ae_locked"] > 0, st
    else:
        assert st["locked_merges"] > 0 and st["lock_buffered"] == 0, st


def test_cfg5_schedule_h2048_lock(gx_lib):
    """cfg 5's schedule (partition, storm at round 5, heal at 50, push-pull every 10 rounds) at
    H = 2048 with the lock modelled, against the OpenMP oracle through round 151."""
    omp = load_oracle(omp=True)
    kw = dict(n_hosts=2048, n_services=16, init_mode=INIT_WARM, ae_period_rounds=10, partition_start=0,
              partition_end=50, storm_round=5, queue_cap=8192)
    g = Engine(default_params(gx_lib, **kw), lib=gx_lib)
    o = Engine(default_params(omp, **kw), lib=omp)
    for chunk in (6, 45, 50, 50):
        g.run_rounds(chunk)
        o.run_rounds(chunk)
        assert_same(g, o, f"cfg5@2048 lock round {g.round}")
    st = g.stats()
    assert st["queue_drops"] == 0 and st["locked_merges"] == 0 and st["ae_locked"] > 0

"""The ServicesState lock held by a blocked looper (gx.h lock_model) on the CPU oracle: the
known-answer cases of tests/lock_cases.py, and lock_model = 0 against 1 on a storm schedule."""
import pytest

from sidecar_amd.abi import INIT_OWN, INIT_WARM, LOCK_DEFER_MERGE, Engine, GxError, default_params
from tests import lock_cases


@pytest.mark.parametrize("name", sorted(lock_cases.CASES))
def test_lock_case(oracle_lib, name):
    lock_cases.CASES[name](oracle_lib)


def test_lock_off_counts_what_lock_on_holds_back(oracle_lib):
    """cfg 5's schedule at H = 128: with the lock off, every host blocked behind the storm's
    ExpireServer jobs keeps merging (locked_merges > 0); with it on, no merge happens on a locked
    host, push-pull exchanges with a locked side do not run and the buffered records drain later."""
    kw = dict(n_hosts=128, n_services=8, init_mode=INIT_WARM, ae_period_rounds=10, partition_start=0,
              partition_end=50, storm_round=5, queue_cap=4096)
    off = Engine(default_params(oracle_lib, lock_model=0, **kw), lib=oracle_lib)
    on = Engine(default_params(oracle_lib, lock_model=1, **kw), lib=oracle_lib)
    off.run_rounds(120)
    on.run_rounds(120)
    a, b = off.stats(), on.stats()
    assert a["locked_merges"] > 0 and a["ae_locked"] == 0 and a["lock_buffered"] == 0
    assert b["locked_merges"] == 0 and b["ae_locked"] > 0 and b["lock_buffered"] > 0
    assert a["first_locked_round"] >= 0 and b["first_locked_round"] >= 0
    assert b["ae_merges"] < a["ae_merges"]


@pytest.mark.parametrize("bad", [dict(lock_readers=2), dict(lock_readers=1, lock_model=0),
                                 dict(lock_readers=1, n_shards=2, shard_id=0), dict(lock_readers=1, lock_defer_slots=4097)])
def test_lock_readers_rejects_unsupported_modes(oracle_lib, bad):
    with pytest.raises(GxError):
        Engine(default_params(oracle_lib, n_hosts=16, n_services=4, **bad), lib=oracle_lib)


@pytest.mark.parametrize("mode", [0, 1])
def test_lock_readers_accounting(oracle_lib, mode):
    """gx.h lock_readers on a small cluster whose locked hosts' pipelines often stay empty: some
    exchanges with a read-locked side run (ae_deferred), every pair of a push-pull round still either
    runs or fails (ae_exchanges + ae_locked), a merge kept in a pool slot that another host holds is
    lost (lock_defer_slots 1), and at most one merge waits per host (its DEFER bit)."""
    kw = dict(n_hosts=32, n_services=4, fanout=1, packet_cap=1, init_mode=INIT_OWN, churn_ppm=100000,
              alive_interval_rounds=2, tombstone_interval_rounds=7, ae_period_rounds=1, queue_cap=4096,
              storm_round=5, push_pull_mode=mode)
    off = Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    on = Engine(default_params(oracle_lib, lock_readers=1, **kw), lib=oracle_lib)
    one = Engine(default_params(oracle_lib, lock_readers=1, lock_defer_slots=1, **kw), lib=oracle_lib)
    for e in (off, on, one):
        e.run_rounds(300)
    a, b, c = off.stats(), on.stats(), one.stats()
    assert a["ae_deferred"] == 0 and b["ae_deferred"] > 0 and b["ae_defer_lost"] == 0 and c["ae_defer_lost"] > 0
    for st in (a, b, c):
        assert st["ae_exchanges"] + st["ae_locked"] == a["ae_exchanges"] + a["ae_locked"]
        assert st["locked_merges"] == 0
    assert b["ae_exchanges"] > a["ae_exchanges"]
    for e, st in ((on, b), (one, c)):
        waiting = sum(1 for h in e.hosts() if h.lock & LOCK_DEFER_MERGE)
        assert waiting <= min(st["ae_deferred"], 64 if e is on else 1)

"""The ServicesState lock held by a blocked looper (gx.h lock_model) on the CPU oracle: the
known-answer cases of tests/lock_cases.py, and lock_model = 0 against 1 on a storm schedule."""
import pytest

from sidecar_amd.abi import INIT_WARM, Engine, default_params
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

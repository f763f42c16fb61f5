"""Parity at BASELINE.json's full configuration sizes.

* cfg 2 (4096 x 16, fanout 3, cap 32, push-pull every 10 rounds) against the CPU oracle, bit
  for bit, for 25 rounds (two push-pull rounds) — the oracle finishes this in seconds.
* cfg 3 (16384 x 16, 5 % churn, aged records) against the oracle for 12 rounds, no push-pull.
* cfg 5 (32768 x 16, partition + storm + push-pull) through size-independent properties: every
  record sent is merged exactly once, the run is deterministic (two engines, same seed, identical
  counters, host digests and per-record min/max), and the catalog converges.
"""
import numpy as np
import pytest
import torch

from sidecar_amd.abi import Engine, default_params
from tests.parity import assert_same

pytestmark = pytest.mark.gpu

CFG2 = dict(n_hosts=4096, n_services=16, fanout=3, packet_cap=32, queue_cap=4096, init_mode=1,
            ae_period_rounds=10)
CFG3 = dict(n_hosts=16384, n_services=16, fanout=3, queue_cap=1024, init_mode=2, churn_ppm=50000,
            aged_ppm=50000)
CFG5 = dict(n_hosts=32768, n_services=16, fanout=3, packet_cap=32, pending_cap=100, queue_cap=20480,
            list_slots=16, init_mode=2, partition_start=0, partition_end=50, storm_round=5,
            ae_period_rounds=10)


def test_cfg2_full_parity(gx_lib, oracle_lib):
    g = Engine(default_params(gx_lib, **CFG2), lib=gx_lib)
    o = Engine(default_params(oracle_lib, **CFG2), lib=oracle_lib)
    for chunk in (4, 7, 14):
        g.run_rounds(chunk)
        o.run_rounds(chunk)
        assert_same(g, o, f"cfg2 round {g.round}")


def test_cfg3_full_parity(gx_lib, oracle_lib):
    g = Engine(default_params(gx_lib, **CFG3), lib=gx_lib)
    o = Engine(default_params(oracle_lib, **CFG3), lib=oracle_lib)
    g.run_rounds(12)
    o.run_rounds(12)
    assert g.stats() == o.stats()
    assert np.array_equal(g.digests(), o.digests())
    for lo in range(0, 16384, 4096):  # views in 4096-row slabs (8.6 GB each)
        assert np.array_equal(g.read_views(lo, lo + 4096), o.read_views(lo, lo + 4096)), lo


def _minmax(e):
    R = e.H * e.S
    mn = torch.empty(R, dtype=torch.int64, device="cuda:0")
    mx = torch.empty(R, dtype=torch.int64, device="cuda:0")
    e.view_minmax(mn.data_ptr(), mx.data_ptr())
    return mn.cpu().numpy(), mx.cpu().numpy()


def test_cfg5_properties_and_determinism(gx_lib):
    runs = []
    for _ in range(2):
        e = Engine(default_params(gx_lib, **CFG5), lib=gx_lib)
        e.run_rounds(31)  # storm at 5, push-pull at 0,10,20,30
        st = e.stats()
        assert st["gossip_merges"] == st["records_sent"]  # every packet record merged once
        assert st["expire_server"] == 32768 * 16384  # every host expired the other half
        assert st["ae_exchanges"] == 4 * (32768 // 2)
        assert st["ae_merges"] <= st["ae_slots"]
        runs.append((st, e.digests(), *_minmax(e)))
        e.close()
        del e
    (s0, d0, mn0, mx0), (s1, d1, mn1, mx1) = runs
    assert s0 == s1
    assert np.array_equal(d0, d1) and np.array_equal(mn0, mn1) and np.array_equal(mx0, mx1)
    e = Engine(default_params(gx_lib, **CFG5), lib=gx_lib)
    e.run_rounds(100)
    ok, bad = e.converged()
    assert ok, bad
    mn, mx = _minmax(e)
    assert np.array_equal(mn, mx)

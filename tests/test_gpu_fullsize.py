"""Parity at BASELINE.json's full configuration sizes.

* cfg 2 (4096 x 16, fanout 3, cap 32, push-pull every 10 rounds) against the CPU oracle, bit
  for bit, for 25 rounds (two push-pull rounds) — the oracle finishes this in seconds.
* cfg 3 (16384 x 16, 5 % churn, aged records) against the oracle for 12 rounds, no push-pull.
* cfg 5 (32768 x 16, partition + storm + push-pull) through size-independent properties: every
  record sent is merged once, held in a locked host's pipeline or dropped there, every ExpireServer
  call of the storm runs or waits for its host's lock, every push-pull pair runs or finds a side
  locked, the run is deterministic (two engines, same seed, identical counters, host digests and
  per-record min/max), and without the lock (lock_model = 0) the catalog converges.
* cfg 5 itself (H = 32768) against the OpenMP oracle, bit for bit, for rounds 0..101 (storm, heal
  and every post-heal push-pull round), GossipMessages 15 on the cfg 5 schedule at H = 32768, and
  cfg 3 as the bench runs it (push-pull) for 51 rounds. The ServicesState lock is modelled
  (gx.h lock_model, the default) in all of them.
"""
import sys

import numpy as np
import pytest
import torch

import bench
from sidecar_amd.abi import Engine, default_params
from tests.parity import assert_same

pytestmark = pytest.mark.gpu

CFG2 = dict(bench.CONFIGS["cfg2"]["p"])  # the bench's configurations
CFG3 = dict(n_hosts=16384, n_services=16, fanout=3, queue_cap=1024, init_mode=2, churn_ppm=50000,
            aged_ppm=50000)
CFG5 = dict(bench.CONFIGS["cfg5"]["p"])


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
    H = 32768
    runs = []
    for _ in range(2):
        e = Engine(default_params(gx_lib, **CFG5), lib=gx_lib)
        e.run_rounds(6)  # the storm at round 5: every host expires the other half, now or once unlocked
        st = e.stats()
        assert st["expire_server"] + st["expire_deferred"] == H * (H // 2)
        e.run_rounds(25)  # push-pull at 0, 10, 20, 30
        st = e.stats()
        held = sum(h.lock_buffered for h in e.hosts())
        # every packet record: merged (on arrival or drained from a pipeline), held, or dropped
        assert st["gossip_merges"] + held + st["lock_drops"] == st["records_sent"]
        assert st["lock_buffered"] == st["lock_drained"] + held
        assert st["ae_exchanges"] + st["ae_locked"] == 4 * (H // 2)
        assert st["ae_merges"] <= st["ae_slots"] and st["locked_merges"] == 0
        runs.append((st, e.digests(), *_minmax(e)))
        e.close()
        del e
    (s0, d0, mn0, mx0), (s1, d1, mn1, mx1) = runs
    assert s0 == s1
    assert np.array_equal(d0, d1) and np.array_equal(mn0, mn1) and np.array_equal(mx0, mx1)
    # without the lock (lock_model = 0, merges run on locked hosts) the catalog agrees by round 100
    e = Engine(default_params(gx_lib, **dict(CFG5, lock_model=0)), lib=gx_lib)
    e.run_rounds(100)
    ok, bad = e.converged()
    assert ok, bad
    mn, mx = _minmax(e)
    assert np.array_equal(mn, mx)
    assert e.stats()["locked_merges"] > 0


CFG4 = dict(bench.CONFIGS["cfg4"]["p"])
FD_DEPART = dict(n_hosts=16384, n_services=16, fanout=3, queue_cap=4096, init_mode=2, ae_period_rounds=10,
                 fd_enable=1, depart_round=5, depart_ppm=20000)


def _omp_oracle():
    # the OpenMP build of the oracle: bit-identical to the serial checker (tests/test_oracle_omp.py,
    # tests/test_fd_cpu.py), fast enough for the full-size push-pull rounds
    from tests.oracle_lib import load_oracle
    return load_oracle(omp=True)


def _slabs_equal(g, o, step):
    for lo in range(0, g.H, step):
        hi = min(g.H, lo + step)
        assert np.array_equal(g.read_views(lo, hi), o.read_views(lo, hi)), lo


def test_cfg4_full_parity(gx_lib):
    """cfg 4 (8192 x 64, push-pull full-state merges every 10 rounds) against the oracle, bit for
    bit, over two push-pull rounds (rounds 0 and 10): 8.6e9 record-merges."""
    orc = _omp_oracle()
    g = Engine(default_params(gx_lib, **CFG4), lib=gx_lib)
    o = Engine(default_params(orc, **CFG4), lib=orc)
    g.run_rounds(11)
    o.run_rounds(11)
    assert g.stats() == o.stats()
    st = g.stats()
    assert st["ae_exchanges"] + st["ae_locked"] == 2 * (8192 // 2)
    assert np.array_equal(g.digests(), o.digests())
    _slabs_equal(g, o, 1024)


def test_fd_depart_full_parity(gx_lib):
    """The failure detector at cfg 3's size (16384 x 16, 2% of hosts crash at round 5) against the
    oracle, bit for bit, for 25 rounds: catalog views, counters, queue digests, every host's probe
    and queue state, and the member lists of 64 hosts."""
    from tests.fd_parity import assert_same_fd  # noqa: F401  (full tables are 8.6 GB: sampled below)
    orc = _omp_oracle()
    g = Engine(default_params(gx_lib, **FD_DEPART), lib=gx_lib)
    o = Engine(default_params(orc, **FD_DEPART), lib=orc)
    g.run_rounds(25)
    o.run_rounds(25)
    sg, so = g.stats(), o.stats()
    assert sg == so
    assert sg["fd_probe_failures"] > 0 and sg["fd_suspicions"] > 0
    assert np.array_equal(g.digests(), o.digests())
    assert [bytes(h) for h in g.fd_hosts()] == [bytes(h) for h in o.fd_hosts()]
    for v in np.linspace(0, 16383, 64).astype(int):
        assert g.fd_members(int(v)) == o.fd_members(int(v)), v
    _slabs_equal(g, o, 4096)


def _minmax_any(e):
    """Per-record (min, max) slot word over every view: device buffers for the HIP engine, host
    buffers for the oracle (gx_view_minmax, XOR 2^63 form)."""
    if e.backend.startswith("hip"):
        return _minmax(e)
    R = e.H * e.S
    mn, mx = np.empty(R, dtype=np.int64), np.empty(R, dtype=np.int64)
    e.view_minmax(mn.ctypes.data, mx.ctypes.data)
    return mn, mx


def _rows_equal(g, o, views, what):
    for v in views:
        v = int(v)
        assert np.array_equal(g.read_views(v, v + 1), o.read_views(v, v + 1)), f"{what}: view {v}"
        assert np.array_equal(g.server_times(v), o.server_times(v)), f"{what}: server times of view {v}"




def _progress(msg):  # past pytest's capture: a long test shows it is alive
    print(msg, file=sys.__stderr__, flush=True)


@pytest.mark.parametrize("lock_readers", [0, 1])
def test_cfg5_full_h32768_parity(gx_lib, lock_readers):
    """The bench's own workload, cfg 5 at its full size (H = 32768, S = 16: 2-way partition for rounds
    [0, 50), ExpireServer storm of the other half at round 5, heal, push-pull every 10 rounds,
    queue_cap 20480), against the OpenMP oracle for rounds 0..101: the storm (5.4e8 ExpireServer
    calls), every partitioned and every post-heal push-pull round (1.9e11 record-merges). At each
    checkpoint: every counter, every host's queue digest and bookkeeping, the per-record min and max
    word over all 32768 views, 24 full rows with their server times, and state.LastChanged of every
    view. The oracle holds 155 GB of host memory; if the box cannot give it, gx_create fails with
    GX_ENOMEM and so does this test (no skip). With lock_readers = 1 (gx.h: an exchange whose locked
    sides hold only BroadcastServices' read lock with no writer waiting runs) the lock words carry
    the write-lock bits and the few exchanges that qualify (2 of 10240 at H = 2048 on the oracle,
    all before the storm's jobs fill the pipelines) merge one way now and one way later, or lose the
    waiting half when the host's pool slot is taken (both engines count it in ae_defer_lost)."""
    orc = _omp_oracle()
    H = 32768
    _progress("cfg5@32768: creating the HIP engine and the OpenMP oracle")
    kw = dict(CFG5, lock_readers=lock_readers)
    g = Engine(default_params(gx_lib, **kw), lib=gx_lib)
    o = Engine(default_params(orc, **kw), lib=orc)
    sample = np.linspace(0, H - 1, 24).astype(int)
    for stop in (6, 51, 101):
        n = stop - g.round
        g.run_rounds(n)
        _progress(f"cfg5@32768: HIP engine at round {g.round}; oracle running")
        o.run_rounds(n)
        what = f"cfg5@32768 round {g.round}"
        _progress(what)
        sg, so = g.stats(), o.stats()
        assert sg == so, what
        assert np.array_equal(g.digests(), o.digests()), what
        assert [bytes(h) for h in g.hosts()] == [bytes(h) for h in o.hosts()], what
        mg, xg = _minmax_any(g)
        mo, xo = _minmax_any(o)
        assert np.array_equal(mg, mo) and np.array_equal(xg, xo), what
        _rows_equal(g, o, sample, what)
        assert np.array_equal(g.last_changed(), o.last_changed()), what
    st = g.stats()
    assert st["expire_server"] <= H * (H // 2) <= st["expire_server"] + st["expire_deferred"]
    assert st["ae_exchanges"] + st["ae_locked"] == 11 * (H // 2)
    # every host blocks behind the storm's 16384 jobs (3 GetBroadcasts calls per round) from round 7:
    # the gossip of these rounds waits in the pipelines (nothing drains before round 101); what
    # gossip ran before carried records every view already held (warm start, storm on every host)
    assert st["gossip_accepts"] == 0 and st["lock_buffered"] > 0 and st["lock_drops"] > 0
    assert st["lock_drained"] == 0 and st["first_locked_round"] == 7
    assert st["queue_drops"] == 0 and st["first_drop_round"] == -1  # faithful to the reference's queues
    _progress(f"cfg5@32768 lock_readers {lock_readers}: ae_deferred {st['ae_deferred']} ae_defer_lost {st['ae_defer_lost']}")
    assert lock_readers or st["ae_deferred"] + st["ae_defer_lost"] == 0


CFG3_BENCH = dict(bench.CONFIGS["cfg3"]["p"])


def test_cfg3_bench_schedule_51_rounds(gx_lib):
    """cfg 3 as bench.py runs it (push-pull every 10 rounds, 5 % churn, 5 % of
    records aged U[0, 100 s]) against the OpenMP oracle for 51 rounds: five expiry scans per view
    (alive-lifespan expiry of the aged records) and six push-pull rounds, every view compared."""
    orc = _omp_oracle()
    g = Engine(default_params(gx_lib, **CFG3_BENCH), lib=gx_lib)
    o = Engine(default_params(orc, **CFG3_BENCH), lib=orc)
    for stop in (21, 51):
        n = stop - g.round
        g.run_rounds(n)
        o.run_rounds(n)
        print(f"cfg3 round {g.round}", flush=True)  # progress (long test)
        assert g.stats() == o.stats(), g.round
        assert np.array_equal(g.digests(), o.digests()), g.round
    st = g.stats()
    assert st["expired"] > 0 and st["ae_exchanges"] + st["ae_locked"] == 6 * 8192 and st["churn_events"] > 0
    _slabs_equal(g, o, 4096)
    _rows_equal(g, o, np.linspace(0, 16383, 16).astype(int), "cfg3 round 51")


def test_cfg5_gossip_messages15_h32768_parity(gx_lib):
    """Sidecar's own GossipMessages default (15, config/config.go:46, main.go:257-259) on the cfg 5
    schedule at its full size (H = 32768) against the OpenMP oracle for 61 rounds (storm, heal, the
    first post-heal push-pull), with the ServicesState lock modelled: up to 45 packets per host and
    round, receivers with many packets. The stored FIFO window (24576 jobs per host) holds every job
    of these rounds (asserted: no LOST dequeue). The oracle holds about 170 GB of host memory; if the
    box cannot give it, gx_create fails with GX_ENOMEM and so does this test (no skip)."""
    orc = _omp_oracle()
    H = 32768
    kw = dict(CFG5, gossip_messages=15, queue_cap=24576)
    _progress("cfg5 GM15 @32768: creating the HIP engine and the OpenMP oracle")
    g = Engine(default_params(gx_lib, **kw), lib=gx_lib)
    o = Engine(default_params(orc, **kw), lib=orc)
    sample = np.linspace(0, H - 1, 16).astype(int)
    for stop in (6, 31, 52, 61):
        n = stop - g.round
        g.run_rounds(n)
        _progress(f"cfg5 GM15 @32768: HIP engine at round {g.round}; oracle running")
        o.run_rounds(n)
        what = f"cfg5 GM15 @32768 round {g.round}"
        _progress(what)
        assert g.stats() == o.stats(), what
        assert np.array_equal(g.digests(), o.digests()), what
        mg, xg = _minmax_any(g)
        mo, xo = _minmax_any(o)
        assert np.array_equal(mg, mo) and np.array_equal(xg, xo), what
        _rows_equal(g, o, sample, what)
    st = g.stats()
    assert st["packets"] > 3 * H * 10 and st["queue_drops"] == 0 and st["locked_merges"] == 0

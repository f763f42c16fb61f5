"""memberlist failure detection on the CPU oracle: the restated memberlist unit
tests (tests/fd_cases.py), round-model invariants of the detector scenarios, and agreement of the
OpenMP build with the serial checker."""
import pytest

from sidecar_amd.abi import GX_EINVAL, INIT_OWN, M_ALIVE, M_DEAD, TOMBSTONE, Engine, GxError, default_params
from tests import fd_cases
from tests.fd_parity import assert_same_fd
from tests.oracle_lib import load_oracle
from tests.parity import assert_same


@pytest.mark.parametrize("case", fd_cases.ALL, ids=lambda f: f.__name__)
def test_oracle_fd_kat(oracle_lib, case):
    case(oracle_lib)


def run(lib, name, **over):
    kw, rounds = fd_cases.SCENARIOS[name]
    e = Engine(default_params(lib, **dict(kw, **over)), lib=lib)
    e.run_rounds(rounds)
    return e


def test_departures_detected_and_expired(oracle_lib):
    """Crashed hosts are declared dead by every live host (NotifyLeave once each), their records
    are tombstoned in every live view, nobody live is declared dead, and the live catalogs agree."""
    e = run(oracle_lib, "depart10")
    H, S = e.H, e.S
    gone = [v for v, h in enumerate(e.fd_hosts()) if h.departed]
    live = [v for v in range(H) if v not in gone]
    assert 0 < len(gone) < H // 4
    for v in live:
        for m in range(H):
            assert e.fd_member(v, m).state == (M_DEAD if m in gone else M_ALIVE), (v, m)
        for o in gone:
            assert all(e.slot(v, o, s)[1] == TOMBSTONE for s in range(S))
    st = e.stats()
    assert st["fd_deaths"] == len(live) * len(gone)
    assert st["lost_packets"] > 0 and st["fd_refutes"] == 0
    assert e.converged() == (True, 0) and e.fd_converged() == (True, 0)


def test_no_failures_no_suspicions(oracle_lib):
    """Without departures or partitions every probe is acked and nothing is suspected."""
    kw = dict(fd_cases.SCENARIOS["depart10"][0])
    kw.update(depart_round=-1, depart_ppm=0)
    e = Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    e.run_rounds(100)
    st = e.stats()
    assert st["fd_probes"] > 0 and st["fd_probe_failures"] == st["fd_suspicions"] == st["fd_deaths"] == 0
    assert st["lost_packets"] == 0 and st["fd_msgs_sent"] == 0


def test_long_partition_splits_membership(oracle_lib):
    """A partition longer than the suspicion timeout: each half declares the other dead and
    ExpireServer()s its records; after GossipToTheDeadTime nobody gossips to the dead, so the halves
    stay apart after the network heals (memberlist has no automatic rejoin)."""
    e = run(oracle_lib, "partition_long")
    H, half = e.H, e.H // 2
    for v in range(H):
        for m in range(H):
            other = (v < half) != (m < half)
            assert e.fd_member(v, m).state == (M_DEAD if other else M_ALIVE)
    st = e.stats()
    assert st["fd_deaths"] == 2 * half * (H - half)
    assert not e.converged()[0]
    assert e.fd_converged() == (False, H)  # every node is dead to the other half


def test_short_partition_recovers(oracle_lib):
    """A partition about as long as the confirmed suspicion timeout: hosts declared dead refute
    (alive with a higher incarnation) once the network heals, and every member is alive again.
    With the catalog's ServicesState lock modelled (gx.h lock_model) most push-pull exchanges
    after the heal fail (the deaths' ExpireServer jobs keep the loopers blocked behind deep
    broadcast queues), so the membership is checked with the lock off, and with it on the
    refutations still spread to all but a few member entries."""
    e = run(oracle_lib, "partition_heal", lock_model=0)
    st = e.stats()
    assert st["fd_refutes"] > 0 and st["fd_alive_updates"] > 0
    assert all(e.fd_member(v, m).state == M_ALIVE for v in range(e.H) for m in range(e.H))
    e = run(oracle_lib, "partition_heal")
    st = e.stats()
    assert st["fd_refutes"] > 0 and st["ae_locked"] > 0 and st["expire_deferred"] > 0
    assert sum(e.fd_member(v, m).state != M_ALIVE for v in range(e.H) for m in range(e.H)) <= 8


def test_fd_param_checks(oracle_lib):
    base = dict(n_hosts=64, n_services=8, fd_enable=1)
    for bad in (dict(n_hosts=65535), dict(fd_msg_cap=0), dict(fd_msg_cap=65),
                dict(fd_suspicion_k=3), dict(fd_retransmit_limit=0), dict(fd_retransmit_limit=33)):
        kw = dict(base, **bad)
        with pytest.raises(GxError, match=f"rc={GX_EINVAL}"):
            Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    e = Engine(default_params(oracle_lib, n_hosts=16), lib=oracle_lib)  # fd off: no fd state
    with pytest.raises(GxError):
        e.fd_members(0)


@pytest.mark.parametrize("name", sorted(fd_cases.SCENARIOS))
def test_fd_omp_equals_serial(oracle_lib, name):
    kw, rounds = fd_cases.SCENARIOS[name]
    omp = load_oracle(omp=True)
    a = Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    b = Engine(default_params(omp, **kw), lib=omp)
    for n in (7, 60, rounds - 67):
        a.run_rounds(n)
        b.run_rounds(n)
        assert_same(a, b, f"{name} round {a.round}")
        if kw.get("fd_enable"):
            assert_same_fd(a, b, f"{name} round {a.round}")


@pytest.mark.parametrize("bad", [dict(fd_handoff_shared=2), dict(fd_handoff_shared=1, fd_enable=0),
                                 dict(fd_handoff_shared=1, lock_model=0),
                                 dict(fd_handoff_shared=1, n_shards=2, shard_id=0)])
def test_fd_handoff_rejects_unsupported_modes(oracle_lib, bad):
    kw = dict(n_hosts=16, n_services=4, fd_enable=1)
    kw.update(bad)
    with pytest.raises(GxError):
        Engine(default_params(oracle_lib, **kw), lib=oracle_lib)


def test_fd_handoff_shared_queues_and_drops(oracle_lib):
    """gx.h fd_handoff_shared: with small pipelines that fill, memberlist messages to hosts whose
    handler is blocked queue (and drain once unlocked) or drop; every message sent is either handled,
    queued or dropped; with the knob off none waits. Departures are still all detected."""
    kw = dict(n_hosts=64, n_services=8, init_mode=INIT_OWN, fd_enable=1, depart_round=3, depart_ppm=100000,
              ae_period_rounds=10, queue_cap=4096, lock_buffer=80)
    off = Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    on = Engine(default_params(oracle_lib, fd_handoff_shared=1, **kw), lib=oracle_lib)
    off.run_rounds(200)
    on.run_rounds(200)
    a, b = off.stats(), on.stats()
    assert a["fd_handoff_queued"] == a["fd_handoff_drops"] == 0
    assert b["fd_handoff_queued"] > 0 and b["fd_handoff_drops"] > 0
    waiting = sum(h.hq_len for h in on.fd_hosts())
    assert b["fd_msgs_received"] + waiting + b["fd_handoff_drops"] <= b["fd_msgs_sent"]
    assert b["fd_msgs_received"] < a["fd_msgs_received"]
    assert b["fd_deaths"] >= 64 * 0.05 and a["fd_deaths"] >= 64 * 0.05

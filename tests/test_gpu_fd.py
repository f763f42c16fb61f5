"""memberlist failure detection on the HIP engine: the restated memberlist unit
tests (tests/fd_cases.py) and bit-exact parity with the CPU oracle over the detector scenarios —
catalog views, host bookkeeping, queue digests, server times, counters, every host's member list
and the memberlist broadcast queues."""
import pytest

from sidecar_amd.abi import INIT_WARM, Engine, default_params
from tests import fd_cases
from tests.fd_parity import assert_same_fd
from tests.parity import assert_same

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", fd_cases.ALL, ids=lambda f: f.__name__)
def test_gpu_fd_kat(gx_lib, case):
    case(gx_lib)


def compare(gx_lib, oracle_lib, kw, rounds, chunks=(1, 6, 33, 60)):
    g = Engine(default_params(gx_lib, **kw), lib=gx_lib)
    o = Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    done = 0
    for c in list(chunks) + [rounds]:
        n = min(c, rounds - done)
        if n <= 0:
            break
        g.run_rounds(n)
        o.run_rounds(n)
        done += n
        assert_same(g, o, f"round {g.round}")
        if kw.get("fd_enable"):
            assert_same_fd(g, o, f"round {g.round}")
    assert g.converged() == o.converged()
    if kw.get("fd_enable"):
        assert g.fd_converged() == o.fd_converged()
    g.close()
    o.close()


@pytest.mark.parametrize("name", sorted(fd_cases.SCENARIOS))
def test_gpu_fd_scenario(gx_lib, oracle_lib, name):
    kw, rounds = fd_cases.SCENARIOS[name]
    compare(gx_lib, oracle_lib, kw, rounds)


def test_gpu_fd_h1024_departures(gx_lib, oracle_lib):
    """A larger cluster: 1024 hosts x 16 services, 5% crash at round 10, push-pull every 10
    rounds; the detector declares them dead well within 160 rounds."""
    kw = dict(n_hosts=1024, n_services=16, init_mode=INIT_WARM, fd_enable=1, depart_round=10,
              depart_ppm=50_000, ae_period_rounds=10, queue_cap=4096)
    compare(gx_lib, oracle_lib, kw, 160, chunks=(12, 40))


def test_gpu_fd_api_fuzz(gx_lib, oracle_lib):
    """Seeded single-host calls (notify, get_broadcasts, probe, timers, round advances) agree."""
    import random
    from sidecar_amd.abi import M_ALIVE, M_DEAD, M_SUSPECT
    rnd = random.Random(7)
    kw = dict(n_hosts=24, n_services=4, init_mode=INIT_WARM, fd_enable=1, depart_round=2, depart_ppm=150_000,
              partition_start=30, partition_end=60, fd_gossip_dead_rounds=20)
    g = Engine(default_params(gx_lib, **kw), lib=gx_lib)
    o = Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    for step in range(400):
        host = rnd.randrange(24)
        op = rnd.random()
        if op < 0.45:
            msgs = [(rnd.choice((M_ALIVE, M_SUSPECT, M_DEAD)), rnd.randrange(24), rnd.randrange(4), rnd.randrange(24))
                    for _ in range(rnd.randrange(1, 6))]
            g.fd_notify(host, msgs)
            o.fd_notify(host, msgs)
        elif op < 0.65:
            lim = rnd.randrange(0, 10)
            assert g.fd_get_broadcasts(host, lim) == o.fd_get_broadcasts(host, lim)
        elif op < 0.85:
            assert g.fd_probe(host) == o.fd_probe(host)
        elif op < 0.95:
            g.fd_timers(host)
            o.fd_timers(host)
        else:
            r = g.round + rnd.randrange(1, 15)
            g.set_round(r)
            o.set_round(r)
        if step % 50 == 49:
            assert_same(g, o, f"step {step}")
            assert_same_fd(g, o, f"step {step}")


def test_gpu_fd_with_listeners(gx_lib, oracle_lib):
    """ChangeEvents of NotifyLeave -> ExpireServer reach buffered listeners identically (the
    event-logging kernel variants run while a listener exists)."""
    kw = dict(n_hosts=64, n_services=8, init_mode=INIT_WARM, fd_enable=1, depart_round=3, depart_ppm=100_000,
              ae_period_rounds=10, queue_cap=4096)
    g = Engine(default_params(gx_lib, **kw), lib=gx_lib)
    o = Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    for e in (g, o):
        e.add_listener(0, 1, 16)
        e.add_listener(17, 2, 4096)
    for n in (40, 60, 80):
        g.run_rounds(n)
        o.run_rounds(n)
        for view, lid in ((0, 1), (17, 2)):
            a = [x.tup() for x in g.drain_listener(view, lid)]
            b = [x.tup() for x in o.drain_listener(view, lid)]
            assert a == b, f"round {g.round}: listener {lid} of view {view} differs"
        assert_same(g, o, f"round {g.round}")
        assert_same_fd(g, o, f"round {g.round}")
    assert g.stats()["listener_drops"] > 0  # the 16-event channel overflowed during the deaths

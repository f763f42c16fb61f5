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


def test_gpu_fd_queue_fuzz(gx_lib, oracle_lib):
    """The memberlist broadcast queue under mass updates: pushPull merges (mergeState) whose remote
    lists flag many queued nodes at once, spread over several transmit stacks and chunks (H = 150:
    three 64-node chunks, the last one ragged), interleaved with GetBroadcasts that move and drop
    whole stack prefixes, notifies and round advances. The lane-parallel queue moves and the
    one-walk GetBroadcasts must leave every member row, link and stack as the oracle's sequential
    unlinks and pushes do."""
    import random
    from sidecar_amd.abi import M_ALIVE, M_DEAD, M_SUSPECT
    rnd = random.Random(11)
    H = 150
    kw = dict(n_hosts=H, n_services=2, init_mode=INIT_WARM, fd_enable=1, fd_gossip_dead_rounds=40)
    pg, po = default_params(gx_lib, **kw), default_params(oracle_lib, **kw)
    pg.fd_retransmit_limit = po.fd_retransmit_limit = 3  # messages reach the limit and leave
    g = Engine(pg, lib=gx_lib)
    o = Engine(po, lib=oracle_lib)
    inc = [0] * H  # a rising incarnation per node, so that alive entries keep winning
    hosts = [3, 64, 127, 149]
    for step in range(300):
        host = rnd.choice(hosts)
        op = rnd.random()
        if (step // 40) % 2:  # drain epochs: messages climb the stacks and leave at the limit
            op = 0.3 + 0.3 * op if op < 0.8 else op
        if op < 0.3:
            dens = rnd.choice((0.05, 0.3, 0.9, 1.0))
            remote = []
            for m in range(H):
                if rnd.random() >= dens:
                    remote.append(None if rnd.random() < 0.5 else (M_ALIVE, 0))
                    continue
                inc[m] += rnd.randrange(0, 3)
                remote.append((rnd.choice((M_ALIVE, M_ALIVE, M_SUSPECT, M_DEAD)), inc[m]))
            g.fd_merge_state(host, remote)
            o.fd_merge_state(host, remote)
        elif op < 0.6:
            lim = rnd.choice((1, 5, 17, 40))
            assert g.fd_get_broadcasts(host, lim) == o.fd_get_broadcasts(host, lim), f"step {step}"
        elif op < 0.85:
            msgs = [(rnd.choice((M_ALIVE, M_SUSPECT, M_DEAD)), m, inc[m] + rnd.randrange(0, 2), rnd.randrange(H))
                    for m in rnd.sample(range(H), rnd.randrange(1, 30))]
            g.fd_notify(host, msgs)
            o.fd_notify(host, msgs)
        elif op < 0.95:
            g.fd_timers(host)
            o.fd_timers(host)
        else:
            r = g.round + rnd.randrange(1, 20)
            g.set_round(r)
            o.set_round(r)
        if step % 25 == 24:
            for v in hosts:
                assert g.fd_queue(v) == o.fd_queue(v), f"step {step}: queue of host {v}"
            assert_same_fd(g, o, f"step {step}")
    assert_same(g, o, "queue fuzz")

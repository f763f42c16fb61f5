"""HIP engine vs CPU oracle: bit-exact views, host bookkeeping, queue digests and counters.

Round-model scenarios at sizes the oracle runs in seconds (cfg 1 = 64 hosts x 8 services,
fanout 3, plus edge configurations), and a seeded fuzz of the single-host ABI calls.
"""
import random

import numpy as np
import pytest

from sidecar_amd.abi import (ALIVE, DRAINING, INIT_EMPTY, INIT_OWN, INIT_WARM, TOMBSTONE, UNHEALTHY,
                             Engine, default_params)
from tests.parity import assert_same

pytestmark = pytest.mark.gpu

SCENARIOS = {
    "cfg1_empty": dict(n_hosts=64, n_services=8, init_mode=INIT_EMPTY),
    "cfg1_own_ae": dict(n_hosts=64, n_services=8, init_mode=INIT_OWN, ae_period_rounds=10),
    "cfg1_storm": dict(n_hosts=64, n_services=8, init_mode=INIT_WARM, ae_period_rounds=10,
                       partition_start=0, partition_end=50, storm_round=5, queue_cap=4096),
    "cfg1_churn_aged": dict(n_hosts=64, n_services=8, init_mode=INIT_OWN, churn_ppm=50000,
                            aged_ppm=50000, ae_period_rounds=20, ae_phase=7),
    "tight_bounds": dict(n_hosts=48, n_services=8, init_mode=INIT_WARM, queue_cap=12, list_slots=2,
                         pending_cap=5, packet_cap=4, ae_period_rounds=10, storm_round=3,
                         partition_start=0, partition_end=20, churn_ppm=100000),
    "odd_sizes": dict(n_hosts=37, n_services=3, init_mode=INIT_OWN, fanout=5, ae_period_rounds=7,
                      ae_phase=3, partition_start=10, partition_end=30, churn_ppm=30000),
    "s64": dict(n_hosts=24, n_services=64, init_mode=INIT_EMPTY, ae_period_rounds=15, churn_ppm=20000),
    "retransmit0_nostop": dict(n_hosts=40, n_services=6, init_mode=INIT_EMPTY, retransmit_rounds=0,
                               gossip_stop_on_empty=0, fanout=4),
    "tiny_h2": dict(n_hosts=2, n_services=2, init_mode=INIT_OWN, ae_period_rounds=3),
    "h1": dict(n_hosts=1, n_services=4, init_mode=INIT_EMPTY),
    # ExpireServer storm at every S class: ballot kernel (S | 64) and the generic LDS kernel
    "storm_s2": dict(n_hosts=130, n_services=2, init_mode=INIT_WARM, partition_start=0, partition_end=12,
                     storm_round=3, queue_cap=512, churn_ppm=50000),
    "storm_s3": dict(n_hosts=90, n_services=3, init_mode=INIT_WARM, partition_start=0, partition_end=12,
                     storm_round=2, queue_cap=256, ae_period_rounds=5),
    "storm_s64": dict(n_hosts=70, n_services=64, init_mode=INIT_WARM, partition_start=0, partition_end=12,
                      storm_round=4, queue_cap=64, churn_ppm=100000),
    "storm_s16_qfull": dict(n_hosts=300, n_services=16, init_mode=INIT_WARM, partition_start=0,
                            partition_end=12, storm_round=1, queue_cap=40),
    "high_fanout": dict(n_hosts=20, n_services=4, init_mode=INIT_OWN, fanout=16, packet_cap=8),
    # receiver inboxes with fewer slots than packets: the serial overflow path (key-order walk of
    # the inbox slots + the shared overflow list) must fold exactly like the in-wave path
    "inbox_overflow": dict(n_hosts=40, n_services=4, init_mode=INIT_OWN, fanout=12, packet_cap=8,
                           inbox_slots=3, ae_period_rounds=10, churn_ppm=50000, queue_cap=1024),
    "inbox_overflow_storm": dict(n_hosts=100, n_services=8, init_mode=INIT_WARM, partition_start=0,
                                 partition_end=12, storm_round=2, queue_cap=256, inbox_slots=1, fanout=4),
    # GossipMessages (config/config.go:46): up to 15 gathers per target and round
    "gossip_messages15": dict(n_hosts=64, n_services=8, init_mode=INIT_OWN, gossip_messages=15,
                              ae_period_rounds=10, churn_ppm=50000, queue_cap=2048),
    "gossip_messages4_storm": dict(n_hosts=96, n_services=4, init_mode=INIT_WARM, gossip_messages=4,
                                   partition_start=0, partition_end=15, storm_round=3, queue_cap=1024,
                                   inbox_slots=6),
    # planned GetBroadcasts (send_planned): batches longer than the packet (lists of expired and own
    # tombstones, EXPIRE jobs of 16 records) leave records pending in front of the ring, several
    # calls of a chunk read what earlier calls left there, pending truncation, ring wrap-around
    "plan_pushes": dict(n_hosts=72, n_services=16, init_mode=INIT_WARM, packet_cap=5, pending_cap=7,
                        queue_cap=512, list_slots=4, churn_ppm=80000, aged_ppm=60000, ae_period_rounds=9,
                        partition_start=0, partition_end=14, storm_round=3, fanout=4),
    # many chunks per host: GossipMessages 16 with 3-record packets
    "plan_gm16_cap3": dict(n_hosts=50, n_services=8, init_mode=INIT_OWN, gossip_messages=16, packet_cap=3,
                           pending_cap=9, churn_ppm=60000, queue_cap=1024, ae_period_rounds=12),
    # wide inboxes (65..256 packets per receiver, the default 256 slots with GossipMessages > 1): the
    # wave merge ranks the headers in LDS; receivers past the slots still take the serial path
    "wide_inbox_gm15_storm": dict(n_hosts=96, n_services=8, init_mode=INIT_WARM, fanout=8, gossip_messages=15,
                                  packet_cap=4, partition_start=0, partition_end=12, storm_round=2,
                                  queue_cap=2048, churn_ppm=50000, ae_period_rounds=10),
    "wide_inbox_slots100": dict(n_hosts=80, n_services=4, init_mode=INIT_OWN, fanout=10, gossip_messages=12,
                                packet_cap=3, inbox_slots=100, churn_ppm=80000, queue_cap=1024,
                                ae_period_rounds=9),
    # memberlist's per-node push-pull initiation (every live host starts one exchange per interval)
    "pp_initiate": dict(n_hosts=64, n_services=8, init_mode=INIT_OWN, push_pull_mode=1, ae_period_rounds=5,
                        churn_ppm=30000),
    "pp_initiate_storm_depart": dict(n_hosts=80, n_services=4, init_mode=INIT_WARM, push_pull_mode=1,
                                     ae_period_rounds=4, partition_start=0, partition_end=20, storm_round=3,
                                     queue_cap=1024, depart_round=6, depart_ppm=50000),
    # the FIFO's stored window (gx.h gx_job): push-pull retransmits and EXPIRE jobs past queue_cap
    # are deferred (counted in place), the loopers' nils keep their positions behind them, deferred
    # jobs reaching the head are LOST; both engines must defer and lose the same jobs
    "window_cold_start": dict(n_hosts=64, n_services=8, init_mode=INIT_OWN, ae_period_rounds=10, churn_ppm=50000,
                              aged_ppm=50000, queue_cap=96),
    "window_storm": dict(n_hosts=96, n_services=4, init_mode=INIT_WARM, ae_period_rounds=10, partition_start=0,
                         partition_end=30, storm_round=3, churn_ppm=20000, queue_cap=96),
    # a list arena of two bitmap words (list_slots > 32): long retransmit sleeps keep up to 40 lists
    # live per host, SendServices jobs whose list does not fit are queued LOST
    "lists_two_words": dict(n_hosts=48, n_services=16, init_mode=INIT_WARM, churn_ppm=300000, aged_ppm=100000,
                            queue_cap=4096, list_slots=40, retransmit_rounds=40, tombstone_count=20),
    "window_lists_gm4": dict(n_hosts=64, n_services=16, init_mode=INIT_OWN, ae_period_rounds=10, churn_ppm=200000,
                             aged_ppm=50000, queue_cap=4096, list_slots=40, gossip_messages=4),
}


def pair(oracle_lib, gx_lib, **kw):
    po = default_params(oracle_lib, **kw)
    pg = default_params(gx_lib, **kw)
    return Engine(pg, lib=gx_lib), Engine(po, lib=oracle_lib)


@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_round_model_parity(oracle_lib, gx_lib, name):
    g, o = pair(oracle_lib, gx_lib, **SCENARIOS[name])
    assert_same(g, o, f"{name} init")
    for chunk in (1, 4, 10, 35, 50, 150, 200):
        g.run_rounds(chunk)
        o.run_rounds(chunk)
        assert_same(g, o, f"{name} round {g.round}")
    assert g.converged() == o.converged()


LISTEN = {  # scenario -> [(view, listener id, capacity)]
    "cfg1_storm": [(0, 1, 4), (0, 2, 4096), (40, 1, 300), (63, 7, 1)],
    "cfg1_churn_aged": [(3, 1, 64), (17, 2, 4096)],
    "storm_s3": [(5, 1, 2048), (60, 1, 17)],
    "odd_sizes": [(0, 1, 100), (36, 1, 4096)],
    "inbox_overflow": [(0, 1, 4096), (5, 2, 60)],
    "pp_initiate": [(0, 1, 4096), (9, 1, 100)],
    "gossip_messages15": [(2, 1, 4096)],
    "wide_inbox_gm15_storm": [(0, 1, 4096), (50, 1, 200)],
}


@pytest.mark.parametrize("name", sorted(LISTEN))
def test_change_events_parity(oracle_lib, gx_lib, name):
    """ChangeEvents reach listeners in the same order, with the same drops, on both engines
    (SURVEY §8f-4); server times and state.LastChanged are compared by assert_same."""
    g, o = pair(oracle_lib, gx_lib, **SCENARIOS[name])
    for v, lid, cap in LISTEN[name]:
        g.add_listener(v, lid, cap)
        o.add_listener(v, lid, cap)
    n_ev = 0
    for chunk in (1, 3, 7, 20, 40):
        g.run_rounds(chunk)
        o.run_rounds(chunk)
        assert_same(g, o, f"{name} round {g.round}")
        for v, lid, cap in LISTEN[name]:
            ge = [x.tup() for x in g.drain_listener(v, lid, cap // 2 + 1)]  # leave some buffered
            oe = [x.tup() for x in o.drain_listener(v, lid, cap // 2 + 1)]
            assert ge == oe, f"{name} view {v} listener {lid} round {g.round}"
            n_ev += len(ge)
    assert n_ev > 0 and g.stats()["change_events"] > 0


@pytest.mark.parametrize("limit", [1398, 600, 230])
def test_byte_limit_parity(oracle_lib, gx_lib, limit):
    """packPacket under memberlist's byte limit: a random static-length table
    (ID/Name/Image/Hostname/Ports sizes differ per service) and the round model with churn."""
    kw = dict(n_hosts=64, n_services=8, init_mode=INIT_OWN, limit_bytes=limit, overhead_bytes=3,
              ae_period_rounds=10, churn_ppm=50000, aged_ppm=20000, queue_cap=2048)
    g, o = pair(oracle_lib, gx_lib, **kw)
    rnd = np.random.default_rng(limit)
    tbl = rnd.integers(120, 420, size=64 * 8).astype(np.uint16)
    g.set_static_bytes(0, 64, tbl)
    o.set_static_bytes(0, 64, tbl)
    for chunk in (1, 9, 20, 50):
        g.run_rounds(chunk)
        o.run_rounds(chunk)
        assert_same(g, o, f"bytes {limit} round {g.round}")
    st = g.stats()
    assert st["bytes_sent"] > 0 and st["cap_cuts"] == 0


def test_cfg2_small_parity(oracle_lib, gx_lib):
    """A 1024 x 16 cluster with anti-entropy, churn and expiry-age records."""
    kw = dict(n_hosts=1024, n_services=16, init_mode=INIT_OWN, ae_period_rounds=10, churn_ppm=20000,
              aged_ppm=20000, queue_cap=512)
    g, o = pair(oracle_lib, gx_lib, **kw)
    for chunk in (3, 9, 12):
        g.run_rounds(chunk)
        o.run_rounds(chunk)
        assert_same(g, o, f"cfg2-small round {g.round}")


def test_fuzz_single_host_api(oracle_lib, gx_lib):
    """Seeded random sequences of the ServicesState / delegate entry points."""
    rnd = random.Random(1234)
    H, S = 12, 6
    g, o = pair(oracle_lib, gx_lib, n_hosts=H, n_services=S, queue_cap=40, list_slots=4, pending_cap=20,
                packet_cap=6, init_mode=INIT_OWN)
    T0 = g.now(0)
    for step in range(400):
        op = rnd.randrange(12)
        now = g.now()
        rec = lambda: (rnd.randrange(H), rnd.randrange(S), now - rnd.randrange(0, 200) * 10**9 + rnd.randrange(3) * 50,
                       rnd.choice([ALIVE, TOMBSTONE, UNHEALTHY, DRAINING]))
        if op == 0:
            items = [rec() for _ in range(rnd.randrange(1, 20))]
            views = [rnd.randrange(H) for _ in items]
            assert g.add_service_entries(views, items) == o.add_service_entries(views, items)
        elif op == 1:
            h = rnd.randrange(H)
            items = [rec() for _ in range(rnd.randrange(0, 12))]
            g.notify_msg(h, items)
            o.notify_msg(h, items)
        elif op == 2:
            h = rnd.randrange(H)
            lim = rnd.choice([None, 0, 1, 3, 6])
            a, b = g.get_broadcasts(h, lim), o.get_broadcasts(h, lim)
            assert (a is None) == (b is None)
            if a is not None:
                assert [x.tup() for x in a] == [x.tup() for x in b]
        elif op == 3:
            v, w = rnd.randrange(H), rnd.randrange(H)
            assert g.expire_server(v, w) == o.expire_server(v, w)
        elif op == 4:
            h = rnd.randrange(H)
            items = [rec() for _ in range(rnd.randrange(0, 40))]
            np_ = rnd.randrange(1, 4)
            g.send_services(h, items, np_)
            o.send_services(h, items, np_)
        elif op == 5:
            h = rnd.randrange(H)
            items = [(h, s, now, rnd.choice([ALIVE, UNHEALTHY])) for s in sorted(rnd.sample(range(S), rnd.randrange(0, S + 1)))]
            g.broadcast_services(h, items)
            o.broadcast_services(h, items)
        elif op == 6:
            h = rnd.randrange(H)
            items = [(h, s, now, ALIVE) for s in sorted(rnd.sample(range(S), rnd.randrange(0, S + 1)))]
            g.broadcast_tombstones(h, items)
            o.broadcast_tombstones(h, items)
        elif op == 7:
            v = rnd.randrange(H)
            a, na = g.tombstone_others(v)
            b, nb = o.tombstone_others(v)
            assert na == nb and [x.tup() for x in a] == [x.tup() for x in b]
        elif op == 8:
            d, s_ = rnd.randrange(H), rnd.randrange(H)
            g.merge(d, s_)
            o.merge(d, s_)
        elif op == 9:
            r = g.round + rnd.randrange(0, 8)
            g.set_round(r)
            o.set_round(r)
        elif op == 10:
            n = rnd.randrange(1, 6)
            g.run_rounds(n)
            o.run_rounds(n)
        else:
            h = rnd.randrange(H)
            run = sorted(rnd.sample(range(S), rnd.randrange(0, S + 1)))
            a = g.tombstone_services(h, run)
            b = o.tombstone_services(h, run)
            assert [x.tup() for x in a] == [x.tup() for x in b]
        if step % 20 == 19:
            assert_same(g, o, f"fuzz step {step}")
    assert_same(g, o, "fuzz end")
    assert T0 <= g.now()

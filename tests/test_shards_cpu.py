"""Host sharding on the CPU oracle: a cluster split into G shards (exchange layer in
sidecar_amd/dist.py) must evolve bit-identically to the unsharded cluster — views, per-host
bookkeeping, queue digests and the summed counters. Also over torch.distributed gloo with two
processes (the same protocol the GPUs run over RCCL)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from sidecar_amd.abi import Engine, default_params
from sidecar_amd.dist import LocalShards
from tests.parity import host_tuples

SCEN = {
    "storm": dict(n_hosts=48, n_services=8, init_mode=2, ae_period_rounds=10, partition_start=0,
                  partition_end=30, storm_round=4, queue_cap=2048),
    "churn_odd": dict(n_hosts=37, n_services=3, init_mode=1, fanout=4, ae_period_rounds=7, ae_phase=2,
                      churn_ppm=60000, aged_ppm=40000, queue_cap=64, list_slots=3),
    "empty": dict(n_hosts=40, n_services=6, init_mode=0, ae_period_rounds=9),
    # rows of several 512-slot digest blocks (R = 1536), and a partial last block (R = 770)
    "blocks3": dict(n_hosts=96, n_services=16, init_mode=2, ae_period_rounds=5, partition_start=0,
                    partition_end=12, storm_round=3, churn_ppm=30000, queue_cap=4096),
    "blocks_ragged": dict(n_hosts=70, n_services=11, init_mode=1, ae_period_rounds=4, ae_phase=1,
                          churn_ppm=80000, aged_ppm=50000, queue_cap=1024),
    # host crashes: lost packets across shards, push-pull pairs with a crashed member skipped
    "departures": dict(n_hosts=60, n_services=8, init_mode=2, ae_period_rounds=5, partition_start=0,
                       partition_end=12, storm_round=3, depart_round=4, depart_ppm=150000, queue_cap=2048),
    # memberlist failure detection across shards: memberlist messages ride in the packet slots,
    # the push-pull initiator's decision travels in the digest header
    "fd": dict(n_hosts=64, n_services=8, init_mode=2, ae_period_rounds=5, partition_start=0,
               partition_end=45, depart_round=3, depart_ppm=100000, fd_enable=1, queue_cap=4096),
    "fd_gm6": dict(n_hosts=56, n_services=6, init_mode=2, ae_period_rounds=5, partition_start=0,
                   partition_end=30, depart_round=4, depart_ppm=80000, fd_enable=1, queue_cap=4096,
                   gossip_messages=6),
    "fd_bytes": dict(n_hosts=50, n_services=6, init_mode=1, ae_period_rounds=4, churn_ppm=30000, depart_round=10,
                     depart_ppm=100000, fd_enable=1, limit_bytes=1398, packet_cap=48, queue_cap=2048),
    # received packets registered in overflowed inboxes (inbox_slots is an engine bound)
    "inbox_overflow": dict(n_hosts=45, n_services=4, init_mode=1, fanout=8, packet_cap=6, inbox_slots=2,
                           ae_period_rounds=6, churn_ppm=50000, queue_cap=512),
}


def assert_sharded_equal(whole: Engine, shards, what):
    sw = whole.stats()
    ss = shards.stats()
    assert sw == ss, {k: (sw[k], ss[k]) for k in sw if sw[k] != ss[k]}
    views = np.concatenate([e.read_views() for e in shards.engines])
    assert np.array_equal(views, whole.read_views()), what
    hosts = sum((host_tuples(e) for e in shards.engines), [])
    assert hosts == host_tuples(whole), what
    dig = np.concatenate([e.digests() for e in shards.engines])
    assert np.array_equal(dig, whole.digests()), what
    c, n = shards.converged()
    cw, nw = whole.converged()
    if cw and whole.params.fd_enable:
        cw, nw = whole.fd_converged()
    assert c == cw, what
    if not whole.params.fd_enable or n == 0 or nw == 0:
        assert n == nw, what  # sharded membership counts sum per shard
    lc = np.concatenate([e.last_changed() for e in shards.engines])
    assert np.array_equal(lc, whole.last_changed()), what
    for e in shards.engines:
        for v in (e.lo, (e.lo + e.hi) // 2, e.hi - 1):
            assert np.array_equal(e.server_times(v), whole.server_times(v)), (what, v)
    if whole.params.fd_enable:  # every host's member list, probe/queue state and queue
        for e in shards.engines:
            assert [bytes(h) for h in e.fd_hosts(e.lo, e.hi)] == [bytes(h) for h in whole.fd_hosts(e.lo, e.hi)], what
            for v in range(e.lo, e.hi):
                assert e.fd_members(v) == whole.fd_members(v), (what, v)
                assert e.fd_queue(v) == whole.fd_queue(v), (what, v)
        assert all(e.fd_converged()[0] for e in shards.engines) == whole.fd_converged()[0], what


@pytest.mark.parametrize("G", [2, 3, 5, 8])
@pytest.mark.parametrize("name", sorted(SCEN))
def test_local_shards_match_whole(oracle_lib, name, G):
    kw = SCEN[name]
    whole = Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    sh = LocalShards(oracle_lib, G, **kw)
    for chunk in (1, 6, 13, 40):
        whole.run_rounds(chunk)
        sh.run_rounds(chunk)
        assert_sharded_equal(whole, sh, f"{name} G={G} round {whole.round}")


def _worker(rank, world, port, kw, rounds, q):
    import torch.distributed as dist
    from sidecar_amd.dist import DistShard
    from tests.oracle_lib import load_oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sh = DistShard(load_oracle(), rank, world, "cpu", **kw)
    sh.run_rounds(rounds)
    st = sh.stats()
    conv = sh.converged()
    q.put((rank, sh.e.read_views(), host_tuples(sh.e), sh.e.digests(), st, conv, sh.ae_skipped))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


LOCKED = dict(n_hosts=64, n_services=16, init_mode=2, ae_period_rounds=10, partition_start=0,
              partition_end=30, storm_round=5, queue_cap=2048)  # every host locked from round ~10


@pytest.mark.parametrize("name", ["storm", "churn_odd", "locked"])
def test_gloo_world2_matches_whole(oracle_lib, name):
    kw, rounds, world = (LOCKED if name == "locked" else SCEN[name]), 45, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, kw, rounds, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in ps], key=lambda x: x[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    whole = Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    whole.run_rounds(rounds)
    assert np.array_equal(np.concatenate([r[1] for r in res]), whole.read_views())
    assert sum((r[2] for r in res), []) == host_tuples(whole)
    assert np.array_equal(np.concatenate([r[3] for r in res]), whole.digests())
    assert res[0][4] == whole.stats()
    assert res[0][5] == whole.converged()
    if name == "locked":  # the census collective found every host locked: the exchange was skipped
        assert res[0][6] == res[1][6] > 0


def test_delta_ships_only_differing_blocks(oracle_lib):
    """Push-pull across shards sends digests, then only the 512-slot blocks that differ (each led
    by one side, run-length coded, and answered with the words that change the leader's merge): a
    converged (warm) cluster ships no blocks at all; after a storm the delta is a fraction of
    the full rows; the views stay identical to the unsharded run either way."""
    kw = dict(n_hosts=96, n_services=16, init_mode=2, ae_period_rounds=5, partition_start=0,
              partition_end=8, storm_round=2, queue_cap=4096)
    whole = Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    sh = LocalShards(oracle_lib, 3, **kw)
    whole.run_rounds(1)
    sh.run_rounds(1)  # round 0 is a push-pull round over identical views
    w = sh.wire.as_dict()
    assert w["ae_digest"] > 0 and w["ae_full_rows_equivalent"] > 0
    n_msgs = w["ae_digest"] // (16 + 16 * 3)
    assert w["ae_lead"] == 16 * n_msgs and w["ae_return"] == (8 + 16) * n_msgs  # headers only
    whole.run_rounds(29)
    sh.run_rounds(29)
    assert_sharded_equal(whole, sh, "delta")
    w = sh.wire.as_dict()
    assert 40 * n_msgs < w["ae_delta"] < w["ae_full_rows_equivalent"]


@pytest.mark.parametrize("field", ["key", "receiver", "len", "local_key", "rec_key", "dup"])
def test_corrupt_inbox_slot_refused(oracle_lib, field):
    import torch
    from tests.corrupt_inbox import run, run_valid
    assert run_valid(oracle_lib, torch.device("cpu")) >= 0
    assert run(oracle_lib, torch.device("cpu"), field) == "einval"


@pytest.mark.parametrize("G", [2, 3])
def test_locked_push_pull_rounds_skip_the_exchange(oracle_lib, G):
    """A push-pull round with every host of the cluster holding the ServicesState lock is replaced
    by gx_ae_skip_locked after one census (gx_lock_census summed over the shards): the same
    counts as the whole exchange (ae_locked once per pair, first_locked_round) and the same state,
    against the unsharded engine and against the shards running the exchange anyway."""
    kw = dict(n_hosts=64, n_services=16, init_mode=2, ae_period_rounds=10, partition_start=0,
              partition_end=30, storm_round=5, queue_cap=2048)
    whole = Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    fast = LocalShards(oracle_lib, G, **kw)
    full = LocalShards(oracle_lib, G, **kw)
    full.skip_locked = False
    for sh in (fast, full):
        sh.run_rounds(41)
    whole.run_rounds(41)
    assert fast.ae_skipped > 0 and full.ae_skipped == 0
    assert whole.stats()["ae_locked"] > 0
    assert_sharded_equal(whole, fast, "skipped locked push-pull rounds")
    assert_sharded_equal(whole, full, "whole exchanges")
    assert fast.wire.ae_digest < full.wire.ae_digest  # nothing moved in the skipped rounds

"""Which gossip exchange a sharded round takes (sidecar_amd.dist.planned_exchange): the planned one
(seeded slot counts, no size collective, no host wait; gx_exchange_plan) iff the failure detector is
off and GossipMessages is at most one message per target, 0 included. Round 4 once sent
GossipMessages 0 down the size-gathered exchange and only a sync-debug GPU test noticed; these tests
pin the choice on the CPU, for LocalShards and for DistShard over gloo."""
import multiprocessing as mp
import os
import socket

import pytest

from sidecar_amd.abi import Engine, default_params
from sidecar_amd.dist import LocalShards, planned_exchange

CASES = [  # (params, planned)
    (dict(gossip_messages=0), True),
    (dict(gossip_messages=1), True),
    (dict(gossip_messages=2), False),
    (dict(gossip_messages=15), False),
    (dict(gossip_messages=0, fd_enable=1), False),
    (dict(gossip_messages=1, fd_enable=1), False),
]
BASE = dict(n_hosts=32, n_services=4, init_mode=2, ae_period_rounds=5, partition_start=0, partition_end=6,
            storm_round=2, queue_cap=2048)


@pytest.mark.parametrize("kw,planned", CASES)
def test_planned_exchange_predicate(oracle_lib, kw, planned):
    assert planned_exchange(default_params(oracle_lib, **dict(BASE, **kw))) is planned


@pytest.mark.parametrize("kw,planned", CASES)
def test_local_shards_take_the_planned_exchange(oracle_lib, kw, planned):
    kw = dict(BASE, **kw)
    sh = LocalShards(oracle_lib, 2, **kw)
    calls = {"plan": 0}
    eng = sh.shards[0].e
    orig = eng.round_gossip_begin  # the planned round's first call (gx_exchange_plan inside)

    def counted(*a):
        calls["plan"] += 1
        return orig(*a)

    eng.round_gossip_begin = counted
    sh.run_rounds(7)
    assert sh.exchange_paths == ({"planned": 7, "sized": 0} if planned else {"planned": 0, "sized": 7})
    assert calls["plan"] == (7 if planned else 0)
    whole = Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    whole.run_rounds(7)
    assert sh.stats()["gossip_merges"] == whole.stats()["gossip_merges"]


def _worker(rank, world, port, kw, q, chunk=None, rounds=6):
    import torch.distributed as dist
    from sidecar_amd.dist import DistShard
    from tests.oracle_lib import load_oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sh = DistShard(load_oracle(), rank, world, "cpu", **kw)
    if chunk:
        sh.CHUNK = chunk  # every per-peer segment in several all-to-all calls
    sh.run_rounds(rounds)
    st = sh.stats()
    q.put((rank, dict(sh.exchange_paths), st["gossip_merges"], st, sh.e.digests()))
    dist.barrier()
    sh.close()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("gm,planned", [(0, True), (1, True), (4, False)])
def test_dist_shard_takes_the_planned_exchange(oracle_lib, gm, planned):
    kw = dict(BASE, gossip_messages=gm)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, kw, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in ps], key=lambda x: x[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = {"planned": 6, "sized": 0} if planned else {"planned": 0, "sized": 6}
    assert all(r[1] == want for r in res), res
    whole = Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    whole.run_rounds(6)
    assert res[0][2] == whole.stats()["gossip_merges"]


def test_fused_round_calls_equal_separate_calls(oracle_lib):
    """gx_round_gossip_begin / _end (ABI 8, what DistShard's planned path calls) do exactly the work
    of round_send + exchange_plan + outbox_pack_planned and inbox_unpack + round_merge (+ round_end
    outside push-pull rounds): two 2-shard clusters, one stepped each way with the same in-process
    exchange, end with equal digests, host bookkeeping and counters."""
    import numpy as np
    kw = dict(BASE, gossip_messages=1)

    def cluster():
        out = []
        for g in range(2):
            p = default_params(oracle_lib, **kw)
            p.n_shards, p.shard_id = 2, g
            out.append(Engine(p, lib=oracle_lib))
        return out

    def step(es, fused):
        bufs, plans = [], []
        for e in es:
            plan = np.zeros(4, dtype=np.uint64)
            cap = int(e.params.n_hosts * e.params.fanout * (16 + 16 * e.params.packet_cap))
            buf = np.zeros(cap, dtype=np.uint8)
            if fused:
                e.round_gossip_begin(plan, buf.ctypes.data, cap)
            else:
                e.round_send()
                plan[:] = e.exchange_plan().reshape(-1)
                e.outbox_pack_planned(buf.ctypes.data, cap)
            bufs.append(buf)
            plans.append(plan.reshape(2, 2))
        m = plans[0]
        ae = []
        for g, e in enumerate(es):
            src = 1 - g
            off = int(m[src][:g].sum())
            n = int(m[src][g])
            x = np.ascontiguousarray(bufs[src][off:off + n])
            if fused:
                ae.append(e.round_gossip_end(x.ctypes.data, n))
            else:
                e.inbox_unpack(x.ctypes.data, n)
                e.round_merge()
                ae.append(e.is_ae_round())
        assert ae[0] == ae[1]
        for e in es:  # (no push-pull round in these steps: the caller would run it before round_end)
            if not fused or ae[0]:
                e.round_end()

    a, b = cluster(), cluster()
    for _ in range(4):  # rounds 0..3: ae_period_rounds 5 keeps push-pull out
        step(a, True)
        step(b, False)
    for ea, eb in zip(a, b):
        assert ea.round == eb.round == 4
        assert np.array_equal(ea.digests(), eb.digests())
        assert [bytes(h) for h in ea.hosts()] == [bytes(h) for h in eb.hosts()]
        assert ea.stats() == eb.stats()


def test_dist_shard_planned_exchange_in_chunks(oracle_lib):
    """A planned round whose per-peer segment exceeds CHUNK goes in several all-to-all calls over
    the persistent buffers (every rank makes ceil(largest / CHUNK) of them): with CHUNK below one
    packet slot (528 B) every gossip round is chunked, and the two gloo ranks end equal to the
    unsharded oracle (counters summed over the shards)."""
    kw = dict(BASE, gossip_messages=1, partition_end=0, n_hosts=48)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, kw, q, 200, 12)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in ps], key=lambda x: x[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[1] == {"planned": 12, "sized": 0} for r in res), res
    whole = Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    whole.run_rounds(12)
    assert res[0][3] == whole.stats()
    import numpy as np
    dig = whole.digests()
    half = kw["n_hosts"] // 2  # each rank's digests are its own hosts'
    assert np.array_equal(res[0][4], dig[:half]) and np.array_equal(res[1][4], dig[half:])

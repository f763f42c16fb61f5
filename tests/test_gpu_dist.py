"""The multi-process sharded path (sidecar_amd.dist.DistShard, what bench.py runs at N > 1) on the
HIP engine: two processes on the one GPU of the test box, collectives over gloo staged through
the host (RCCL refuses two ranks on one device). Everything the ranks do on the device — outbox
plan and pack, inbox unpack, cross-shard push-pull digests, lead and return blocks, merges — is
the RCCL path's; the views, per-host bookkeeping, queue digests and summed counters must equal
the unsharded CPU oracle's."""
import os

import numpy as np
import pytest
import torch.multiprocessing as mp

from sidecar_amd.abi import Engine, default_params
from tests.parity import host_tuples
from tests.test_shards_cpu import SCEN, _free_port

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, kw, rounds, q):
    import torch
    import torch.distributed as dist
    from sidecar_amd.abi import load_product
    from sidecar_amd.dist import DistShard
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        sh = DistShard(load_product(), rank, world, "cuda:0", **kw)
        assert sh.stage
        sh.run_rounds(rounds)
        st = sh.stats()
        conv = sh.converged()
        fd = sh.e.fd_converged()[1] if kw.get("fd_enable") else 0
        q.put((rank, sh.e.read_views(), host_tuples(sh.e), sh.e.digests(), st, (conv, fd), None))
        dist.barrier()
        sh.close()
        dist.destroy_process_group()
    except Exception as ex:  # reported to the parent instead of a silent hang on q.get
        q.put((rank, None, None, None, None, None, repr(ex)))
        raise


@pytest.mark.parametrize("name,world", [("storm", 2), ("blocks3", 2), ("fd", 2), ("departures", 3)])
def test_gpu_dist_gloo_matches_oracle(oracle_lib, name, world):
    kw, rounds = SCEN[name], 40
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, kw, rounds, q)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        res = sorted([q.get(timeout=100) for _ in ps], key=lambda x: x[0])
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    errs = [r[6] for r in res if r[6]]
    assert not errs, errs
    for p in ps:
        assert p.exitcode == 0
    whole = Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    whole.run_rounds(rounds)
    assert np.array_equal(np.concatenate([r[1] for r in res]), whole.read_views())
    assert sum((r[2] for r in res), []) == host_tuples(whole)
    assert np.array_equal(np.concatenate([r[3] for r in res]), whole.digests())
    assert res[0][4] == whole.stats()
    (c, n), fd = res[0][5][0], [r[5][1] for r in res]
    cw, nw = whole.converged()
    if nw == 0 and kw.get("fd_enable"):
        cw, nw = whole.fd_converged()
        # a node misjudged in several shards counts once per shard in the sharded sum
        assert max(fd) <= nw <= sum(fd) and n == sum(fd)
    else:
        assert n == nw
    assert c == cw

"""bench.py's N>1 path (Cluster over DistShard, run_converge) rehearsed on the CPU oracle over
gloo with two ranks: the sharded cluster must report the unsharded cluster's counters and
rounds-to-converge, and the exchange byte accounting must add up."""
import os
import socket

import torch.multiprocessing as mp


import pytest


def _worker(rank, port, q, cfg):
    import torch.distributed as dist
    import bench
    from tests.oracle_lib import load_oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        lib = load_oracle()
        c = bench.Cluster(lib, cfg, 0x5EED, rank, 2, rank, dist.barrier, device="cpu")
        c.run_rounds(45)
        st, x = c.stats(), c.exchange_bytes()
        c.close()
        conv = bench.run_converge(lib, cfg, 0x5EED, rank, 2, rank, dist.barrier, 600, 10, device="cpu")
        q.put((rank, st, x, conv[0]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cfg", ["cfg1", "cfg1fd"])
def test_bench_cluster_gloo_world2(oracle_lib, cfg):
    import bench
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, port, q, cfg)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    whole = bench.make_engine(oracle_lib, cfg, 0x5EED, 0)
    whole.run_rounds(45)
    ref = whole.stats()
    whole.close()
    (_, st0, x0, conv0), (_, st1, x1, conv1) = res
    assert st0 == st1 == ref
    assert x0 == x1 and x0["packets"] > 0
    assert conv0 == conv1
    ref_conv = bench.run_converge(oracle_lib, cfg, 0x5EED, 0, 1, 0, lambda: None, 600, 10)
    assert conv0 == ref_conv[0]

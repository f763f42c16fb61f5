"""The RCCL (backend "nccl") calls bench.py makes at N > 1, on the one GPU of the test box.

RCCL refuses two ranks on one device, so the multi-rank exchange is rehearsed over gloo
(tests/test_gpu_dist.py). This file runs a one-rank RCCL group instead: DistShard's collectives
(size all-gather, chunked all_to_all_single with split sizes, MIN/MAX/SUM all-reduce on int64
device tensors) and a whole sharded run through them, on RCCL's own stream, so the API use and
the stream ordering between the engine's kernels and the collectives are exercised on hardware.
"""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from sidecar_amd.abi import Engine, default_params
from tests.parity import host_tuples
from tests.test_shards_cpu import SCEN

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(port, kw, rounds, q):
    import torch
    import torch.distributed as dist
    from sidecar_amd.abi import load_product
    from sidecar_amd.dist import DistShard
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1)
        sh = DistShard(load_product(), 0, 1, "cuda:0", **kw)
        assert not sh.stage and dist.get_backend() == "nccl"

        # chunked all-to-all of a device buffer the packer fills (a device-to-device copy into
        # the pointer it is handed, as the engine's pack kernels do)
        hip = ctypes.CDLL("libamdhip64.so")
        n = 4500
        src = torch.arange(n, dtype=torch.int64, device="cuda:0").to(torch.uint8)

        def packer(ptr, cap):
            assert cap == n
            assert hip.hipMemcpy(ctypes.c_void_p(ptr), ctypes.c_void_p(src.data_ptr()), ctypes.c_size_t(n), 3) == 0

        sh.CHUNK = 1000  # five calls
        got = sh._exchange(np.array([n], dtype=np.uint64), packer)
        ok_a2a = bool(torch.equal(got, src))
        sizes = torch.tensor([n], dtype=torch.int64, device="cuda:0")  # device-side sizes
        got2 = sh._exchange(sizes, packer)
        ok_a2a &= bool(torch.equal(got2, src))
        t = torch.tensor([5, -3, 1 << 62], dtype=torch.int64, device="cuda:0")
        sh._all_reduce(t, dist.ReduceOp.MIN)
        ok_red = t.tolist() == [5, -3, 1 << 62]
        del sh.CHUNK

        sh.run_rounds(rounds)
        st = sh.stats()
        conv = sh.converged()
        q.put((sh.e.read_views(), host_tuples(sh.e), sh.e.digests(), st, conv, ok_a2a, ok_red, None))
        sh.close()  # the engine's streams drained and its buffers freed before RCCL's teardown
        torch.cuda.synchronize()
        dist.destroy_process_group()
    except Exception as ex:  # reported to the parent instead of a silent hang on q.get
        q.put((None,) * 7 + (repr(ex),))
        raise


@pytest.mark.parametrize("name", ["storm", "fd"])
def test_gpu_rccl_one_rank_matches_oracle(oracle_lib, name):
    kw, rounds = SCEN[name], 30
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), kw, rounds, q))
    p.start()
    try:
        views, hosts, dig, st, conv, ok_a2a, ok_red, err = q.get(timeout=100)
    finally:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert err is None, err
    assert p.exitcode == 0
    assert ok_a2a and ok_red
    whole = Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    whole.run_rounds(rounds)
    assert np.array_equal(views, whole.read_views())
    assert hosts == host_tuples(whole)
    assert np.array_equal(dig, whole.digests())
    assert st == whole.stats()
    cw, nw = whole.converged()
    if cw and kw.get("fd_enable"):
        cw, nw = whole.fd_converged()
    assert conv == (cw, nw)

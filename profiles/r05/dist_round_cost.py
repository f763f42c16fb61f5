"""Wall time of a sharded round (sidecar_amd.dist.DistShard, what bench.py runs at N > 1) against the
unsharded engine, on the one GPU of the test box: a one-rank RCCL group, so every collective runs
but moves nothing across GPUs. The difference is the host's cost per round (Python, ctypes, the
collectives' launch) that an N-GPU run pays on every rank.

    python profiles/r05/dist_round_cost.py [--config cfg5] [--start 21] [--rounds 29] [--lock-model 1]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg5")
    ap.add_argument("--start", type=int, default=21)
    ap.add_argument("--rounds", type=int, default=29)
    ap.add_argument("--lock-model", type=int, default=1)
    ap.add_argument("--cprofile", action="store_true", help="profile the host side of the sharded rounds")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    import bench
    from sidecar_amd.abi import load_product
    from sidecar_amd.dist import DistShard
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    lib = load_product()
    kw = dict(bench.CONFIGS[a.config]["p"], seed=0x5EED, lock_model=a.lock_model)
    out = {"config": a.config, "lock_model": a.lock_model, "rounds": [a.start, a.start + a.rounds - 1]}
    for mode in ("engine", "dist"):
        if mode == "engine":
            e = bench.make_engine(lib, a.config, 0x5EED, 0, lock_model=a.lock_model)
            run, close = e.run_rounds, e.close
        else:
            sh = DistShard(lib, 0, 1, "cuda:0", **kw)
            e = sh.e
            run, close = sh.run_rounds, e.close
        run(a.start)
        torch.cuda.synchronize()
        per = []
        for _ in range(a.rounds):
            t0 = time.perf_counter()
            r = e.round
            run(1)
            torch.cuda.synchronize()
            per.append((r, 1e3 * (time.perf_counter() - t0)))
        prof = None
        if a.cprofile and mode == "dist":
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        t0 = time.perf_counter()
        run(a.rounds)  # back to back, one sync at the end
        torch.cuda.synchronize()
        if prof is not None:
            prof.disable()
            import io
            import pstats
            buf = io.StringIO()
            pstats.Stats(prof, stream=buf).sort_stats("tottime").print_stats(25)
            print(buf.getvalue(), file=sys.stderr)
        out[mode] = {"ms_per_round_synced": {str(r): round(ms, 3) for r, ms in per},
                     "ms_per_round_back_to_back": round(1e3 * (time.perf_counter() - t0) / a.rounds, 3)}
        close()
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

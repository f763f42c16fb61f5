"""Device time of the gossip-only rounds between two push-pull rounds (cfg 5 rounds 11..19), with
two events around them on a dedicated stream; run under rocprofv3 --kernel-trace to see the
kernels and the gaps between them.

  python profiles/gossip_span.py [config] [first_round] [n]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from sidecar_amd.abi import load_product  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg5"
r0 = int(sys.argv[2]) if len(sys.argv) > 2 else 11
n = int(sys.argv[3]) if len(sys.argv) > 3 else 9
lib = load_product()
e = bench.make_engine(lib, cfg, 1, 0)
e.run_rounds(r0)
st = torch.cuda.Stream()
e.set_stream(st.cuda_stream, False)
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for rep in range(2):
    a.record(st)
    e.run_rounds(n)
    b.record(st)
    b.synchronize()
    print(f"rounds {e.round - n}..{e.round - 1}: {1e3 * a.elapsed_time(b) / n:.1f} us per round", flush=True)
    e.run_rounds(1)  # the push-pull round

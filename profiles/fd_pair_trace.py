"""One falsely-dead pair of the cfg5fd scenario at H = 256 on the CPU oracle:
host Y's member entry for X, X's own incarnation, Y's catalog record of X's first service, X's own
view of it, and X's BroadcastServices looper and broadcast-queue depth, every round in which any
of them changes.

  python profiles/fd_pair_trace.py [H] [partition_end] [rounds] [X] [Y]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from sidecar_amd.abi import Engine, default_params  # noqa: E402
from tests.oracle_lib import load_oracle  # noqa: E402

H = int(sys.argv[1]) if len(sys.argv) > 1 else 256
pe = int(sys.argv[2]) if len(sys.argv) > 2 else 100
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 1500
X = int(sys.argv[4]) if len(sys.argv) > 4 else 1
Y = int(sys.argv[5]) if len(sys.argv) > 5 else H - 1
e = Engine(default_params(load_oracle(), **dict(bench.CONFIGS["cfg5fd"]["p"], n_hosts=H, partition_end=pe)),
           lib=load_oracle())
S, T0 = e.S, e.params.t0_ns
STATE = {0: "alive", 1: "suspect", 2: "dead"}
STATUS = {0: "ALIVE", 1: "TOMBSTONE", 2: "UNHEALTHY", 3: "UNKNOWN", 4: "DRAINING", None: "-"}
print(f"H={H} partition [0,{pe}) X={X} Y={Y}; times are seconds after t0")


def rec(view):
    s = e.slot(view, X, 0)
    return "-" if s is None else f"{STATUS[s[1]]}@{(s[0] - T0) / 1e9:.1f}s"


last = None
for r in range(rounds):
    e.run_rounds(1)
    my, mx = e.fd_member(Y, X), e.fd_member(X, X)
    hx = e.hosts()[X]
    row = (STATE[my.state], my.incarnation, mx.incarnation, rec(Y), rec(X),
           "blocked" if hx.flags & 1 else "running", hx.fifo_tail - hx.fifo_head)
    key = row[:6]
    if key != last:
        print(f"round {e.round:5d}: Y sees X {row[0]:7s} inc {row[1]:3d} | X inc {row[2]:3d} | Y's record {row[3]:20s}"
              f" | X's record {row[4]:20s} | X BroadcastServices {row[5]}, queue {row[6]}")
        last = key

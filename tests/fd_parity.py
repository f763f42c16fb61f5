"""Bit-for-bit comparison of two engines' memberlist failure-detection state:
every host's member list (incarnation, state, StateChange, suspicion deadline and confirmers,
queued message and queue links), per-host probe/queue bookkeeping, and the broadcast queues."""


def fd_snapshot(e, queues=8):
    H = e.H
    step = max(1, H // queues)
    return {
        "members": [e.fd_members(v) for v in range(H)],
        "hosts": [bytes(h) for h in e.fd_hosts()],
        "queues": {v: e.fd_queue(v) for v in range(0, H, step)},
    }


def assert_same_fd(a, b, what=""):
    sa, sb = fd_snapshot(a), fd_snapshot(b)
    for v, (x, y) in enumerate(zip(sa["hosts"], sb["hosts"])):
        assert x == y, f"{what}: fd host state of {v} differs"
    for v, (x, y) in enumerate(zip(sa["members"], sb["members"])):
        assert x == y, f"{what}: member list of host {v} differs"
    assert sa["queues"] == sb["queues"], f"{what}: memberlist broadcast queues differ"

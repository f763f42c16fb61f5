"""Known-answer cases for the ServicesState lock held by a blocked looper (gx.h lock_model,
DESIGN.md §3c), restated from the reference's code paths:

- BroadcastServices holds state.RLock() while it blocks on `Broadcasts <- nil`
  (catalog/services_state.go:535-536,569); BroadcastTombstones holds state.Lock() while it blocks on
  its own nil (:610-611,628);
- AddServiceEntry (:296), ExpireServer (:151) and, behind a pending writer, LocalState
  (services_delegate.go:148) wait for the lock; gossip records queue in the inbound pipeline
  (memberlist's handoff queue, notifications :38, ServiceMsgs :97) and merge in arrival order once the
  lock is released.

Each case drives a small cluster through gx_run_rounds and checks the observable effect round by
round; tests/test_lock_cpu.py runs them on the oracle, tests/test_gpu_lock.py on the HIP engine
against the oracle. The reference has no test for this behaviour (its unit tests never block a
looper behind a queue), so the cases pin the restatement, not a reference fixture.
"""
from sidecar_amd.abi import (INIT_OWN, INIT_WARM, LOCK_DEFER_MERGE, LOCK_PENDING_EXPIRE, TOMBSTONE, Engine,
                             default_params)

# loopers tick only when a case makes them (their phase is seeded within a 1000-round interval)
QUIET = dict(alive_interval_rounds=1000, tombstone_interval_rounds=1000)


def _engine(lib, **kw):
    return Engine(default_params(lib, **kw), lib=lib)


def _block_bs(e, host, k):
    """Queue k one-pass SendServices jobs at `host`, then run its BroadcastServices body until it
    has nothing new and no refresh due: it sends a nil behind the queued jobs and the looper blocks
    holding the read lock. Returns the nil's queue position p: with one GetBroadcasts call per round
    from round 0 on, the nil is taken in round p, so round p + 1 is the host's first unlocked round."""
    own = [(host, s, e.now()) for s in range(e.S)]
    for _ in range(k):
        e.send_services(host, own, 1)
    e.broadcast_services(host, own)
    if not e.hosts()[host].flags & 1:  # it announced (a refresh was due): the next call sends a nil
        e.broadcast_services(host, own)
    h = e.hosts()[host]
    assert h.flags & 1 and h.locked_at(e.round) and h.fifo_head == 0
    return h.nil_pos_bs


def _has(e, view, owner):
    return all(e.slot(view, owner, s) is not None for s in range(e.S))


def bs_nil_blocks_receive(lib, lock_model=1, k=6):
    """Host 1's BroadcastServices looper waits on its nil behind k + 1 jobs (one GetBroadcasts call
    per round at fanout 1). Host 0's announcement reaches host 1 in round 0: with the lock modelled
    it waits in host 1's pipeline, with every other record host 1 receives meanwhile, until the
    receive phase of host 1's first unlocked round, which merges them before that round's packets.
    With lock_model = 0 it merges at once and counts as a locked merge."""
    e = _engine(lib, n_hosts=2, n_services=2, fanout=1, init_mode=INIT_OWN, lock_model=lock_model, **QUIET)
    p = _block_bs(e, 1, k)
    e.send_services(0, [(0, s, e.now()) for s in range(e.S)], 1)
    trace = []
    for r in range(p + 3):
        e.run_rounds(1)
        st = e.stats()
        trace.append((e.round, _has(e, 1, 0), e.hosts()[1].lock_buffered, st["lock_buffered"],
                      st["lock_drained"], st["locked_merges"]))
    if lock_model:
        final = trace[-1][3]
        assert final >= 2
        for rnd, has, nbuf, buffered, drained, _ in trace:
            if rnd <= p + 1:  # rounds 0 .. p ran with host 1 locked
                assert not has and nbuf == buffered and drained == 0, trace
            else:
                assert has and nbuf == 0 and drained == buffered == final, trace
        st = e.stats()
        assert st["locked_merges"] == 0 and st["first_locked_round"] == 0 and st["lock_drops"] == 0
    else:
        assert all(has for _, has, *_ in trace), trace
        assert e.stats()["locked_merges"] >= 2 and e.stats()["first_locked_round"] == 0
    return e


def bt_nil_holds_write_lock(lib, k=8):
    """Host 1's BroadcastTombstones looper blocks on its nil holding the write lock (nothing to
    expire, nothing to tombstone). Its BroadcastServices tick falls due meanwhile and waits: it runs
    at the first owner phase after the nil was taken (round k + 2), not before."""
    e = _engine(lib, n_hosts=2, n_services=2, fanout=1, init_mode=INIT_OWN, alive_interval_rounds=3,
                tombstone_interval_rounds=1000)
    own = [(1, s, e.now()) for s in range(e.S)]
    for _ in range(k):
        e.send_services(1, own, 1)
    e.broadcast_tombstones(1, own)  # both services running: nothing to tombstone -> nil
    h = e.hosts()[1]
    assert h.flags == 2 and h.locked_at(e.round)
    lb0 = h.last_bcast_ns
    for r in range(k + 3):
        e.run_rounds(1)
        h = e.hosts()[1]
        if e.round <= k + 1:  # the nil (position k) is taken in round k
            assert h.last_bcast_ns == lb0 and not (h.flags & 1), (e.round, h.flags)
    assert h.last_bcast_ns > lb0  # BroadcastServices ran once the lock was free
    return e


def push_pull_with_locked_side(lib, lock_model=1, k=6):
    """A push-pull exchange whose side holds the lock does not run (LocalState blocks behind the
    pending writer past memberlist's TCP deadline); the other pair runs. lock_model = 0 runs both
    and counts the merges applied on the locked host."""
    e = _engine(lib, n_hosts=4, n_services=2, fanout=1, init_mode=INIT_OWN, ae_period_rounds=1,
                lock_model=lock_model, **QUIET)
    _block_bs(e, 1, k)
    e.run_rounds(1)
    st = e.stats()
    if lock_model:
        assert st["ae_locked"] == 1 and st["ae_exchanges"] == 1 and st["locked_merges"] == 0, st
        assert not _has(e, 1, 3) and not _has(e, 1, 2) or not _has(e, 1, 0)
    else:
        assert st["ae_locked"] == 0 and st["ae_exchanges"] == 2 and st["locked_merges"] > 0, st
    assert st["first_locked_round"] == 0
    return e


def storm_waits_for_lock(lib, k=6):
    """The departure storm's ExpireServer calls on a locked host wait for the lock: host 1 tombstones
    the other half only at the end of the owner phase of its first unlocked round, at that round's
    now; host 0 does at the storm."""
    e = _engine(lib, n_hosts=4, n_services=2, fanout=1, init_mode=INIT_WARM, storm_round=1, **QUIET)
    p = _block_bs(e, 1, k)
    for r in range(p + 4):
        e.run_rounds(1)
        h1 = e.hosts()[1]
        st = e.stats()
        if 2 <= e.round <= p + 1:
            assert st["expire_deferred"] == 2 and h1.lock & LOCK_PENDING_EXPIRE
            assert e.slot(1, 2, 0)[1] != TOMBSTONE and e.slot(0, 2, 0)[1] == TOMBSTONE
    assert not e.hosts()[1].lock & LOCK_PENDING_EXPIRE
    w = [e.slot(1, o, s) for o in (2, 3) for s in range(e.S)]
    assert all(st_ == TOMBSTONE and ts == e.now(p + 1) for ts, st_ in w), w
    return e


def pipeline_overflow(lib, k=10):
    """A locked host's pipeline holds lock_buffer records; memberlist drops what arrives at a full
    handoff queue. The buffered ones merge at unlock, the dropped ones never."""
    e = _engine(lib, n_hosts=3, n_services=4, fanout=2, init_mode=INIT_OWN, lock_buffer=3, **QUIET)
    _block_bs(e, 1, 2 * k)
    for h in (0, 2):
        for _ in range(3):
            e.send_services(h, [(h, s, e.now()) for s in range(e.S)], 1)
    e.run_rounds(4)
    st = e.stats()
    assert e.hosts()[1].lock_buffered == 3 and st["lock_buffered"] == 3 and st["lock_drops"] > 0, st
    return e


def push_pull_read_locked_side(lib, k=6):
    """gx.h lock_readers: host 1's only lock holder is its blocked BroadcastServices (the read lock)
    and no writer waits (empty pipeline, QUIET loopers), so LocalState's RLock succeeds
    (services_delegate.go:148) and round 0's exchange with host 1 runs. The partner merges host 1's
    state at once. Host 1's merge waits behind the lock: its pool slot holds the partner's state,
    and it merges in host 1's first unlocked round (p + 1). While that merge waits, a writer is
    waiting too, so host 1's later exchanges fail."""
    e = _engine(lib, n_hosts=4, n_services=2, fanout=1, init_mode=INIT_OWN, ae_period_rounds=1, lock_readers=1,
                **QUIET)
    p = _block_bs(e, 1, k)
    e.run_rounds(1)
    st = e.stats()
    assert st["ae_deferred"] == 1 and st["ae_locked"] == 0 and st["ae_exchanges"] == 2, st
    assert e.hosts()[1].lock & LOCK_DEFER_MERGE
    partner = [x for x in (0, 2, 3) if _has(e, x, 1)]
    assert len(partner) == 1, partner  # host 1's state reached its partner only
    x = partner[0]
    assert not _has(e, 1, x)
    while e.round <= p:
        e.run_rounds(1)
        assert not _has(e, 1, x) and e.hosts()[1].lock & LOCK_DEFER_MERGE
    e.run_rounds(1)  # round p + 1: host 1 is unlocked, the waiting merge runs first
    assert _has(e, 1, x) and not e.hosts()[1].lock & LOCK_DEFER_MERGE
    st = e.stats()
    assert st["ae_locked"] >= 1 and st["ae_deferred"] == 1 and st["ae_defer_lost"] == 0, st
    return e


def push_pull_read_locked_writer_waiting(lib, k=6):
    """gx.h lock_readers: host 1 read-locked, but a gossip record from host 0 reached its pipeline
    earlier in the round (ProcessServiceMsgs waits in AddServiceEntry's Lock: a writer is pending),
    so LocalState's RLock waits too and the exchange fails, as it does when BroadcastTombstones holds
    the write lock."""
    e = _engine(lib, n_hosts=2, n_services=2, fanout=1, init_mode=INIT_OWN, ae_period_rounds=1, lock_readers=1,
                **QUIET)
    _block_bs(e, 1, k)
    e.send_services(0, [(0, s, e.now()) for s in range(e.S)], 1)
    e.run_rounds(1)
    st = e.stats()
    assert st["lock_buffered"] > 0 and st["ae_locked"] == 1 and st["ae_deferred"] == 0, st
    w = _engine(lib, n_hosts=2, n_services=2, fanout=1, init_mode=INIT_OWN, ae_period_rounds=1, lock_readers=1,
                **QUIET)
    own = [(1, s, w.now()) for s in range(w.S)]
    for _ in range(k):
        w.send_services(1, own, 1)
    w.broadcast_tombstones(1, own)  # BroadcastTombstones blocks holding the write lock
    w.run_rounds(1)
    st = w.stats()
    assert st["ae_locked"] == 1 and st["ae_deferred"] == 0, st
    return e


def push_pull_read_locked_slot_taken(lib, k=6):
    """gx.h lock_readers with one pool slot: hosts 1 and 2 are both read-locked with no writer
    waiting, so both of round 0's exchanges run, but only the lowest host id keeps its waiting
    merge; host 2's is dropped and counted (ae_defer_lost)."""
    e = _engine(lib, n_hosts=4, n_services=2, fanout=1, init_mode=INIT_OWN, ae_period_rounds=1, lock_readers=1,
                lock_defer_slots=1, **QUIET)
    _block_bs(e, 1, k)
    _block_bs(e, 2, k)
    e.run_rounds(1)
    st = e.stats()
    assert st["ae_deferred"] == 1 and st["ae_defer_lost"] == 1 and st["ae_locked"] == 0, st
    assert e.hosts()[1].lock & LOCK_DEFER_MERGE and not e.hosts()[2].lock & LOCK_DEFER_MERGE
    return e


CASES = {
    "push_pull_read_locked_side": push_pull_read_locked_side,
    "push_pull_read_locked_writer_waiting": push_pull_read_locked_writer_waiting,
    "push_pull_read_locked_slot_taken": push_pull_read_locked_slot_taken,
    "bs_nil_blocks_receive": bs_nil_blocks_receive,
    "bs_nil_blocks_receive_lock_off": lambda lib: bs_nil_blocks_receive(lib, lock_model=0),
    "bt_nil_holds_write_lock": bt_nil_holds_write_lock,
    "push_pull_with_locked_side": push_pull_with_locked_side,
    "push_pull_with_locked_side_lock_off": lambda lib: push_pull_with_locked_side(lib, lock_model=0),
    "storm_waits_for_lock": storm_waits_for_lock,
    "pipeline_overflow": pipeline_overflow,
}

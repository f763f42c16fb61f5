"""The broadcast FIFO's stored window (gx.h gx_job): the reference's queue is unbounded
(services_state.go:94,384-391,581-603, every blocked sender a goroutine), the engine stores the
first queue_cap jobs of each host's queue and counts the rest in place. These tests check on the
CPU oracle that a run with a small window is observably identical to a run whose window never
fills, up to the first LOST dequeue, that the loopers' nils keep their positions behind deferred
jobs, and that the LOST accounting starts exactly where the windows diverge.
"""
import pytest

from sidecar_amd.abi import INIT_OWN, INIT_WARM, JOB_LOST, JOB_SEND, Engine, default_params

IGNORE_STATS = {"queue_deferred", "queue_drops", "first_drop_round", "list_drops"}


def _engines(lib, small_q, big_q, **kw):
    a = Engine(default_params(lib, queue_cap=small_q, **kw), lib=lib)
    b = Engine(default_params(lib, queue_cap=big_q, **kw), lib=lib)
    return a, b


def _same_observables(a, b, what):
    sa, sb = a.stats(), b.stats()
    diff = {k: (sa[k], sb[k]) for k in sa if k not in IGNORE_STATS and sa[k] != sb[k]}
    assert not diff, f"{what}: {diff}"
    assert (a.read_views() == b.read_views()).all(), what
    assert (a.last_changed() == b.last_changed()).all(), what
    for x, y in zip(a.hosts(), b.hosts()):
        for f, _ in x._fields_:
            if f != "fifo_stored":
                assert getattr(x, f) == getattr(y, f), f"{what}: host field {f}"
    for h in range(a.H):
        qa, qb = [j.tup() for j in a.queue(h)], [j.tup() for j in b.queue(h)]
        assert qa == qb[:len(qa)], f"{what}: host {h} stored window is not a prefix of the full queue"
        assert [s.tup() for s in a.sleepers(h)] == [s.tup() for s in b.sleepers(h)], what


@pytest.mark.parametrize("kw", [
    # cold start: push-pull accepts pile up retransmits behind the loopers' nils
    dict(n_hosts=64, n_services=8, init_mode=INIT_OWN, ae_period_rounds=10, churn_ppm=50000, aged_ppm=50000),
    # departure storm: EXPIRE jobs fill the window, then heal and push-pull
    dict(n_hosts=96, n_services=4, init_mode=INIT_WARM, ae_period_rounds=10, partition_start=0,
         partition_end=30, storm_round=3, churn_ppm=20000),
])
def test_window_is_exact_until_first_loss(oracle_lib, kw):
    a, b = _engines(oracle_lib, 96, 1 << 16, **kw)
    deferred_nil = False
    for _ in range(400):
        a.run_rounds(1)
        b.run_rounds(1)
        st = a.stats()
        if st["first_drop_round"] >= 0:
            break
        _same_observables(a, b, f"round {a.round}")
        for h in a.hosts():  # a looper blocked on a nil behind deferred jobs
            if (h.flags & 1 and (h.nil_pos_bs - h.fifo_stored) % (1 << 32) < (h.fifo_tail - h.fifo_stored) % (1 << 32)):
                deferred_nil = True
    st = a.stats()
    assert st["queue_deferred"] > 0, "the window never filled"
    assert b.stats()["queue_deferred"] == 0 and b.stats()["queue_drops"] == 0
    assert deferred_nil, "no looper nil was deferred"
    assert st["first_drop_round"] >= 0, "no deferred job reached the head"
    assert st["queue_drops"] > 0


def test_lost_job_counts_and_nil_positions(oracle_lib):
    """A deferred job that reaches the head is LOST (an empty batch, counted once), a deferred nil
    still unblocks its looper, and the window refills behind the deferred run."""
    e = Engine(default_params(oracle_lib, n_hosts=4, n_services=2, init_mode=INIT_OWN, queue_cap=2), lib=oracle_lib)
    h = 0
    recs = [(1, 0, e.now() + i, 0) for i in range(1, 6)]
    for r in recs:  # 5 foreign accepts -> 5 retransmits: 2 stored, 3 deferred
        e.add_service_entry(h, r)
    hs = e.hosts(h, h + 1)[0]
    assert (hs.fifo_tail - hs.fifo_head, hs.fifo_stored - hs.fifo_head) == (5, 2)
    assert e.stats()["queue_deferred"] == 3
    e.broadcast_services(h, [])  # nothing to send: the looper's nil, deferred at position 5
    hs = e.hosts(h, h + 1)[0]
    assert hs.flags & 1 and hs.nil_pos_bs == hs.fifo_head + 5
    got = [e.get_broadcasts(h, 1) for _ in range(6)]
    assert [len(x or []) for x in got[:2]] == [1, 1]  # the stored retransmits
    assert e.stats()["queue_drops"] == 3 and e.stats()["first_drop_round"] == e.round
    hs = e.hosts(h, h + 1)[0]
    assert not (hs.flags & 1), "the deferred nil did not unblock the looper"
    assert hs.fifo_head == hs.fifo_tail == hs.fifo_stored
    e.add_service_entry(h, (2, 1, e.now() + 9, 0))  # stored again
    assert [j.kind for j in e.queue(h)] == [2] and JOB_LOST == 5


def _list_refs(e, h):
    """SendServices jobs of host h that hold a list (stored window and sleep ring): slot -> length."""
    refs = {}
    for j in list(e.queue(h)) + [s.job for s in e.sleepers(h)]:
        if j.kind == JOB_SEND:
            slot, n = j.c & 0xFFFF, j.c >> 16
            assert slot not in refs, f"two live jobs share list {slot}"
            refs[slot] = n
    return refs


def test_deferred_send_holds_no_list(oracle_lib):
    """A SendServices job queued past the stored window holds no list (gx.h GX_LIST_NONE): queueing
    it must not release the list of a live multi-pass job (slot 0 here), and after the first LOST
    dequeue a new list must not take that slot while its job still sleeps between passes."""
    e = Engine(default_params(oracle_lib, n_hosts=2, n_services=4, fanout=1, init_mode=INIT_OWN, queue_cap=2,
                              list_slots=4, alive_interval_rounds=1000, tombstone_interval_rounds=1000),
               lib=oracle_lib)
    now = e.now()
    a = [(0, s, now + 1000 * s) for s in range(4)]
    e.send_services(0, a, 3)       # stored: list 0, three passes with TOMBSTONE_RETRANSMIT sleeps
    e.send_services(0, a[:1], 1)   # stored: list 1 (the window of 2 is full)
    e.send_services(0, a[1:], 1)   # deferred: no list
    assert [j.c & 0xFFFF for j in e.queue(0)] == [0, 1]
    assert e.hosts()[0].fifo_tail - e.hosts()[0].fifo_head == 3
    before = [x.tup() for x in e.read_list(0, 0)]
    assert len(before) == 4
    for r in range(40):
        e.run_rounds(1)
        if r == 3:  # after the LOST dequeue the window stores again: a new list is allocated
            e.send_services(0, [(0, 0, now + 99_999)], 1)
        refs = _list_refs(e, 0)
        if 0 in refs:
            assert [x.tup() for x in e.read_list(0, 0)] == before, f"round {e.round}: list 0 overwritten"
        for slot, n in refs.items():
            assert len(e.read_list(0, slot)) == n, f"round {e.round}: list {slot}"
    st = e.stats()
    assert st["queue_drops"] >= 1 and st["list_drops"] == 0
    assert not _list_refs(e, 0)  # every pass ran; no list leaked either
    assert all(not e.read_list(0, s) for s in range(4))

"""memberlist failure detection — known-answer cases written against the gx C-ABI.

memberlist is absent from the reference tree (github.com/NinesStack/memberlist
v0.0.0-20170522194404-cfac2b5cf519, go.mod:6, a fork of hashicorp/memberlist), so these cases
restate the published algorithm's own unit tests (hashicorp/memberlist state_test.go,
queue_test.go, suspicion_test.go, util_test.go — named per case) under the engine's round model,
plus the one reference hook on the path: NotifyLeave -> go ExpireServer(node)
(services_delegate.go:173-176). Parity against the fork is unpinned; every case
takes a loaded library, so the same cases pin the CPU oracle (tests/test_fd_cpu.py) and check the
HIP engine (tests/test_gpu_fd.py).
"""
from sidecar_amd.abi import (ALIVE, FD_NO_DEADLINE, FD_NONE, INIT_OWN, INIT_WARM, M_ALIVE, M_DEAD, M_SUSPECT,
                             TOMBSTONE, Engine, default_params)

H = 8
ME, A, B, C, D = 0, 1, 2, 3, 4


def mk(lib, **kw):
    base = dict(n_hosts=H, n_services=4, init_mode=INIT_WARM, fd_enable=1, queue_cap=256)
    base.update(kw)
    return Engine(default_params(lib, **base), lib=lib)


def member(e, host, node):
    m = e.fd_member(host, node)
    return m.state, m.incarnation


def timeouts(e):
    return list(e.params.fd_suspicion_rounds)[: e.params.fd_suspicion_k + 1]


# ------------------------------------------------------------------------ state_test.go ----
def kat_suspect_node(lib):
    """TestMemberList_SuspectNode: an alive node is suspected, the suspicion is re-gossiped, and
    the timer declares it dead after the (unconfirmed) maximum timeout; NotifyLeave then
    ExpireServer()s its records in the host's catalog (services_delegate.go:173-176)."""
    e = mk(lib)
    e.fd_notify(ME, [(M_SUSPECT, A, 0, B)])
    m = e.fd_member(ME, A)
    assert (m.state, m.incarnation, m.change_round) == (M_SUSPECT, 0, 0)
    t0 = timeouts(e)[0]
    assert m.deadline == t0 and e.fd_hosts(ME, ME + 1)[0].min_deadline == t0
    assert e.fd_queue(ME) == [((M_SUSPECT, A, 0, B), 0)]
    e.set_round(t0 - 1)
    e.fd_timers(ME)
    assert member(e, ME, A) == (M_SUSPECT, 0)
    e.set_round(t0)
    e.fd_timers(ME)
    m = e.fd_member(ME, A)
    assert (m.state, m.change_round, m.deadline) == (M_DEAD, t0, FD_NO_DEADLINE)
    assert [q for q, _ in e.fd_queue(ME)][0] == (M_DEAD, A, 0, ME)  # deadNode{From: us}
    now = e.now()
    assert all(e.slot(ME, A, s) == (now, TOMBSTONE) for s in range(4))  # ExpireServer
    st = e.stats()
    assert (st["fd_suspicions"], st["fd_deaths"], st["expire_server"]) == (1, 1, 1)


def kat_suspect_double(lib):
    """TestMemberList_SuspectNode_DoubleSuspect: a second suspicion from the same accuser is not
    a confirmation and is not re-gossiped."""
    e = mk(lib)
    e.fd_notify(ME, [(M_SUSPECT, A, 0, B)])
    e.fd_get_broadcasts(ME, 16)  # the first suspicion went out once
    e.fd_notify(ME, [(M_SUSPECT, A, 0, B)])
    assert e.fd_queue(ME) == [((M_SUSPECT, A, 0, B), 1)]
    assert e.fd_member(ME, A).n_conf == 0 and e.stats()["fd_confirmations"] == 0


def kat_suspect_old(lib):
    """TestMemberList_SuspectNode_OldSuspect: an older incarnation is ignored."""
    e = mk(lib)
    e.fd_notify(ME, [(M_ALIVE, A, 5, A)])
    e.fd_get_broadcasts(ME, 16)
    q0 = e.fd_queue(ME)
    e.fd_notify(ME, [(M_SUSPECT, A, 4, B)])
    assert member(e, ME, A) == (M_ALIVE, 5) and e.fd_queue(ME) == q0


def kat_suspect_refute(lib):
    """TestMemberList_SuspectNode_Refute: a suspicion about ourselves is refuted with a higher
    incarnation (max(own + 1, accused + 1)) broadcast as alive."""
    e = mk(lib)
    e.fd_notify(ME, [(M_SUSPECT, ME, 3, B)])
    assert member(e, ME, ME) == (M_ALIVE, 4)
    assert e.fd_queue(ME) == [((M_ALIVE, ME, 4, ME), 0)]
    e.fd_notify(ME, [(M_SUSPECT, ME, 1, C)])  # older than ours: ignored
    assert member(e, ME, ME) == (M_ALIVE, 4)
    e.fd_notify(ME, [(M_DEAD, ME, 4, C)])  # deadNode about us: refute again
    assert member(e, ME, ME) == (M_ALIVE, 5) and e.stats()["fd_refutes"] == 2


def kat_suspicion_confirmations(lib):
    """suspicion_test.go TestSuspicion_Timer: independent confirmations shrink the timeout from
    max towards min (log(c+1)/log(k+1)); a repeat accuser and confirmations beyond k count for
    nothing; each new confirmation re-gossips the suspicion."""
    e = mk(lib)
    t = timeouts(e)
    assert len(t) == 3 and t[0] > t[1] > t[2]
    e.set_round(10)
    e.fd_notify(ME, [(M_SUSPECT, A, 0, B)])
    assert e.fd_member(ME, A).deadline == 10 + t[0]
    e.set_round(12)
    e.fd_notify(ME, [(M_SUSPECT, A, 0, B), (M_SUSPECT, A, 0, C)])
    m = e.fd_member(ME, A)
    assert (m.n_conf, m.deadline, list(m.susp_from)) == (1, 10 + t[1], [B, C, FD_NONE])
    assert e.fd_queue(ME)[0] == ((M_SUSPECT, A, 0, C), 0)
    e.fd_notify(ME, [(M_SUSPECT, A, 7, D)])  # a higher incarnation still just confirms
    m = e.fd_member(ME, A)
    assert (m.n_conf, m.incarnation, m.deadline) == (2, 0, 10 + t[2])
    e.fd_notify(ME, [(M_SUSPECT, A, 0, 5)])  # k = 2 reached
    assert e.fd_member(ME, A).n_conf == 2 and e.stats()["fd_confirmations"] == 2


def kat_confirm_past_deadline(lib):
    """suspicion.Confirm: a confirmation whose shrunken timeout has already elapsed fires the
    timer (here: at the next timer phase)."""
    e = mk(lib)
    t = timeouts(e)
    e.fd_notify(ME, [(M_SUSPECT, A, 0, B)])
    e.set_round(t[1] + 3)
    e.fd_notify(ME, [(M_SUSPECT, A, 0, C)])
    assert e.fd_member(ME, A).deadline == t[1]
    e.fd_timers(ME)
    assert member(e, ME, A) == (M_DEAD, 0)


def kat_dead_node(lib):
    """TestMemberList_DeadNode / _Double / _OldDead: a dead message is applied once (NotifyLeave
    once), a repeat or an older incarnation is ignored."""
    e = mk(lib)
    e.fd_notify(ME, [(M_ALIVE, A, 2, A)])
    e.fd_notify(ME, [(M_DEAD, A, 1, B)])
    assert member(e, ME, A) == (M_ALIVE, 2)
    e.fd_notify(ME, [(M_DEAD, A, 2, B)])
    assert member(e, ME, A) == (M_DEAD, 2)
    assert e.fd_queue(ME)[0] == ((M_DEAD, A, 2, B), 0)
    e.fd_notify(ME, [(M_DEAD, A, 3, C)])
    assert member(e, ME, A) == (M_DEAD, 2)
    st = e.stats()
    assert (st["fd_deaths"], st["expire_server"]) == (1, 1)


def kat_dead_clears_suspicion(lib):
    """deadNode deletes the node's suspicion timer: the timer does not fire again."""
    e = mk(lib)
    e.fd_notify(ME, [(M_SUSPECT, A, 0, B), (M_DEAD, A, 0, C)])
    m = e.fd_member(ME, A)
    assert (m.state, m.deadline) == (M_DEAD, FD_NO_DEADLINE)
    e.set_round(timeouts(e)[0] + 1)
    e.fd_timers(ME)
    assert e.stats()["fd_deaths"] == 1


def kat_alive_replay_after_dead(lib):
    """TestMemberList_DeadNode_AliveReplay: an alive message with the dead incarnation is ignored;
    a higher incarnation brings the node back (NotifyJoin, which Sidecar only logs)."""
    e = mk(lib)
    e.fd_notify(ME, [(M_DEAD, A, 0, B), (M_ALIVE, A, 0, A)])
    assert member(e, ME, A) == (M_DEAD, 0)
    e.set_round(3)
    e.fd_notify(ME, [(M_ALIVE, A, 1, A)])
    m = e.fd_member(ME, A)
    assert (m.state, m.incarnation, m.change_round) == (M_ALIVE, 1, 3)
    assert e.stats()["fd_alive_updates"] == 1


def kat_alive_clears_suspect(lib):
    """TestMemberList_AliveNode_SuspectNode / _Idempotent: a newer alive clears the suspicion and
    its timer; the same incarnation again changes nothing."""
    e = mk(lib)
    e.set_round(4)
    e.fd_notify(ME, [(M_SUSPECT, A, 0, B), (M_ALIVE, A, 1, A)])
    m = e.fd_member(ME, A)
    assert (m.state, m.incarnation, m.change_round, m.deadline) == (M_ALIVE, 1, 4, FD_NO_DEADLINE)
    assert e.fd_queue(ME)[0] == ((M_ALIVE, A, 1, A), 0)
    e.fd_get_broadcasts(ME, 16)
    q = e.fd_queue(ME)
    e.fd_notify(ME, [(M_ALIVE, A, 1, A)])
    assert e.fd_queue(ME) == q and e.stats()["fd_alive_updates"] == 1
    e.set_round(timeouts(e)[0] + 10)
    e.fd_timers(ME)
    assert member(e, ME, A) == (M_ALIVE, 1)


# ------------------------------------------------------------------------ queue_test.go ----
def kat_queue_order_and_limit(lib):
    """TestTransmitLimited_GetBroadcasts / _Limit / _Invalidate: one queued message per node (a
    newer one replaces it), fewest transmits first and newest first among equals, and every
    message leaves after retransmitLimit = 4 * ceil(log10(n + 1)) transmissions."""
    e = mk(lib)
    L = e.params.fd_retransmit_limit
    assert L == 4 * 1  # n = 8
    e.fd_notify(ME, [(M_ALIVE, A, 1, A), (M_ALIVE, B, 1, B), (M_ALIVE, C, 1, C)])
    assert [q[0][1] for q in e.fd_queue(ME)] == [C, B, A]
    assert [m[1] for m in e.fd_get_broadcasts(ME, 2)] == [C, B]
    assert [(q[0][1], q[1]) for q in e.fd_queue(ME)] == [(A, 0), (C, 1), (B, 1)]
    e.fd_notify(ME, [(M_ALIVE, B, 2, B)])  # invalidates B's queued alive
    assert [(q[0][1], q[0][2], q[1]) for q in e.fd_queue(ME)] == [(B, 2, 0), (A, 1, 0), (C, 1, 1)]
    sent = [e.fd_get_broadcasts(ME, 8) for _ in range(L + 1)]
    assert [len(s) for s in sent] == [3, 3, 3, 2, 0]  # C leaves one call earlier
    assert e.fd_queue(ME) == [] and e.fd_hosts(ME, ME + 1)[0].q_len == 0


# ------------------------------------------------------------------------ probes ----------
def kat_probe_departed(lib):
    """TestMemberList_ProbeNode_Suspect: a node that acks neither directly nor through the
    IndirectChecks relays is suspected by the prober (suspectNode{inc, node, From: us})."""
    e = mk(lib, depart_round=0, depart_ppm=1_000_000 // 4)
    gone = [h for h, x in enumerate(e.fd_hosts()) if x.departed]
    assert gone and ME not in gone  # seed-dependent sanity
    seen = set()
    for _ in range(H - 1):
        t, ack = e.fd_probe(ME)
        seen.add(t)
        assert ack == (t not in gone)
        if t in gone:
            m = e.fd_member(ME, t)
            assert (m.state, list(m.susp_from)[0]) == (M_SUSPECT, ME)
    assert seen == set(range(1, H))  # one pass over the shuffled list visits everyone once
    st = e.stats()
    assert st["fd_probes"] == H - 1 and st["fd_probe_failures"] == len(gone)


def kat_probe_partition_indirect(lib):
    """probeNode across a partition: no relay reaches both sides, so the target is suspected;
    inside the prober's half every probe is acked."""
    e = mk(lib, partition_start=0, partition_end=1000)
    for _ in range(H - 1):
        t, ack = e.fd_probe(ME)
        assert ack == (t < H // 2)
        assert e.fd_member(ME, t).state == (M_ALIVE if t < H // 2 else M_SUSPECT)


def kat_probe_skips_dead_and_reaps(lib):
    """probe() skips dead nodes; resetNodes at the end of a pass reaps nodes dead for longer than
    GossipToTheDeadTime: afterwards suspect/dead messages about them are ignored and an alive
    message re-adds them (aliveNode of an unknown node: dead, incarnation 0, then the update)."""
    e = mk(lib, fd_gossip_dead_rounds=5)
    e.fd_notify(ME, [(M_DEAD, A, 3, B)])
    targets = {e.fd_probe(ME)[0] for _ in range(H - 2)}
    assert A not in targets and len(targets) == H - 2
    e.set_round(20)
    e.fd_probe(ME)  # wraps: resetNodes at round 20 reaps A (dead since round 0)
    h = e.fd_hosts(ME, ME + 1)[0]
    assert (h.probe_pass, h.wrap_round) == (1, 20)
    e.fd_notify(ME, [(M_ALIVE, A, 0, A)])  # incarnation 0 <= re-added 0: still dead
    m = e.fd_member(ME, A)
    assert (m.state, m.incarnation) == (M_DEAD, 0)
    e.fd_notify(ME, [(M_ALIVE, A, 1, A)])
    assert member(e, ME, A) == (M_ALIVE, 1)


def kat_merge_state(lib):
    """TestMemberList_MergeState: pushPull's mergeState applies a remote member list — a newer
    alive incarnation updates, a dead node is only suspected (From: us), an equal incarnation
    changes nothing, unlisted nodes are untouched; a list that calls us dead makes us refute."""
    e = mk(lib)
    e.fd_notify(ME, [(M_ALIVE, A, 1, A), (M_ALIVE, B, 1, B), (M_ALIVE, C, 1, C)])
    remote = [None] * H
    remote[A] = (M_ALIVE, 2)
    remote[B] = (M_DEAD, 1)
    remote[C] = (M_ALIVE, 1)
    remote[D] = (M_ALIVE, 2)
    e.fd_merge_state(ME, remote)
    assert member(e, ME, A) == (M_ALIVE, 2)
    m = e.fd_member(ME, B)
    assert (m.state, m.incarnation, m.susp_from[0]) == (M_SUSPECT, 1, ME)
    assert member(e, ME, C) == (M_ALIVE, 1) and member(e, ME, D) == (M_ALIVE, 2)
    assert member(e, ME, 5) == (M_ALIVE, 0)
    st = e.stats()
    assert (st["fd_state_merges"], st["fd_suspicions"], st["fd_alive_updates"]) == (4, 1, 3 + 2)
    e.fd_merge_state(ME, [None] * ME + [(M_DEAD, 0)] + [None] * (H - ME - 1))
    assert member(e, ME, ME) == (M_ALIVE, 1) and e.stats()["fd_refutes"] == 1


ALL = [kat_suspect_node, kat_merge_state, kat_suspect_double, kat_suspect_old, kat_suspect_refute,
       kat_suspicion_confirmations, kat_confirm_past_deadline, kat_dead_node, kat_dead_clears_suspicion,
       kat_alive_replay_after_dead, kat_alive_clears_suspect, kat_queue_order_and_limit,
       kat_probe_departed, kat_probe_partition_indirect, kat_probe_skips_dead_and_reaps]


# -------------------------------------------------------------------- round-model scenarios --
# (name, params, rounds): run by the oracle-invariant tests (CPU) and the GPU parity tests.
SCENARIOS = {
    "depart10": (dict(n_hosts=64, n_services=8, init_mode=INIT_WARM, fd_enable=1, depart_round=5,
                      depart_ppm=100_000, ae_period_rounds=10, queue_cap=4096), 300),
    "partition_heal": (dict(n_hosts=64, n_services=8, init_mode=INIT_WARM, fd_enable=1, partition_start=0,
                            partition_end=40, ae_period_rounds=10, queue_cap=4096), 260),
    "partition_long": (dict(n_hosts=48, n_services=4, init_mode=INIT_WARM, fd_enable=1, partition_start=0,
                            partition_end=400, ae_period_rounds=10, queue_cap=4096), 500),
    "churn_depart_bytes": (dict(n_hosts=96, n_services=8, init_mode=INIT_OWN, fd_enable=1, depart_round=20,
                                depart_ppm=50_000, churn_ppm=20_000, limit_bytes=1398, overhead_bytes=3,
                                packet_cap=48, ae_period_rounds=10, queue_cap=4096), 250),
    "depart_no_fd": (dict(n_hosts=64, n_services=8, init_mode=INIT_WARM, depart_round=5, depart_ppm=100_000,
                          ae_period_rounds=10, queue_cap=4096), 200),
    # GossipMessages with the detector: each of a target's gathers takes memberlist's queue first
    "partition_heal_gm15": (dict(n_hosts=64, n_services=8, init_mode=INIT_WARM, fd_enable=1, partition_start=0,
                                 partition_end=40, ae_period_rounds=10, queue_cap=4096, gossip_messages=15), 260),
    "depart_bytes_gm4": (dict(n_hosts=80, n_services=8, init_mode=INIT_OWN, fd_enable=1, depart_round=10,
                              depart_ppm=60_000, churn_ppm=20_000, limit_bytes=1398, overhead_bytes=3,
                              packet_cap=48, ae_period_rounds=10, queue_cap=4096, gossip_messages=4), 220),
    # the packets' memberlist messages walked in key order through overflowed inboxes
    "depart_inbox_overflow": (dict(n_hosts=64, n_services=8, init_mode=INIT_WARM, fd_enable=1, depart_round=5,
                                   depart_ppm=100_000, ae_period_rounds=10, queue_cap=4096, fanout=6,
                                   inbox_slots=2), 200),
}

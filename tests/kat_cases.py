"""Known-answer tests restated from the reference's own Go tests, written against the gx C-ABI.

Each case cites the reference test it restates (paths relative to the reference root). Every
case takes a loaded library exporting include/gx.h, so the same cases pin the CPU oracle
(tests/test_oracle_kat.py) and check the HIP engine (tests/test_gpu_kat.py).

Host-name interning used throughout: LOCAL = the machine's own hostname (state.Hostname after
NewServicesState()), SH = "shakespeare", CH = "chaucer"; docker1/docker2 for the delegate
fixtures. The simulated clock replaces time.Now(): "time passes" is a round advance.
"""
import datetime as _dt

from sidecar_amd.abi import (ALIVE, DRAINING, Engine, JOB_NIL_BS, JOB_RETX, JOB_SEND, TOMBSTONE,
                             UNHEALTHY, UNKNOWN, default_params)

LOCAL, SH, CH, OTHER, OTHER2, DOCKER1, DOCKER2 = 0, 1, 2, 3, 4, 5, 6
SEC = 10**9
MIN = 60 * SEC
HOUR = 60 * MIN
T0 = 1_700_000_000 * SEC  # a whole second, like baseTime.Round(time.Second)
TOMBSTONE_LIFESPAN = 3 * HOUR
ALIVE_LIFESPAN = 80 * SEC
DRAINING_LIFESPAN = 10 * MIN


def mk(lib, **kw):
    p = default_params(lib, n_hosts=8, n_services=8, t0_ns=T0, retransmit_rounds=0,
                       queue_cap=64, list_slots=8)
    for k, v in kw.items():
        setattr(p, k, v)
    return Engine(p, lib=lib)


def tup(s):
    return (s.host, s.svc, s.updated_ns, s.status)


# ----------------------------------------------------------------- catalog/services_state_test.go
def kat_add_merges_new(lib):
    """services_state_test.go:126-133 — AddServiceEntry merges in a new service."""
    e = mk(lib)
    assert e.local_state(LOCAL) == []
    e.add_service_entry(LOCAL, (CH, 0, T0, ALIVE))
    assert e.slot(LOCAL, CH, 0) == (T0, ALIVE)


def kat_older_update_ignored(lib):
    """services_state_test.go:135-155 — an update older than what we have is not merged."""
    e = mk(lib)
    e.add_service_entry(LOCAL, (CH, 0, T0, ALIVE))
    assert e.add_service_entry(LOCAL, (CH, 0, T0 - MIN, ALIVE)) == 0
    assert e.slot(LOCAL, CH, 0) == (T0, ALIVE)


def kat_stale_dropped(lib):
    """services_state_test.go:157-175 — a record older than now-3h-1min is dropped and no server
    is created. The reference reads time.Now() again inside IsStale, so the record is strictly
    older than the cut-off; restated by letting one round pass. service.go:68-72 is strict."""
    e = mk(lib)
    base = e.now()
    e.set_round(1)
    assert e.add_service_entry(LOCAL, (CH, 0, base - MIN - TOMBSTONE_LIFESPAN, ALIVE)) == 0
    assert all(e.slot(LOCAL, CH, s) is None for s in range(e.S))
    assert e.stats()["stale_drops"] == 1
    # boundary: exactly at the cut-off is not Before() it -> accepted
    now = e.now()
    assert e.add_service_entry(LOCAL, (CH, 1, now - MIN - TOMBSTONE_LIFESPAN, ALIVE)) == 1


def kat_updates_timestamp(lib):
    """services_state_test.go:177-183 — a newer record replaces the stored Updated."""
    e = mk(lib)
    e.add_service_entry(LOCAL, (CH, 0, T0, ALIVE))
    nd = T0 + 5 * 24 * HOUR
    e.add_service_entry(LOCAL, (CH, 0, nd, ALIVE))
    assert e.slot(LOCAL, CH, 0) == (nd, ALIVE)


def kat_retransmit_on_change(lib):
    """services_state_test.go:214-225 — an accepted foreign change is retransmitted exactly once,
    as the stored record."""
    e = mk(lib)
    e.add_service_entry(LOCAL, (CH, 0, T0, ALIVE))
    q = e.queue(LOCAL)
    assert len(q) == 1 and q[0].kind == JOB_RETX
    first = e.get_broadcasts(LOCAL)  # catch the retransmit from the initial add
    assert [tup(s) for s in first] == [(CH, 0, T0, ALIVE)]
    e.set_round(1)
    ts = e.now()  # svc.Tombstone(): Updated = now
    e.add_service_entry(LOCAL, (CH, 0, ts, TOMBSTONE))
    pkt = e.get_broadcasts(LOCAL)
    assert len(pkt) == 1 and tup(pkt[0]) == (CH, 0, ts, TOMBSTONE)
    assert e.get_broadcasts(LOCAL) is None


def kat_no_retransmit_own(lib):
    """services_state_test.go:227-243 — adding a service of this host is not retransmitted."""
    e = mk(lib)
    e.add_service_entry(SH, (SH, 0, T0, ALIVE))
    assert e.queue(SH) == []
    assert e.get_broadcasts(SH) is None


def kat_sets_draining(lib):
    """services_state_test.go:245-256 — ALIVE -> DRAINING applies."""
    e = mk(lib)
    e.add_service_entry(LOCAL, (CH, 0, T0, ALIVE))
    e.set_round(1)
    e.add_service_entry(LOCAL, (CH, 0, e.now(), DRAINING))
    assert e.slot(LOCAL, CH, 0)[1] == DRAINING


def kat_draining_sticky(lib):
    """services_state_test.go:258-270 — a newer ALIVE does not overwrite DRAINING
    (services_state.go:329-331); the timestamp still advances."""
    e = mk(lib)
    e.add_service_entry(LOCAL, (CH, 0, T0, DRAINING))
    e.set_round(1)
    e.add_service_entry(LOCAL, (CH, 0, e.now(), ALIVE))
    assert e.slot(LOCAL, CH, 0) == (e.now(), DRAINING)


def kat_merge(lib):
    """services_state_test.go:299-308 — Merge() brings another state's servers in."""
    e = mk(lib)
    e.add_service_entry(OTHER, (CH, 0, T0, ALIVE))
    e.merge(OTHER2, OTHER)
    assert [s.tup() for s in e.local_state(OTHER2)] == [s.tup() for s in e.local_state(OTHER)]


# Test_TrackingAndBroadcasting: state.Hostname = shakespeare, tombstoneRetransmit = 1ns
def _tb(lib):
    e = mk(lib)
    s1 = (SH, 0, T0, ALIVE)
    s2 = (SH, 1, T0, ALIVE)
    return e, s1, s2


def kat_send_services_count(lib):
    """services_state_test.go:345-353 — SendServices with a 5-pass looper emits 5 batches;
    :402-424 — each pass adds 50ns to Updated."""
    e, s1, s2 = _tb(lib)
    e.send_services(SH, [s1, s2], 5)
    for p in range(5):
        b = e.get_broadcasts(SH)
        assert [tup(x) for x in b] == [(SH, 0, T0 + 50 * p, ALIVE), (SH, 1, T0 + 50 * p, ALIVE)]
    assert e.get_broadcasts(SH) is None


def kat_track_new_services(lib):
    """services_state_test.go:355-366 — tracked local services are added to state."""
    e, s1, s2 = _tb(lib)
    e.add_service_entries([SH, SH], [s1, s2])
    assert e.slot(SH, SH, 0) == (T0, ALIVE) and e.slot(SH, SH, 1) == (T0, ALIVE)


def kat_broadcast_new_in_order(lib):
    """services_state_test.go:368-378 — BroadcastServices serialises new services in order."""
    e, s1, s2 = _tb(lib)
    e.broadcast_services(SH, [s1, s2])
    q = e.queue(SH)
    assert len(q) == 1 and q[0].kind == JOB_SEND and q[0].n_passes == 5  # ALIVE_COUNT: new
    b = e.get_broadcasts(SH)
    assert [tup(x) for x in b] == [s1[:2] + (T0, ALIVE), s2[:2] + (T0, ALIVE)]


def kat_broadcast_nil_when_idle(lib):
    """services_state_test.go:380-386 — a nil batch when there are no services."""
    e, s1, s2 = _tb(lib)
    e.broadcast_services(SH, [])
    q = e.queue(SH)
    assert len(q) == 1 and q[0].kind == JOB_NIL_BS
    assert e.hosts(SH, SH + 1)[0].flags & 1  # the looper is blocked on its nil send
    assert e.get_broadcasts(SH) is None
    assert e.queue(SH) == [] and not (e.hosts(SH, SH + 1)[0].flags & 1)


def kat_tombstones_serialized(lib):
    """services_state_test.go:388-400 — an own service missing from discovery is tombstoned and
    emitted twice with Status 1."""
    e, s1, s2 = _tb(lib)
    junk = (SH, 2, T0, ALIVE)
    e.add_service_entries([SH, SH, SH], [junk, s1, s2])
    e.broadcast_tombstones(SH, [s1, s2])
    b = e.get_broadcasts(SH)
    assert len(b) == 2
    assert all((x.host, x.svc, x.status) == (SH, 2, TOMBSTONE) for x in b)


def kat_alive_not_tombstoned(lib):
    """services_state_test.go:437-444 — services still alive are not tombstoned (empty batch)."""
    e, s1, s2 = _tb(lib)
    e.add_service_entries([SH, SH], [s1, s2])
    e.broadcast_tombstones(SH, [s1, s2])
    assert e.get_broadcasts(SH) is None
    assert e.slot(SH, SH, 0) == (T0, ALIVE)


def kat_nil_when_no_tombstones(lib):
    """services_state_test.go:446-452 — nil into the channel when no tombstones."""
    e, s1, s2 = _tb(lib)
    e.broadcast_tombstones(SH, [])
    assert e.get_broadcasts(SH) is None
    assert e.stats()["nil_batches"] == 1


def kat_last_tombstone_gc(lib):
    """services_state_test.go:467-478 — when the last tombstone expires the server goes away."""
    e, s1, s2 = _tb(lib)
    e.add_service_entry(SH, s1)
    e.write_slot(SH, (SH, 0, T0 - TOMBSTONE_LIFESPAN - MIN, TOMBSTONE))
    e.tombstone_others(SH)
    assert all(e.slot(SH, SH, s) is None for s in range(e.S))


def kat_alive_lifespan(lib):
    """services_state_test.go:480-492 — alive services are tombstoned at Updated+1s after
    ALIVE_LIFESPAN."""
    e, s1, s2 = _tb(lib)
    e.add_service_entry(SH, s1)
    stamp = T0 - ALIVE_LIFESPAN - 5 * SEC
    e.write_slot(SH, (SH, 0, stamp, ALIVE))
    out, n = e.tombstone_others(SH)
    assert n == 1 and tup(out[0]) == (SH, 0, stamp + SEC, TOMBSTONE)
    assert e.slot(SH, SH, 0) == (stamp + SEC, TOMBSTONE)


def kat_draining_lifespan(lib):
    """services_state_test.go:494-507 — draining services expire after DRAINING_LIFESPAN."""
    e, s1, s2 = _tb(lib)
    e.add_service_entry(SH, (SH, 0, T0, DRAINING))
    stamp = T0 - DRAINING_LIFESPAN - 5 * SEC
    e.write_slot(SH, (SH, 0, stamp, DRAINING))
    e.tombstone_others(SH)
    assert e.slot(SH, SH, 0) == (stamp + SEC, TOMBSTONE)


def kat_draining_survives_alive_lifespan(lib):
    """services_state_test.go:509-522 — draining services outlive ALIVE_LIFESPAN."""
    e, s1, s2 = _tb(lib)
    e.add_service_entry(SH, (SH, 0, T0, DRAINING))
    stamp = T0 - ALIVE_LIFESPAN - 5 * SEC
    e.write_slot(SH, (SH, 0, stamp, DRAINING))
    e.tombstone_others(SH)
    assert e.slot(SH, SH, 0) == (stamp, DRAINING)


def kat_unhealthy_unknown_lifespan(lib):
    """services_state_test.go:524-541 — UNHEALTHY and UNKNOWN use the alive lifespan."""
    e, s1, s2 = _tb(lib)
    e.add_service_entries([SH, SH], [(SH, 3, T0, UNHEALTHY), (SH, 4, T0, UNKNOWN)])
    stamp = T0 - ALIVE_LIFESPAN - 5 * SEC
    e.write_slot(SH, (SH, 3, stamp, UNHEALTHY))
    e.write_slot(SH, (SH, 4, stamp, UNKNOWN))
    e.tombstone_others(SH)
    assert e.slot(SH, SH, 3)[1] == TOMBSTONE and e.slot(SH, SH, 4)[1] == TOMBSTONE


def kat_tombstones_not_retombstoned(lib):
    """services_state_test.go:543-550 — tombstones aren't re-tombstoned."""
    e, s1, s2 = _tb(lib)
    e.add_service_entry(SH, (SH, 5, T0, TOMBSTONE))
    out, n = e.tombstone_others(SH)
    assert n == 0 and out == []


def kat_is_new_service(lib):
    """services_state_test.go:552-559 — a status change makes a service new."""
    e, s1, s2 = _tb(lib)
    e.add_service_entry(SH, (SH, 0, T0, UNHEALTHY))
    assert e.is_new_service(SH, (SH, 0, T0, ALIVE))


def kat_tombstone_not_new(lib):
    """services_state_test.go:561-568 — tombstones are not called new services."""
    e, s1, s2 = _tb(lib)
    e.add_service_entry(SH, (SH, 0, T0, UNHEALTHY))
    assert not e.is_new_service(SH, (SH, 0, T0, TOMBSTONE))


# Test_ClusterMembershipManagement
def kat_expire_server_tombstones_all(lib):
    """services_state_test.go:691-714 — ExpireServer tombstones all services of the host and
    announces them (2 records, Status 1)."""
    e = mk(lib)
    e.add_service_entries([SH, SH], [(SH, 0, T0, ALIVE), (SH, 1, T0, ALIVE)])
    assert e.expire_server(SH, SH)
    b = e.get_broadcasts(SH)
    assert len(b) == 2 and all(x.status == TOMBSTONE and x.updated_ns == T0 for x in b)
    assert e.slot(SH, SH, 0) == (T0, TOMBSTONE) and e.slot(SH, SH, 1) == (T0, TOMBSTONE)
    # TOMBSTONE_COUNT passes, each +50ns
    n = 1
    while e.get_broadcasts(SH) is not None:
        n += 1
    assert n == 10


def kat_expire_server_no_services(lib):
    """services_state_test.go:716-720 — no announcement for a host with no services."""
    e = mk(lib)
    assert not e.expire_server(SH, SH)
    assert e.queue(SH) == []


def kat_expire_server_only_tombstones(lib):
    """services_state_test.go:722-729 — no announcement for a host with no live services."""
    e = mk(lib)
    e.add_service_entry(SH, (SH, 0, T0, TOMBSTONE))
    assert not e.expire_server(SH, SH)
    assert len(e.local_state(SH)) == 1 and e.queue(SH) == []


# ------------------------------------------------------------------------ service/service_test.go
def kat_is_stale(lib):
    """service/service_test.go:142-159 — IsStale: with a 1h lifespan, now-1h-2min is stale; with
    a 62min lifespan, now-1h is not."""
    e = mk(lib, tombstone_lifespan_ns=HOUR)
    now = e.now()
    assert e.add_service_entry(LOCAL, (CH, 0, now - HOUR - 2 * MIN, ALIVE)) == 0
    e2 = mk(lib, tombstone_lifespan_ns=62 * MIN)
    assert e2.add_service_entry(LOCAL, (CH, 0, now - HOUR, ALIVE)) == 1


# ------------------------------------------- change bookkeeping and listeners
def _times(e, view, owner):
    lu, lc = e.server_times(view, owner, owner + 1)[0]
    return int(lu), int(lc)


def kat_new_server_times_epoch(lib):
    """services_state_test.go:53-61, :74-77 — NewServer and NewServicesState start LastUpdated and
    LastChanged at time.Unix(0, 0)."""
    e = mk(lib)
    assert _times(e, LOCAL, CH) == (0, 0)
    assert int(e.last_changed(LOCAL, LOCAL + 1)[0]) == 0


def kat_last_updated_newer_record(lib):
    """services_state_test.go:177-183 — a newer record sets the server's LastUpdated to its Updated."""
    e = mk(lib)
    e.add_service_entry(LOCAL, (CH, 0, T0, ALIVE))
    nd = T0 + 5 * 24 * HOUR  # svc.Updated.AddDate(0, 0, 5)
    e.add_service_entry(LOCAL, (CH, 0, nd, ALIVE))
    assert _times(e, LOCAL, CH)[0] == nd


def kat_last_changed_on_new(lib):
    """services_state_test.go:185-194 — a new service moves state.LastChanged and the server's."""
    e = mk(lib)
    before = int(e.last_changed(LOCAL, LOCAL + 1)[0])
    e.add_service_entry(LOCAL, (CH, 0, T0, ALIVE))
    assert int(e.last_changed(LOCAL, LOCAL + 1)[0]) > before
    assert _times(e, LOCAL, CH)[1] > before
    assert _times(e, LOCAL, CH) == (T0, T0)


def kat_last_changed_on_status_change(lib):
    """services_state_test.go:196-203 — a status change (svc.Tombstone()) moves state.LastChanged."""
    e = mk(lib)
    e.add_service_entry(LOCAL, (CH, 0, T0, ALIVE))
    before = int(e.last_changed(LOCAL, LOCAL + 1)[0])
    e.set_round(1)
    e.add_service_entry(LOCAL, (CH, 0, e.now(), TOMBSTONE))
    assert int(e.last_changed(LOCAL, LOCAL + 1)[0]) > before


def kat_last_changed_skips_same_status(lib):
    """services_state_test.go:205-212 — a newer record with the same status leaves
    state.LastChanged (and the server's LastChanged) alone; LastUpdated still moves."""
    e = mk(lib)
    e.add_service_entry(LOCAL, (CH, 0, T0, ALIVE))
    before = int(e.last_changed(LOCAL, LOCAL + 1)[0])
    e.set_round(1)
    e.add_service_entry(LOCAL, (CH, 0, e.now(), ALIVE))
    assert int(e.last_changed(LOCAL, LOCAL + 1)[0]) == before
    assert _times(e, LOCAL, CH) == (e.now(), T0)


def kat_last_changed_draining_sticky(lib):
    """services_state.go:329-340 — a newer ALIVE over DRAINING is stored as DRAINING: no status
    change, so only LastUpdated moves."""
    e = mk(lib)
    e.add_service_entry(LOCAL, (CH, 0, T0, DRAINING))
    e.set_round(1)
    e.add_service_entry(LOCAL, (CH, 0, e.now(), ALIVE))
    assert _times(e, LOCAL, CH) == (e.now(), T0)
    assert e.stats()["change_events"] == 1


def kat_last_changed_when_tombstoned(lib):
    """services_state_test.go:426-435 — BroadcastTombstones tombstoning a service that stopped
    running moves state.LastChanged and the server's LastChanged."""
    e = mk(lib)
    e.add_service_entry(SH, (SH, 5, T0, ALIVE))  # "runs": not in the container list
    before = int(e.last_changed(SH, SH + 1)[0])
    e.set_round(1)
    out = e.tombstone_services(SH, running=[])
    assert len(out) == 2
    assert int(e.last_changed(SH, SH + 1)[0]) > before and _times(e, SH, SH)[1] > before
    assert _times(e, SH, SH) == (e.now(), e.now())


def kat_last_changed_on_expiry(lib):
    """services_state_test.go:480-492, :494-507 — lifespan expiry tombstones at Updated + 1 s and
    moves the server's LastChanged (to that time)."""
    e, s1, s2 = _tb(lib)
    e.add_service_entry(SH, s1)
    e.add_service_entry(SH, (SH, 1, T0, DRAINING))
    stamp = T0 - ALIVE_LIFESPAN - 5 * SEC
    e.write_slot(SH, (SH, 0, stamp, ALIVE))
    e.write_slot(SH, (SH, 1, T0 - DRAINING_LIFESPAN - 5 * SEC, DRAINING))
    e.tombstone_others(SH)
    # key order: service 1's expiry is the later change
    t1 = T0 - DRAINING_LIFESPAN - 5 * SEC + SEC
    assert _times(e, SH, SH) == (t1, t1)
    assert int(e.last_changed(SH, SH + 1)[0]) == t1


def kat_expire_server_times(lib):
    """services_state.go:176-181 — ExpireServer tombstones every record at now and ServiceChanged
    runs for each, including existing tombstones."""
    e = mk(lib)
    e.add_service_entries([LOCAL] * 3, [(CH, 0, T0, ALIVE), (CH, 1, T0, TOMBSTONE), (CH, 2, T0, DRAINING)])
    n0 = e.stats()["change_events"]
    e.set_round(3)
    assert e.expire_server(LOCAL, CH) == 1
    assert e.stats()["change_events"] - n0 == 3
    assert _times(e, LOCAL, CH) == (e.now(), e.now())


def kat_listener_receives_changes(lib):
    """services_state_test.go:609-626 — a major state change notifies every listener; the event
    carries the record, the previous status (UNKNOWN for a new one) and state.LastChanged."""
    e = mk(lib)
    e.add_listener(LOCAL, 1, 4)
    e.add_listener(LOCAL, 2, 4)
    e.add_service_entry(LOCAL, (LOCAL, 0, T0, ALIVE))
    e.add_service_entry(LOCAL, (LOCAL, 0, T0 + SEC, ALIVE))  # newer, same status: no event
    e.add_service_entry(LOCAL, (LOCAL, 0, T0 + 2 * SEC, TOMBSTONE))
    for lid in (1, 2):
        ev = [x.tup() for x in e.drain_listener(LOCAL, lid)]
        assert ev == [(LOCAL, 0, T0, ALIVE, UNKNOWN, T0),
                      (LOCAL, 0, T0 + 2 * SEC, TOMBSTONE, ALIVE, T0 + 2 * SEC)]
    assert e.drain_listener(LOCAL, 1) == []


def kat_listener_full_channel_drops(lib):
    """services_state.go:230-236 — a full channel does not block: the event is dropped for that
    listener only."""
    e = mk(lib)
    e.add_listener(LOCAL, 1, 1)
    e.add_listener(LOCAL, 2, 3)
    e.add_service_entries([LOCAL] * 3, [(CH, s, T0, ALIVE) for s in range(3)])
    assert [x.service.svc for x in e.drain_listener(LOCAL, 1)] == [0]
    assert [x.service.svc for x in e.drain_listener(LOCAL, 2)] == [0, 1, 2]
    assert e.stats()["listener_drops"] == 2


def kat_listener_add_remove(lib):
    """services_state_test.go:581-605 — AddListener refuses an unbuffered channel; RemoveListener
    removes by name and reports a missing one."""
    from sidecar_amd.abi import GX_EINVAL, GX_ENOENT
    e = mk(lib)
    assert lib.gx_add_listener(e.h, LOCAL, 9, 0) == GX_EINVAL
    e.add_listener(LOCAL, 1, 2)
    assert e.remove_listener(LOCAL, 1) == 0
    assert e.remove_listener(LOCAL, 1) == GX_ENOENT
    e.add_service_entry(LOCAL, (CH, 0, T0, ALIVE))
    assert e.stats()["listener_drops"] == 0


def kat_listener_other_views_silent(lib):
    """Listeners are per ServicesState: a change in another view does not reach them."""
    e = mk(lib)
    e.add_listener(LOCAL, 1, 8)
    e.add_service_entry(SH, (CH, 0, T0, ALIVE))
    assert e.drain_listener(LOCAL, 1) == [] and e.stats()["change_events"] == 1


# ---------------------------------------------------------------------- services_delegate_test.go
# Fixture records (services_delegate_test.go:15-20): byte lengths drive packPacket.
_FIX = {
    "d419": '{"ID":"d419fa7ad1a7","Name":"/dockercon-6adfe629eebc91","Image":"nginx:latest","Created":"2015-02-25T19:04:46Z","Hostname":"docker2","Ports":[{"Type":"tcp","Port":10234}],"Updated":"2015-03-04T01:12:46.669648453Z","Status":0}',
    "dead": '{"ID":"deadbeefabba","Name":"/dockercon-6c01869525db08","Image":"nginx:latest","Created":"2015-02-25T19:04:46Z","Hostname":"docker2","Ports":[{"Type":"tcp","Port":10234}],"Updated":"2015-03-04T01:12:46.669648453Z","Status":0}',
    "1b32": '{"ID":"1b3295bf300f","Name":"/romantic_brown","Image":"0415448f2cc2","Created":"2014-10-02T23:58:48Z","Hostname":"docker1","Ports":[{"Type":"tcp","Port":9494}],"Updated":"2015-03-04T01:12:32.630357657Z","Status":0}',
}


def _ns(iso):
    head, frac = iso.rstrip("Z").split(".")
    d = _dt.datetime.strptime(head, "%Y-%m-%dT%H:%M:%S").replace(tzinfo=_dt.timezone.utc)
    return int(d.timestamp()) * SEC + int(frac.ljust(9, "0"))


_T46 = _ns("2015-03-04T01:12:46.669648453Z")
_T32 = _ns("2015-03-04T01:12:32.630357657Z")
BCAST = [(DOCKER2, 0, _T46, ALIVE), (DOCKER2, 1, _T46, ALIVE)]
BCAST2 = [(DOCKER1, 0, _T32, ALIVE), (DOCKER2, 1, _T46, ALIVE)]
_SIZE = {BCAST[0]: len(_FIX["d419"]), BCAST[1]: len(_FIX["dead"]), BCAST2[0]: len(_FIX["1b32"])}


def records_fitting(queue, limit, overhead=3):
    """packPacket (services_delegate.go:186-223) over byte sizes -> the record limit to pass."""
    total = n = 0
    for rec in queue:
        if total + _SIZE[rec] + overhead > limit:
            break
        total += _SIZE[rec] + overhead
        n += 1
    return n


def _delegate(lib):
    return mk(lib, n_hosts=8, t0_ns=_T46 + 10 * SEC)


def _set_pending(e, host, recs):
    """delegate.pendingBroadcasts = recs, restated through the API: a batch that does not fit."""
    e.send_services(host, recs, 1)
    assert e.get_broadcasts(host, limit=0) is None
    assert [tup(x) for x in e.pending(host)] == [(h, s, t, st) for h, s, t, st in recs]


def kat_getbroadcasts_nothing(lib):
    """services_delegate_test.go:41-43 — nil when there is nothing to send."""
    e = _delegate(lib)
    assert e.get_broadcasts(LOCAL, limit=records_fitting([], 1398)) is None


def kat_getbroadcasts_pending_only(lib):
    """services_delegate_test.go:45-52 — returns from the pending list when nothing is new."""
    e = _delegate(lib)
    _set_pending(e, LOCAL, [BCAST[0]])
    r = e.get_broadcasts(LOCAL, limit=records_fitting([BCAST[0]], 1398))
    assert [tup(x) for x in r] == [BCAST[0]]


def kat_getbroadcasts_channel(lib):
    """services_delegate_test.go:54-63 — returns what's in the channel."""
    e = _delegate(lib)
    e.send_services(LOCAL, BCAST, 1)
    r = e.get_broadcasts(LOCAL, limit=records_fitting(BCAST, 1398))
    assert [tup(x) for x in r] == BCAST and e.pending(LOCAL) == []


def kat_getbroadcasts_leftover(lib):
    """services_delegate_test.go:65-73 — returns what's left when nothing is new."""
    e = _delegate(lib)
    _set_pending(e, LOCAL, BCAST)
    r = e.get_broadcasts(LOCAL, limit=records_fitting(BCAST, 1398))
    assert [tup(x) for x in r] == BCAST and e.pending(LOCAL) == []


def kat_getbroadcasts_new_and_left(lib):
    """services_delegate_test.go:75-86 — what's new first, then what's left, when it fits."""
    e = _delegate(lib)
    _set_pending(e, LOCAL, BCAST)
    e.send_services(LOCAL, BCAST2, 1)
    r = e.get_broadcasts(LOCAL, limit=records_fitting(BCAST2 + BCAST, 1398))
    assert [tup(x) for x in r] == BCAST2 + BCAST and e.pending(LOCAL) == []


def kat_getbroadcasts_many_runs(lib):
    """services_delegate_test.go:88-103 — many runs with leftovers (limits 100/300/100/1398)."""
    e = _delegate(lib)
    _set_pending(e, LOCAL, BCAST)
    e.send_services(LOCAL, BCAST2 + BCAST, 1)
    queue = BCAST2 + BCAST + BCAST
    assert e.get_broadcasts(LOCAL, limit=records_fitting(queue, 100)) is None
    r = e.get_broadcasts(LOCAL, limit=records_fitting(queue, 300))  # 1 message fits here
    assert [tup(x) for x in r] == [BCAST2[0]]
    queue = queue[1:]
    assert e.get_broadcasts(LOCAL, limit=records_fitting(queue, 100)) is None
    r = e.get_broadcasts(LOCAL, limit=records_fitting(queue, 1398))
    assert len(r) == 5
    assert [tup(x) for x in r][:3] == BCAST2[1:] + BCAST
    assert e.pending(LOCAL) == []


# ---- the same delegate tests with packPacket's byte limit computed by the engine
def go_rfc3339nano(ts):
    """time.Time.UTC().Format(time.RFC3339Nano) for the parity tests, independent of the engine."""
    sec, frac = divmod(int(ts), SEC)
    s = _dt.datetime.fromtimestamp(sec, tz=_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%S")
    if frac:
        s += "." + f"{frac:09d}".rstrip("0")
    return s + "Z"


def _fixture_static(doc):
    """len(doc) minus the bytes of its Updated value (quoted) and its Status digits."""
    upd = doc.split('"Updated":', 1)[1].split(",", 1)[0]
    status = doc.rsplit('"Status":', 1)[1].rstrip("}")
    return len(doc) - len(upd) - len(status)


def _delegate_bytes(lib):
    e = _delegate(lib)
    tbl = {(DOCKER2, 0): _FIX["d419"], (DOCKER2, 1): _FIX["dead"], (DOCKER1, 0): _FIX["1b32"]}
    for host in (DOCKER1, DOCKER2):
        row = [0] * e.S
        for (h, j), doc in tbl.items():
            if h == host:
                row[j] = _fixture_static(doc)
        e.set_static_bytes(host, host + 1, row)
    # the engine's len(svc.Encode()) reproduces the fixture lengths 225 / 225 / 214
    assert e.message_bytes(BCAST + BCAST2[:1]) == [len(_FIX["d419"]), len(_FIX["dead"]), len(_FIX["1b32"])]
    return e


def kat_message_bytes_rfc3339nano(lib):
    """service_ffjson.go:370-436 — Updated is encoded by time.Time.MarshalJSON (RFC3339Nano, UTC,
    trailing fractional zeros trimmed); Status in decimal. Static bytes 0 isolate those two."""
    e = mk(lib)
    e.set_static_bytes(0, e.H, [0] * (e.H * e.S))
    ts = [T0, T0 + 1, T0 + 10, T0 + 50, T0 + 100, T0 + 120_000_000, T0 + 999_999_999, T0 + SEC,
          _T46, _T32, _T46 + 50, _T46 + 4 * 50, T0 - 3 * HOUR - MIN, T0 + 1_000_000]
    # across the engine's whole time window (gx.h GX_TS_SHIFT; the epoch is whole seconds)
    E = e.epoch
    ts += [E + 1, E + 86_399 * SEC + 500_000_000, E + 2**60 + 12345, E + 2**61 - 1]
    import random as _r
    rnd = _r.Random(7)
    ts += [E + rnd.randrange(1, 2**61) for _ in range(200)]
    ts += [E + 1 + (rnd.randrange(0, 2**50) * 10 ** rnd.randrange(0, 10) % (2**61 - 1)) for _ in range(200)]
    st = [ALIVE, TOMBSTONE, UNHEALTHY, UNKNOWN, DRAINING]
    recs = [(i % e.H, i % e.S, t, st[i % 5]) for i, t in enumerate(ts)]
    want = [len('"' + go_rfc3339nano(t) + '"') + len(str(s_)) for (_, _, t, s_) in recs]
    assert e.message_bytes(recs) == want


def kat_getbroadcasts_bytes_nothing(lib):
    """services_delegate_test.go:41-43 — GetBroadcasts(3, 1398) is nil when there is nothing to send."""
    e = _delegate_bytes(lib)
    assert e.get_broadcasts_bytes(LOCAL, 3, 1398) is None


def kat_getbroadcasts_bytes_pending_only(lib):
    """services_delegate_test.go:45-52 — returns from the pending list when nothing is new."""
    e = _delegate_bytes(lib)
    _set_pending(e, LOCAL, [BCAST[0]])
    r = e.get_broadcasts_bytes(LOCAL, 3, 1398)
    assert [tup(x) for x in r] == [BCAST[0]] and e.pending(LOCAL) == []


def kat_getbroadcasts_bytes_channel(lib):
    """services_delegate_test.go:54-63 — returns what's in the channel (2 x 225 B fit in 1398)."""
    e = _delegate_bytes(lib)
    e.send_services(LOCAL, BCAST, 1)
    r = e.get_broadcasts_bytes(LOCAL, 3, 1398)
    assert [tup(x) for x in r] == BCAST and e.pending(LOCAL) == []
    assert e.stats()["bytes_sent"] == 2 * (225 + 3)


def kat_getbroadcasts_bytes_leftover(lib):
    """services_delegate_test.go:65-73 — returns what's left when nothing is new."""
    e = _delegate_bytes(lib)
    _set_pending(e, LOCAL, BCAST)
    r = e.get_broadcasts_bytes(LOCAL, 3, 1398)
    assert [tup(x) for x in r] == BCAST and e.pending(LOCAL) == []


def kat_getbroadcasts_bytes_new_and_left(lib):
    """services_delegate_test.go:75-86 — what's new first, then what's left, when it fits."""
    e = _delegate_bytes(lib)
    _set_pending(e, LOCAL, BCAST)
    e.send_services(LOCAL, BCAST2, 1)
    r = e.get_broadcasts_bytes(LOCAL, 3, 1398)
    assert [tup(x) for x in r] == BCAST2 + BCAST and e.pending(LOCAL) == []


def kat_getbroadcasts_bytes_many_runs(lib):
    """services_delegate_test.go:88-103 — GetBroadcasts(3,100) nil, (3,300) one message (214+3),
    (3,100) nil, (3,1398) the other five: bCast2[1:] ++ bCast ++ bCast... as listed there."""
    e = _delegate_bytes(lib)
    _set_pending(e, LOCAL, BCAST)
    e.send_services(LOCAL, BCAST2 + BCAST, 1)
    assert e.get_broadcasts_bytes(LOCAL, 3, 100) is None
    r = e.get_broadcasts_bytes(LOCAL, 3, 300)  # 1 message fits here
    assert [tup(x) for x in r] == [BCAST2[0]]
    assert e.get_broadcasts_bytes(LOCAL, 3, 100) is None
    r = e.get_broadcasts_bytes(LOCAL, 3, 1398)
    assert len(r) == 5
    assert [tup(x) for x in r][:3] == BCAST2[1:] + BCAST
    assert e.pending(LOCAL) == []
    st = e.stats()
    assert st["bytes_sent"] == (214 + 3) + 5 * (225 + 3) and st["cap_cuts"] == 0


def kat_getbroadcasts_bytes_exact_fit(lib):
    """packPacket's test is total + len + overhead > limit (services_delegate.go:195): a message
    ending exactly at the limit fits, one byte less does not."""
    e = _delegate_bytes(lib)
    e.send_services(LOCAL, BCAST, 1)
    assert [tup(x) for x in e.get_broadcasts_bytes(LOCAL, 3, 2 * 228 - 1)] == [BCAST[0]]
    assert [tup(x) for x in e.get_broadcasts_bytes(LOCAL, 3, 228)] == [BCAST[1]]
    e.send_services(LOCAL, BCAST, 1)
    assert e.get_broadcasts_bytes(LOCAL, 3, 227) is None
    assert [tup(x) for x in e.pending(LOCAL)] == BCAST


def kat_getbroadcasts_bytes_pass_length(lib):
    """Each SendServices pass adds 50 ns (services_state.go:599), which changes the encoded length
    ("...453Z" -> "...503Z" -> "...553Z" keeps 9 digits; a fraction ending in zeros is shorter)."""
    e = _delegate_bytes(lib)
    t = _T46 - 453 + 400  # fraction .6696484 (7 digits), then .66964845 (8), then .6696485 (7)
    e.send_services(LOCAL, [(DOCKER2, 0, t, ALIVE)], 3)  # retransmit_rounds = 0: passes back to back
    sent = []
    for p in range(3):
        r = e.get_broadcasts_bytes(LOCAL, 0, 1398)
        assert [tup(x) for x in r] == [(DOCKER2, 0, t + 50 * p, ALIVE)]
        sent.append(e.stats()["bytes_sent"])
    lens = [sent[0], sent[1] - sent[0], sent[2] - sent[1]]
    static = _fixture_static(_FIX["d419"])
    assert lens == [static + len('"' + go_rfc3339nano(t + 50 * p) + '"') + 1 for p in range(3)]
    assert lens == [223, 224, 223]


# --------------------------------------------------------------- round-model semantic pins
def kat_order_dependence(lib):
    """SURVEY.md §7 hard part: the merge is not a semilattice. old=(t1,DRAINING):
    (t3,ALIVE) then (t2,TOMBSTONE) -> (t3,DRAINING); the reverse -> (t3,ALIVE)."""
    t1, t2, t3 = T0 - 3 * SEC, T0 - 2 * SEC, T0 - SEC
    e = mk(lib)
    e.add_service_entry(LOCAL, (CH, 0, t1, DRAINING))
    e.notify_msg(LOCAL, [(CH, 0, t3, ALIVE), (CH, 0, t2, TOMBSTONE)])
    assert e.slot(LOCAL, CH, 0) == (t3, DRAINING)
    e2 = mk(lib)
    e2.add_service_entry(LOCAL, (CH, 0, t1, DRAINING))
    e2.notify_msg(LOCAL, [(CH, 0, t2, TOMBSTONE), (CH, 0, t3, ALIVE)])
    assert e2.slot(LOCAL, CH, 0) == (t3, ALIVE)


def kat_equal_timestamp_first_wins(lib):
    """service.go:64-66 — Invalidates is strict: an equal timestamp keeps the first arrival."""
    e = mk(lib)
    e.notify_msg(LOCAL, [(CH, 0, T0, ALIVE), (CH, 0, T0, TOMBSTONE)])
    assert e.slot(LOCAL, CH, 0) == (T0, ALIVE)
    assert e.stats()["retransmits"] == 1


def kat_pending_truncation(lib):
    """services_delegate.go:109-115 — leftovers beyond MAX_PENDING_LENGTH are dropped; a batch
    longer than packet_cap + pending_cap can never send its tail."""
    e = mk(lib, n_hosts=4, n_services=64)
    recs = [(h, s, T0, ALIVE) for h in range(3) for s in range(64)][:150]
    e.send_services(LOCAL, recs, 1)
    b = e.get_broadcasts(LOCAL)
    assert [tup(x) for x in b] == recs[:32]
    assert [tup(x) for x in e.pending(LOCAL)] == recs[32:132]
    assert e.stats()["pending_drops"] == 0  # the stored list was already cut to 132
    e.send_services(LOCAL, recs[:40], 1)
    b = e.get_broadcasts(LOCAL)
    assert [tup(x) for x in b] == recs[:32]
    assert [tup(x) for x in e.pending(LOCAL)] == recs[32:40] + recs[32:124]
    assert e.stats()["pending_drops"] == 8


# ---------------------------------------------------------------- batched boundary calls (§8b)
def kat_notify_msgs_batched(lib):
    """SURVEY.md §8b gx_notify_msgs: one call for many hosts equals NotifyMsg per run of one host
    (services_delegate.go:71-83), in order; gx_read_view unpacks the same slots."""
    recs = [(SH, 0, T0, ALIVE), (SH, 1, T0, ALIVE), (CH, 0, T0 + SEC, DRAINING), (SH, 0, T0 + 2 * SEC, ALIVE),
            (CH, 0, T0, ALIVE)]
    hosts = [LOCAL, LOCAL, OTHER, LOCAL, OTHER]
    a, b = mk(lib), mk(lib)
    a.notify_msgs(hosts, recs)
    b.notify_msg(LOCAL, recs[:2])
    b.notify_msg(OTHER, recs[2:3])
    b.notify_msg(LOCAL, recs[3:4])
    b.notify_msg(OTHER, recs[4:5])
    assert (a.read_views() == b.read_views()).all()
    assert a.stats() == b.stats()
    for v in (LOCAL, OTHER):
        assert [bytes(j) for j in a.queue(v)] == [bytes(j) for j in b.queue(v)]
    ts, st = a.read_view(LOCAL)
    assert (ts[SH * 8 + 0], st[SH * 8 + 0]) == (T0 + 2 * SEC, ALIVE)
    assert (ts[SH * 8 + 1], st[SH * 8 + 1]) == (T0, ALIVE)
    assert st[CH * 8 + 0] == 7 and ts[CH * 8 + 0] == -(2**63)  # empty in LOCAL's view
    ts, st = a.read_view(OTHER)
    assert (ts[CH * 8 + 0], st[CH * 8 + 0]) == (T0 + SEC, DRAINING)  # the older ALIVE lost


# ------------------------------------------------------------------------- catalog/view_test.go
# hostname1..3 = shakespeare, chaucer, bocaccio; svcId1/2/3 = deadbeef123 / deadbeef101 / deadbeef105
# interned as service slots 1, 0, 2 of every host (slot = the ID's rank, so key order = ID order
# among one host's records). baseTime is a whole second.
BOC = 3  # "bocaccio"
ID1, ID2, ID3 = 1, 0, 2  # deadbeef123, deadbeef101, deadbeef105
IDS = {ID1: "deadbeef123", ID2: "deadbeef101", ID3: "deadbeef105"}


def _view_state(lib):
    e = mk(lib)
    e.add_service_entry(LOCAL, (SH, ID1, T0 + 5 * SEC, ALIVE))
    e.add_service_entry(LOCAL, (CH, ID2, T0, ALIVE))
    e.add_service_entry(LOCAL, (BOC, ID3, T0 + 10 * SEC, ALIVE))
    return e


def kat_view_sorted_services(lib):
    """view_test.go:50-69 — Server.SortedServices: bocaccio's services by Updated."""
    e = _view_state(lib)
    e.add_service_entry(LOCAL, (BOC, ID3, T0 + 10 * SEC, ALIVE))
    e.add_service_entry(LOCAL, (BOC, ID2, T0, ALIVE))
    e.add_service_entry(LOCAL, (BOC, ID1, T0 + 5 * SEC, ALIVE))
    ids = [IDS[x.svc] for x in e.each_service_sorted(LOCAL, BOC)]
    assert ids == ["deadbeef101", "deadbeef123", "deadbeef105"]


def kat_view_each_service_sorted(lib):
    """view_test.go:71-91 — EachServiceSorted over every server: IDs by Updated
    (deadbeef101 x2 at baseTime, deadbeef123 x2 at +5 s, deadbeef105 at +10 s). bocaccio's
    deadbeef105 at the same time is not newer, so it is not added twice."""
    e = _view_state(lib)
    e.add_service_entry(LOCAL, (BOC, ID1, T0 + 5 * SEC, ALIVE))
    e.add_service_entry(LOCAL, (BOC, ID2, T0, ALIVE))
    e.add_service_entry(LOCAL, (BOC, ID3, T0 + 10 * SEC, ALIVE))
    got = e.each_service_sorted(LOCAL)
    assert [IDS[x.svc] for x in got] == ["deadbeef101", "deadbeef101", "deadbeef123", "deadbeef123", "deadbeef105"]
    times = [x.updated_ns for x in got]
    assert times == sorted(times)
    # equal Updated: key order (Go's sort.Sort leaves it unspecified)
    assert [(x.host, x.svc) for x in got[:2]] == [(CH, ID2), (BOC, ID2)]


def kat_by_service_groups_by_name(lib):
    """services_state.go:738-748 — ByService groups EachServiceSorted's services by Service.Name.
    Names: every deadbeef123 record is "web", deadbeef101 "db", deadbeef105 "web"."""
    e = _view_state(lib)
    e.add_service_entry(LOCAL, (BOC, ID1, T0 + 5 * SEC, ALIVE))
    e.add_service_entry(LOCAL, (BOC, ID2, T0, ALIVE))
    names = []
    for h in range(e.H):
        for sv in range(e.S):
            names.append({ID1: "web", ID2: "db", ID3: "web"}.get(sv, f"other{sv}"))
    e.set_service_names(names)
    got = e.by_service(LOCAL)
    groups = {}
    for g, x in got:
        groups.setdefault(g, []).append((x.host, IDS[x.svc], x.updated_ns))
    # groups in bytewise name order: "db" < "web"
    assert list(groups) == sorted(groups)
    db, web = groups[min(groups)], groups[max(groups)]
    assert [i for _, i, _ in db] == ["deadbeef101", "deadbeef101"]
    assert [(h, i) for h, i, _ in web] == [(SH, "deadbeef123"), (BOC, "deadbeef123"), (BOC, "deadbeef105")]


def kat_by_service_needs_names(lib):
    """ByService without a name table: GX_ENOENT."""
    from sidecar_amd.abi import GxError
    e = _view_state(lib)
    try:
        e.by_service(LOCAL)
    except GxError as x:
        assert "-2" in str(x) or "ENOENT" in str(x)
    else:
        raise AssertionError("expected GX_ENOENT")


# ---------------------------------------------------- the engine's time window (gx.h GX_TS_SHIFT)
# The packed slot keeps Updated relative to the engine epoch (t0 - 2^60, whole seconds): with t0
# in November 2023 the 73-year window runs May 1987 .. May 2060. Records from both sides of 2043
# (the old 2^61 ns horizon) merge exactly; times outside the window clamp to its ends.
Y2050 = 2_524_608_000 * SEC  # 2050-01-01T00:00:00Z
Y2055 = 2_682_374_400 * SEC  # 2055-01-01T00:00:00Z
Y2100 = 4_102_444_800 * SEC  # 2100-01-01T00:00:00Z, past the window
ZERO_TIME_NS = -(2**63)      # time.Time{} (year 1) has no UnixNano; a binding passes INT64_MIN


def kat_time_window_far_future(lib):
    """services_state_test.go:177-183 (a newer record replaces the stored Updated) and :135-155
    (an older one is ignored) with Updated past 2043: 2050 and 2055 merge and read back exactly; a
    record from 2100 (past the window) still wins every later merge, as the reference's would, and
    reads back as the window's end (engine bound)."""
    e = mk(lib)
    E = e.epoch
    assert E % SEC == 0 and E < T0 - 2**59 and E + 2**61 > Y2055
    assert e.add_service_entry(LOCAL, (CH, 0, Y2050, ALIVE)) == 1
    assert e.slot(LOCAL, CH, 0) == (Y2050, ALIVE)
    assert e.add_service_entry(LOCAL, (CH, 0, T0, TOMBSTONE)) == 0  # older
    assert e.add_service_entry(LOCAL, (CH, 0, Y2055 + 123, DRAINING)) == 1
    assert e.slot(LOCAL, CH, 0) == (Y2055 + 123, DRAINING)
    assert e.add_service_entry(LOCAL, (CH, 0, Y2100, TOMBSTONE)) == 1
    end = E + 2**61 - 1
    assert e.slot(LOCAL, CH, 0) == (end, TOMBSTONE)
    assert e.add_service_entry(LOCAL, (CH, 0, Y2055 + 124, ALIVE)) == 0
    # every reader hands out absolute times
    got = [tup(x) for x in e.local_state(LOCAL) if x.host == CH]
    assert got == [(CH, 0, end, TOMBSTONE)]
    ts, st = e.read_view(LOCAL)
    assert (ts[CH * e.S], st[CH * e.S]) == (end, TOMBSTONE)


def kat_time_window_pre_1970_and_zero(lib):
    """service/service.go:68-72 IsStale + services_state.go:302-308: a record whose Updated is
    before 1970, the zero time.Time, or any time before the window is older than now - 3h - 1min,
    so AddServiceEntry drops it (stale) and creates nothing."""
    e = mk(lib)
    e.set_round(1)
    for t in (-SEC, -500_000_000, ZERO_TIME_NS, 0, 315_532_800 * SEC):  # 1969, zero, 1970, 1980
        assert e.add_service_entries([LOCAL], [(CH, 1, t, ALIVE)]) == 0
        assert e.add_service_entries([LOCAL], [(CH, 2, t, TOMBSTONE)]) == 0
    assert all(e.slot(LOCAL, CH, s) is None for s in range(e.S))
    assert e.stats()["stale_drops"] == 10


def _window_doc(e, names, recs):
    """A ServicesState JSON holding `recs` = [(host, svc, Updated text or None, Status)]."""
    import json as _json
    servers = {}
    for h, sv, upd, st in recs:
        host = names.hosts[h].decode()
        svc = {"ID": names.ids[h * e.S + sv].decode(), "Hostname": host, "Status": st}
        if upd is not None:
            svc["Updated"] = upd
        servers.setdefault(host, {"Name": host, "Services": {}})["Services"][svc["ID"]] = svc
    return _json.dumps({"Servers": servers, "ClusterName": "default"}).encode()


def kat_time_window_decode(lib):
    """catalog.Decode + MergeRemoteState (services_state.go:355-373) of records from 2050, past the
    window (2100), 1969, and with Updated missing (the zero time.Time): Decode reads them all (none
    invalid), the merge keeps the 2050 and 2100 records and drops the other two as stale."""
    from sidecar_amd.codec import synthetic_names
    e = mk(lib)
    names = synthetic_names(e.H, e.S, seed=5)
    e.set_names(names)
    e.set_round(1)
    recs = [(CH, 0, "2050-01-01T00:00:00.5Z", ALIVE), (CH, 1, "2100-01-01T00:00:00Z", DRAINING),
            (SH, 0, "1969-12-31T23:59:59.5Z", ALIVE), (SH, 1, None, TOMBSTONE),
            (SH, 2, "0001-01-01T00:00:00Z", ALIVE)]
    doc = _window_doc(e, names, recs)
    rc, got, ds = e.decode_state_json(doc)
    assert rc == 0 and ds["invalid"] == 0 and ds["unknown"] == 0 and ds["records"] == 5, ds
    E, end = e.epoch, e.epoch + 2**61 - 1
    want = {(CH, 0): (Y2050 + 500_000_000, ALIVE), (CH, 1): (end, DRAINING), (SH, 0): (E, ALIVE),
            (SH, 1): (E, TOMBSTONE), (SH, 2): (E, ALIVE)}
    assert {(h, sv): (t, st) for t, h, sv, st in got} == want
    rc, ds = e.merge_remote_state_json(LOCAL, doc)
    assert rc == 0
    assert e.slot(LOCAL, CH, 0) == (Y2050 + 500_000_000, ALIVE)
    assert e.slot(LOCAL, CH, 1) == (end, DRAINING)
    assert all(e.slot(LOCAL, SH, s) is None for s in range(3))
    assert e.stats()["stale_drops"] == 3
    # and the encoder writes the 2050 record back as Go would
    assert b'"Updated":"2050-01-01T00:00:00.5Z"' in e.local_state_json(LOCAL)


ALL = [v for k, v in sorted(globals().items()) if k.startswith("kat_")]

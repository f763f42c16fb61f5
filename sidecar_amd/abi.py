"""ctypes mirror of include/gx.h and a thin Python handle over the C-ABI.

The product library is ``sidecar_amd/libgx.so`` (HIP kernels for gfx950). ``Engine`` loads it by
default and raises if it is missing — there is no CPU fallback in the product path. Tests may
pass another library exporting the same ABI (the CPU oracle) explicitly via ``lib=``.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Iterable, Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIBGX_PATH = os.path.join(HERE, "libgx.so")

GX_OK = 0
GX_EIO = -5
GX_ENOMEM = -12
GX_EINVAL = -22
GX_ENOENT = -2
GX_ENOSYS = -38

ALIVE, TOMBSTONE, UNHEALTHY, UNKNOWN, DRAINING, ABSENT = 0, 1, 2, 3, 4, 7
SLOT_ABSENT = 7
TS_SHIFT = 3

JOB_NIL_BS, JOB_NIL_BT, JOB_RETX, JOB_SEND, JOB_EXPIRE, JOB_LOST = 0, 1, 2, 3, 4, 5
INIT_EMPTY, INIT_OWN, INIT_WARM = 0, 1, 2
LIMIT_DEFAULT = 0xFFFFFFFF
LOCK_PENDING_EXPIRE, LOCK_DEFER_MERGE, LOCK_BUF_SHIFT = 4, 8, 8  # gx_host_state.lock (gx.h)

K_NAMES = ["owner", "scan", "storm", "send", "route", "merge", "ae", "converge", "encode", "decode", "fd"]


class GxService(C.Structure):
    _fields_ = [("updated_ns", C.c_int64), ("host", C.c_uint32), ("svc", C.c_uint16),
                ("status", C.c_uint8), ("flags", C.c_uint8)]

    def tup(self):
        return (self.updated_ns, self.host, self.svc, self.status)

    def __repr__(self):
        return f"Svc(h={self.host},s={self.svc},t={self.updated_ns},st={self.status})"


class GxJob(C.Structure):
    """gx.h gx_job (16 B): meta = kind | pass << 3 | n_passes << 9 | owner << 15."""
    _fields_ = [("a", C.c_uint64), ("c", C.c_uint32), ("meta", C.c_uint32)]

    @property
    def kind(self):
        return self.meta & 7

    @property
    def pass_(self):
        return (self.meta >> 3) & 63

    @property
    def n_passes(self):
        return (self.meta >> 9) & 63

    @property
    def owner(self):
        return self.meta >> 15

    def tup(self):
        return (self.a, self.c, self.meta)


class GxSleeper(C.Structure):
    _fields_ = [("job", GxJob), ("wake", C.c_uint32), ("pad", C.c_uint32 * 3)]

    @property
    def kind(self):
        return self.job.kind

    @property
    def pass_(self):
        return self.job.pass_

    @property
    def n_passes(self):
        return self.job.n_passes

    def tup(self):
        return self.job.tup() + (self.wake,)


class GxParams(C.Structure):
    _fields_ = [
        ("n_hosts", C.c_uint32), ("n_services", C.c_uint32), ("fanout", C.c_uint32),
        ("packet_cap", C.c_uint32), ("pending_cap", C.c_uint32), ("queue_cap", C.c_uint32),
        ("list_slots", C.c_uint32), ("gossip_stop_on_empty", C.c_uint32),
        ("alive_interval_rounds", C.c_uint32), ("tombstone_interval_rounds", C.c_uint32),
        ("retransmit_rounds", C.c_uint32), ("alive_count", C.c_uint32),
        ("tombstone_count", C.c_uint32), ("ae_period_rounds", C.c_uint32),
        ("ae_phase", C.c_uint32), ("init_mode", C.c_uint32),
        ("t0_ns", C.c_int64), ("round_ns", C.c_int64), ("alive_lifespan_ns", C.c_int64),
        ("draining_lifespan_ns", C.c_int64), ("tombstone_lifespan_ns", C.c_int64),
        ("stale_fudge_ns", C.c_int64), ("alive_broadcast_interval_ns", C.c_int64),
        ("pass_increment_ns", C.c_int64), ("tombstone_bump_ns", C.c_int64),
        ("seed", C.c_uint64), ("churn_ppm", C.c_uint32), ("aged_ppm", C.c_uint32),
        ("aged_max_ns", C.c_int64), ("partition_start", C.c_int32), ("partition_end", C.c_int32),
        ("storm_round", C.c_int32), ("device", C.c_int32), ("n_shards", C.c_uint32),
        ("shard_id", C.c_uint32),
        ("limit_bytes", C.c_uint32),
        ("overhead_bytes", C.c_uint32),
        ("fd_enable", C.c_uint32), ("fd_probe_rounds", C.c_uint32), ("fd_indirect_checks", C.c_uint32),
        ("fd_retransmit_limit", C.c_uint32), ("fd_msg_cap", C.c_uint32), ("fd_msg_bytes", C.c_uint32),
        ("fd_gossip_dead_rounds", C.c_uint32), ("fd_suspicion_k", C.c_uint32),
        ("fd_suspicion_rounds", C.c_uint32 * 8), ("depart_round", C.c_int32), ("depart_ppm", C.c_uint32),
        ("fd_push_pull_state", C.c_uint32),
        ("gossip_messages", C.c_uint32), ("push_pull_mode", C.c_uint32), ("inbox_slots", C.c_uint32),
        ("lock_model", C.c_uint32), ("lock_buffer", C.c_uint32), ("probe_piggyback", C.c_uint32),
        ("push_pull_stagger", C.c_uint32), ("lock_readers", C.c_uint32), ("lock_defer_slots", C.c_uint32),
        ("fd_handoff_shared", C.c_uint32),
    ]

    # fields memberlist derives from the cluster size (gx_fd_defaults)
    FD_DERIVED = ("fd_retransmit_limit", "fd_suspicion_k", "fd_suspicion_rounds")


class GxServerTimes(C.Structure):
    _fields_ = [("last_updated_ns", C.c_int64), ("last_changed_ns", C.c_int64)]


class GxChangeEvent(C.Structure):
    _fields_ = [("service", GxService), ("time_ns", C.c_int64), ("previous_status", C.c_uint32),
                ("pad", C.c_uint32)]

    def tup(self):
        return (self.service.host, self.service.svc, self.service.updated_ns, self.service.status,
                self.previous_status, self.time_ns)


class GxHostState(C.Structure):
    _fields_ = [("fifo_head", C.c_uint32), ("fifo_tail", C.c_uint32), ("sleep_head", C.c_uint32),
                ("sleep_tail", C.c_uint32), ("dq_head", C.c_uint32), ("dq_len", C.c_uint32),
                ("arena_used", C.c_uint32), ("flags", C.c_uint32), ("bs_next", C.c_int64),
                ("bt_next", C.c_int64), ("last_bcast_ns", C.c_int64), ("running", C.c_uint64),
                ("fifo_stored", C.c_uint32), ("nil_pos_bs", C.c_uint32), ("nil_pos_bt", C.c_uint32),
                ("lock", C.c_uint32)]

    def locked_at(self, round_):
        """A looper held the ServicesState lock at the start of round `round_` (gx.h lock)."""
        return (self.lock >> (round_ & 1)) & 1

    @property
    def lock_buffered(self):
        return self.lock >> LOCK_BUF_SHIFT


class GxStats(C.Structure):
    _fields_ = [("round", C.c_int64)] + [(n, C.c_uint64) for n in (
        "gossip_merges", "ae_merges", "local_merges", "gossip_accepts", "ae_accepts",
        "local_accepts", "stale_drops", "retransmits", "queue_drops", "list_drops", "sleep_drops",
        "pending_drops", "dequeues", "nil_batches", "packets", "records_sent", "expired", "gc",
        "own_tombstones", "expire_server", "send_jobs", "ae_exchanges", "churn_events")] + [
        ("last_change_round", C.c_int64), ("scan_slots", C.c_uint64), ("ae_slots", C.c_uint64),
        ("bytes_sent", C.c_uint64), ("cap_cuts", C.c_uint64), ("change_events", C.c_uint64),
        ("listener_drops", C.c_uint64)] + [(n, C.c_uint64) for n in (
        "lost_packets", "fd_probes", "fd_probe_failures", "fd_suspicions", "fd_confirmations",
        "fd_deaths", "fd_refutes", "fd_alive_updates", "fd_msgs_sent", "fd_msgs_received",
        "fd_state_merges", "queue_deferred")] + [("first_drop_round", C.c_int64)] + [
        ("locked_merges", C.c_uint64), ("first_locked_round", C.c_int64)] + [(n, C.c_uint64) for n in (
        "lock_buffered", "lock_drops", "lock_drained", "ae_locked", "expire_deferred", "ae_deferred",
        "ae_defer_lost", "fd_handoff_queued", "fd_handoff_drops", "false_expiries")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_ if n != "reserved"}


M_ALIVE, M_SUSPECT, M_DEAD = 0, 1, 2
FD_NONE = 0xFFFF
FD_NO_DEADLINE = 0x7FFFFFFF


class GxMember(C.Structure):
    _fields_ = [("incarnation", C.c_uint32), ("msg_incarnation", C.c_uint32), ("change_round", C.c_int32),
                ("deadline", C.c_int32), ("state", C.c_uint8), ("n_conf", C.c_uint8), ("tx", C.c_uint8),
                ("msg_kind", C.c_uint8), ("msg_from", C.c_uint16), ("susp_from", C.c_uint16 * 3),
                ("q_prev", C.c_uint16), ("q_next", C.c_uint16)]


class GxFdHost(C.Structure):
    _fields_ = [("probe_pass", C.c_uint32), ("probe_index", C.c_uint32), ("wrap_round", C.c_int32),
                ("min_deadline", C.c_int32), ("q_len", C.c_uint32), ("departed", C.c_uint32),
                ("q_head", C.c_uint16 * 32), ("hq_len", C.c_uint32)]


class GxFdMsg(C.Structure):
    _fields_ = [("incarnation", C.c_uint32), ("node", C.c_uint16), ("from_", C.c_uint16), ("kind", C.c_uint8),
                ("pad", C.c_uint8 * 3)]

    def tup(self):
        return (self.kind, self.node, self.incarnation, self.from_)


def fd_msg(kind, node, inc, frm=None) -> GxFdMsg:
    return GxFdMsg(int(inc), int(node), int(node if frm is None else frm), int(kind))


class GxTiming(C.Structure):
    _fields_ = [("ms", C.c_double * 11), ("launches", C.c_uint64 * 11), ("bytes", C.c_uint64 * 11),
                ("units", C.c_uint64 * 11)]

    def as_dict(self):
        return {K_NAMES[i]: {"ms": self.ms[i], "launches": self.launches[i],
                             "bytes": self.bytes[i], "units": self.units[i]} for i in range(len(K_NAMES))}


class GxNames(C.Structure):
    _fields_ = [("cluster_name", C.c_char_p), ("cluster_name_len", C.c_uint64),
                ("hosts", C.c_char_p), ("host_off", C.c_void_p), ("ids", C.c_char_p), ("id_off", C.c_void_p),
                ("pre", C.c_char_p), ("pre_off", C.c_void_p), ("post", C.c_char_p), ("post_off", C.c_void_p)]


class GxDecodeStats(C.Structure):
    _fields_ = [("bytes", C.c_uint64), ("tokens", C.c_uint64), ("services", C.c_uint32),
                ("records", C.c_uint32), ("unknown", C.c_uint32), ("invalid", C.c_uint32),
                ("error_at", C.c_int64)]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


ABI_FUNCS = [
    "gx_abi_version", "gx_backend", "gx_params_default", "gx_create", "gx_destroy", "gx_set_round",
    "gx_get_round", "gx_epoch", "gx_outbox_sizes_async", "gx_owner_slots_in_use", "gx_enable_timing", "gx_run_rounds", "gx_add_service_entries", "gx_merge",
    "gx_tombstone_others", "gx_tombstone_services", "gx_expire_server", "gx_send_services",
    "gx_broadcast_services", "gx_broadcast_tombstones", "gx_is_new_service", "gx_notify_msg", "gx_notify_msgs", "gx_read_view",
    "gx_get_broadcasts", "gx_local_state", "gx_merge_remote_state", "gx_notify_leave",
    "gx_read_views", "gx_write_views", "gx_write_slot", "gx_read_hosts", "gx_read_queue",
    "gx_read_sleepers", "gx_read_pending", "gx_read_list", "gx_host_digests", "gx_stats_get",
    "gx_timing_get", "gx_converged", "gx_round_send", "gx_outbox_bytes", "gx_outbox_pack",
    "gx_inbox_unpack", "gx_exchange_plan", "gx_outbox_pack_planned", "gx_round_merge", "gx_ae_bytes", "gx_ae_pack", "gx_ae_merge", "gx_round_end",
    "gx_round_gossip_begin", "gx_round_gossip_end", "gx_lock_census", "gx_ae_skip_locked",
    "gx_view_minmax", "gx_owner_words", "gx_read_server_times", "gx_read_last_changed", "gx_add_listener",
    "gx_remove_listener", "gx_listener_drain", "gx_ae_merge_local", "gx_ae_delta_bytes", "gx_ae_delta_pack", "gx_ae_return_bytes", "gx_ae_return_pack", "gx_set_stream", "gx_get_broadcasts_bytes", "gx_set_static_bytes", "gx_message_bytes",
    "gx_set_names", "gx_local_state_json", "gx_decode_state_json", "gx_merge_remote_state_json",
    "gx_fd_defaults", "gx_fd_read_members", "gx_fd_read_hosts", "gx_fd_read_queue", "gx_fd_notify",
    "gx_fd_get_broadcasts", "gx_fd_probe", "gx_fd_timers", "gx_fd_converged", "gx_fd_merge_state",
    "gx_each_service_sorted", "gx_set_service_names", "gx_by_service",
]
ALL_OWNERS = 0xFFFFFFFF


def _declare(lib):
    P = C.POINTER
    vp = C.c_void_p
    u32, i32, i64, u16 = C.c_uint32, C.c_int, C.c_int64, C.c_uint16
    sig = {
        "gx_abi_version": ([], i32), "gx_backend": ([], C.c_char_p),
        "gx_params_default": ([P(GxParams)], None), "gx_create": ([P(GxParams), P(vp)], i32),
        "gx_destroy": ([vp], i32), "gx_set_round": ([vp, i64], i32),
        "gx_get_round": ([vp, P(i64)], i32), "gx_epoch": ([vp, P(i64)], i32), "gx_outbox_sizes_async": ([vp, vp], i32), "gx_owner_slots_in_use": ([vp, u32, P(C.c_uint64)], i32), "gx_enable_timing": ([vp, i32], i32),
        "gx_run_rounds": ([vp, u32], i32),
        "gx_add_service_entries": ([vp, P(u32), P(GxService), u32, P(u32)], i32),
        "gx_merge": ([vp, u32, u32], i32),
        "gx_tombstone_others": ([vp, u32, P(GxService), u32, P(u32)], i32),
        "gx_tombstone_services": ([vp, u32, P(u16), u32, P(GxService), u32, P(u32)], i32),
        "gx_expire_server": ([vp, u32, u32, P(i32)], i32),
        "gx_send_services": ([vp, u32, P(GxService), u32, u32], i32),
        "gx_broadcast_services": ([vp, u32, P(GxService), u32], i32),
        "gx_broadcast_tombstones": ([vp, u32, P(GxService), u32], i32),
        "gx_is_new_service": ([vp, u32, P(GxService), P(i32)], i32),
        "gx_notify_msg": ([vp, u32, P(GxService), u32], i32),
        "gx_notify_msgs": ([vp, P(u32), P(GxService), u32], i32),
        "gx_read_view": ([vp, u32, vp, vp], i32),
        "gx_get_broadcasts": ([vp, u32, u32, P(GxService), u32, P(u32)], i32),
        "gx_local_state": ([vp, u32, P(GxService), u32, P(u32)], i32),
        "gx_merge_remote_state": ([vp, u32, P(GxService), u32], i32),
        "gx_notify_leave": ([vp, u32, u32], i32),
        "gx_read_views": ([vp, u32, u32, vp], i32), "gx_write_views": ([vp, u32, u32, vp], i32),
        "gx_write_slot": ([vp, u32, P(GxService)], i32),
        "gx_read_hosts": ([vp, u32, u32, P(GxHostState)], i32),
        "gx_read_queue": ([vp, u32, P(GxJob), u32, P(u32)], i32),
        "gx_read_sleepers": ([vp, u32, P(GxSleeper), u32, P(u32)], i32),
        "gx_read_pending": ([vp, u32, P(GxService), u32, P(u32)], i32),
        "gx_read_list": ([vp, u32, u32, P(GxService), u32, P(u32)], i32),
        "gx_host_digests": ([vp, vp], i32), "gx_stats_get": ([vp, P(GxStats)], i32),
        "gx_timing_get": ([vp, P(GxTiming)], i32),
        "gx_converged": ([vp, P(i32), P(C.c_uint64)], i32),
        "gx_round_send": ([vp], i32), "gx_outbox_bytes": ([vp, vp], i32),
        "gx_outbox_pack": ([vp, vp, C.c_uint64], i32), "gx_inbox_unpack": ([vp, vp, C.c_uint64], i32),
        "gx_exchange_plan": ([vp, vp], i32), "gx_outbox_pack_planned": ([vp, vp, C.c_uint64], i32),
        "gx_round_merge": ([vp], i32), "gx_ae_bytes": ([vp, vp], i32),
        "gx_ae_pack": ([vp, vp, C.c_uint64], i32), "gx_ae_merge": ([vp, vp, C.c_uint64, vp, C.c_uint64], i32),
        "gx_round_end": ([vp], i32), "gx_view_minmax": ([vp, vp, vp], i32), "gx_owner_words": ([vp, vp], i32),
        "gx_round_gossip_begin": ([vp, vp, vp, C.c_uint64], i32),
        "gx_round_gossip_end": ([vp, vp, C.c_uint64, P(i32)], i32),
        "gx_lock_census": ([vp, P(u32)], i32), "gx_ae_skip_locked": ([vp], i32),
        "gx_ae_merge_local": ([vp], i32),
        "gx_read_server_times": ([vp, u32, u32, u32, vp], i32),
        "gx_read_last_changed": ([vp, u32, u32, vp], i32),
        "gx_add_listener": ([vp, u32, u32, u32], i32),
        "gx_remove_listener": ([vp, u32, u32], i32),
        "gx_listener_drain": ([vp, u32, u32, P(GxChangeEvent), u32, P(u32)], i32),
        "gx_ae_delta_bytes": ([vp, vp, C.c_uint64, vp], i32),
        "gx_ae_delta_pack": ([vp, vp, C.c_uint64], i32),
        "gx_ae_return_bytes": ([vp, vp, C.c_uint64, vp], i32),
        "gx_set_stream": ([vp, vp, i32], i32),
        "gx_ae_return_pack": ([vp, vp, C.c_uint64, vp, C.c_uint64], i32),
        "gx_get_broadcasts_bytes": ([vp, u32, u32, u32, P(GxService), u32, P(u32)], i32),
        "gx_set_static_bytes": ([vp, u32, u32, P(u16)], i32),
        "gx_message_bytes": ([vp, P(GxService), u32, P(u32)], i32),
        "gx_set_names": ([vp, P(GxNames)], i32),
        "gx_local_state_json": ([vp, u32, vp, C.c_uint64, P(C.c_uint64)], i32),
        "gx_decode_state_json": ([vp, vp, C.c_uint64, P(GxService), u32, P(u32), P(GxDecodeStats)], i32),
        "gx_merge_remote_state_json": ([vp, u32, vp, C.c_uint64, P(GxDecodeStats)], i32),
        "gx_fd_defaults": ([P(GxParams)], i32),
        "gx_fd_read_members": ([vp, u32, u32, u32, P(GxMember)], i32),
        "gx_fd_read_hosts": ([vp, u32, u32, P(GxFdHost)], i32),
        "gx_fd_read_queue": ([vp, u32, P(GxFdMsg), P(C.c_uint8), u32, P(u32)], i32),
        "gx_fd_notify": ([vp, u32, P(GxFdMsg), u32], i32),
        "gx_fd_get_broadcasts": ([vp, u32, u32, P(GxFdMsg), P(u32)], i32),
        "gx_fd_probe": ([vp, u32, P(u32), P(i32)], i32),
        "gx_fd_timers": ([vp, u32], i32),
        "gx_fd_converged": ([vp, P(i32), P(C.c_uint64)], i32),
        "gx_fd_merge_state": ([vp, u32, vp], i32),
        "gx_each_service_sorted": ([vp, u32, u32, P(GxService), u32, P(u32)], i32),
        "gx_set_service_names": ([vp, vp, P(C.c_uint64)], i32),
        "gx_by_service": ([vp, u32, P(GxService), P(u32), u32, P(u32)], i32),
    }
    for name, (args, res) in sig.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = res
    return lib


_LIB_CACHE = {}


def load_library(path: str):
    path = os.path.abspath(path)
    if path not in _LIB_CACHE:
        if not os.path.exists(path):
            raise RuntimeError(f"gx library not found: {path} (build it: python __graft_entry__.py build)")
        _LIB_CACHE[path] = _declare(C.CDLL(path))
    return _LIB_CACHE[path]


def load_product():
    """The HIP engine. Raises if the extension was not built — no fallback."""
    lib = load_library(LIBGX_PATH)
    be = lib.gx_backend().decode()
    if not be.startswith("hip"):
        raise RuntimeError(f"libgx.so reports backend {be!r}, expected the HIP engine")
    return lib


class GxError(RuntimeError):
    pass


def check(rc: int, what: str = ""):
    if rc != GX_OK:
        raise GxError(f"{what} failed with rc={rc}")


def default_params(lib=None, **kw) -> GxParams:
    p = GxParams()
    lib = lib or load_product()
    lib.gx_params_default(C.byref(p))
    for k, v in kw.items():
        if not hasattr(p, k):
            raise KeyError(k)
        if k == "fd_suspicion_rounds":
            v = (C.c_uint32 * 8)(*v)
        setattr(p, k, v)
    if not any(k in kw for k in GxParams.FD_DERIVED):
        check(lib.gx_fd_defaults(C.byref(p)), "gx_fd_defaults")  # memberlist's size-derived values
    return p


def svc(host, s, ts, status=ALIVE) -> GxService:
    return GxService(int(ts), int(host), int(s), int(status), 0)


def svc_array(items: Sequence) -> "C.Array":
    arr = (GxService * max(1, len(items)))()
    for i, it in enumerate(items):
        if isinstance(it, GxService):
            arr[i] = it
        else:
            arr[i] = svc(*it)
    return arr


class Engine:
    """One simulated cluster (H hosts x S services) behind the gx C-ABI."""

    def __init__(self, params: Optional[GxParams] = None, lib=None, **kw):
        self.lib = lib if lib is not None else load_product()
        if params is None:
            params = default_params(self.lib, **kw)
        else:
            for k, v in kw.items():
                setattr(params, k, v)
        self.params = params
        self.H = params.n_hosts
        self.S = params.n_services
        self.G = max(1, params.n_shards)
        gid = params.shard_id if self.G > 1 else 0
        self.lo = (gid * self.H) // self.G
        self.hi = ((gid + 1) * self.H) // self.G
        h = C.c_void_p()
        check(self.lib.gx_create(C.byref(params), C.byref(h)), "gx_create")
        self.h = h

    # lifecycle -------------------------------------------------------------------------
    def close(self):
        if self.h:
            self.lib.gx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def backend(self):
        return self.lib.gx_backend().decode()

    @property
    def round(self) -> int:
        r = C.c_int64()
        check(self.lib.gx_get_round(self.h, C.byref(r)))
        return r.value

    @property
    def epoch(self) -> int:
        """Absolute time of slot time 0: view words hold (updated_ns - epoch) << 3 (gx.h GX_TS_SHIFT)."""
        if not hasattr(self, "_epoch"):
            x = C.c_int64()
            check(self.lib.gx_epoch(self.h, C.byref(x)), "gx_epoch")
            self._epoch = x.value
        return self._epoch

    def owner_slots_in_use(self, owner: int) -> int:
        """Bit s set: some view of this engine holds a record for (owner, s) (gx.h)."""
        m = C.c_uint64()
        check(self.lib.gx_owner_slots_in_use(self.h, owner, C.byref(m)), "gx_owner_slots_in_use")
        return m.value

    def word_time(self, w: int) -> int:
        """Absolute Updated of a packed view word."""
        return (int(w) >> TS_SHIFT) + self.epoch

    def now(self, round_=None) -> int:
        r = self.round if round_ is None else round_
        return self.params.t0_ns + r * self.params.round_ns

    def set_round(self, r: int):
        check(self.lib.gx_set_round(self.h, int(r)), "gx_set_round")

    def enable_timing(self, on=True):
        check(self.lib.gx_enable_timing(self.h, 1 if on else 0))

    def run_rounds(self, n: int):
        check(self.lib.gx_run_rounds(self.h, int(n)), "gx_run_rounds")

    # ServicesState ---------------------------------------------------------------------
    def add_service_entries(self, views: Sequence[int], items: Sequence) -> int:
        n = len(items)
        va = (C.c_uint32 * max(1, n))(*views)
        acc = C.c_uint32()
        check(self.lib.gx_add_service_entries(self.h, va, svc_array(items), n, C.byref(acc)),
              "gx_add_service_entries")
        return acc.value

    def add_service_entry(self, view: int, item) -> int:
        return self.add_service_entries([view], [item])

    def merge(self, dst: int, src: int):
        check(self.lib.gx_merge(self.h, dst, src), "gx_merge")

    def merge_remote_state(self, view: int, items: Sequence):
        check(self.lib.gx_merge_remote_state(self.h, view, svc_array(items), len(items)))

    def tombstone_others(self, view: int, cap: int = 4096):
        out = (GxService * max(1, cap))()
        n = C.c_uint32()
        check(self.lib.gx_tombstone_others(self.h, view, out, cap, C.byref(n)))
        return [out[i] for i in range(min(n.value, cap))], n.value

    def tombstone_services(self, host: int, running: Iterable[int], cap: int = 256):
        run = list(running)
        ra = (C.c_uint16 * max(1, len(run)))(*run)
        out = (GxService * cap)()
        n = C.c_uint32()
        check(self.lib.gx_tombstone_services(self.h, host, ra, len(run), out, cap, C.byref(n)))
        return [out[i] for i in range(min(n.value, cap))]

    def expire_server(self, view: int, owner: int) -> bool:
        x = C.c_int()
        check(self.lib.gx_expire_server(self.h, view, owner, C.byref(x)))
        return bool(x.value)

    def send_services(self, host: int, items: Sequence, n_passes: int):
        check(self.lib.gx_send_services(self.h, host, svc_array(items), len(items), n_passes))

    def broadcast_services(self, host: int, items: Sequence):
        check(self.lib.gx_broadcast_services(self.h, host, svc_array(items), len(items)))

    def broadcast_tombstones(self, host: int, items: Sequence):
        check(self.lib.gx_broadcast_tombstones(self.h, host, svc_array(items), len(items)))

    def is_new_service(self, view: int, item) -> bool:
        x = C.c_int()
        a = svc_array([item])
        check(self.lib.gx_is_new_service(self.h, view, a, C.byref(x)))
        return bool(x.value)

    # delegate --------------------------------------------------------------------------
    def notify_msg(self, host: int, items: Sequence):
        check(self.lib.gx_notify_msg(self.h, host, svc_array(items), len(items)))

    def notify_msgs(self, hosts: Sequence[int], items: Sequence):
        """Batched NotifyMsg: items[i] to hosts[i], runs of one host form one message."""
        hs = (C.c_uint32 * len(hosts))(*hosts)
        check(self.lib.gx_notify_msgs(self.h, hs, svc_array(items), len(items)), "gx_notify_msgs")

    def read_view(self, view: int):
        """One view unpacked: (ts_ns int64[R], INT64_MIN where empty; status uint8[R])."""
        R = self.H * self.S
        ts = np.empty(R, dtype=np.int64)
        st = np.empty(R, dtype=np.uint8)
        check(self.lib.gx_read_view(self.h, view, ts.ctypes.data_as(C.c_void_p), st.ctypes.data_as(C.c_void_p)),
              "gx_read_view")
        return ts, st

    def get_broadcasts(self, host: int, limit: Optional[int] = None):
        cap = 256
        out = (GxService * cap)()
        n = C.c_uint32()
        lim = LIMIT_DEFAULT if limit is None else int(limit)
        check(self.lib.gx_get_broadcasts(self.h, host, lim, out, cap, C.byref(n)), "gx_get_broadcasts")
        if n.value == 0:
            return None
        return [out[i] for i in range(n.value)]

    def get_broadcasts_bytes(self, host: int, overhead: int, limit: int, cap: Optional[int] = None):
        """GetBroadcasts(overhead, limit) with the reference's byte limit; None = nil."""
        cap = 1024 if cap is None else int(cap)
        out = (GxService * max(1, cap))()
        n = C.c_uint32()
        check(self.lib.gx_get_broadcasts_bytes(self.h, host, overhead, limit, out, cap, C.byref(n)),
              "gx_get_broadcasts_bytes")
        if n.value == 0:
            return None
        return [out[i] for i in range(n.value)]

    def set_static_bytes(self, owner_lo: int, owner_hi: int, nbytes):
        a = np.ascontiguousarray(np.asarray(nbytes, dtype=np.uint16).reshape(-1))
        assert a.size == (owner_hi - owner_lo) * self.S
        check(self.lib.gx_set_static_bytes(self.h, owner_lo, owner_hi,
                                           a.ctypes.data_as(C.POINTER(C.c_uint16))), "gx_set_static_bytes")

    def message_bytes(self, recs):
        """len(Service.Encode()) of each record (service/service_ffjson.go:370-436)."""
        n = len(recs)
        out = (C.c_uint32 * max(1, n))()
        check(self.lib.gx_message_bytes(self.h, svc_array(recs), n, out), "gx_message_bytes")
        return [out[i] for i in range(n)]

    def local_state(self, view: int):
        n = C.c_uint32()
        check(self.lib.gx_local_state(self.h, view, None, 0, C.byref(n)))
        cap = max(1, n.value)
        out = (GxService * cap)()
        check(self.lib.gx_local_state(self.h, view, out, cap, C.byref(n)))
        return [out[i] for i in range(n.value)]

    # full-state JSON codec ------------------------------------------------
    def set_names(self, names) -> None:
        """gx_set_names from a sidecar_amd.codec.Names."""
        hosts, hoff = names._blob(names.hosts)
        ids, ioff = names._blob(names.ids)
        pre, poff = names._blob(names.pre)
        post, qoff = names._blob(names.post)
        self._names_keep = (hosts, hoff, ids, ioff, pre, poff, post, qoff, names.cluster_name)
        nm = GxNames(names.cluster_name, len(names.cluster_name), hosts, hoff.ctypes.data, ids, ioff.ctypes.data,
                     pre, poff.ctypes.data, post, qoff.ctypes.data)
        check(self.lib.gx_set_names(self.h, C.byref(nm)), "gx_set_names")

    def local_state_json(self, view: int) -> bytes:
        """LocalState(): the view's ServicesState JSON (services_delegate.go:146-151)."""
        n = C.c_uint64()
        check(self.lib.gx_local_state_json(self.h, view, None, 0, C.byref(n)), "gx_local_state_json")
        buf = C.create_string_buffer(max(1, n.value))
        check(self.lib.gx_local_state_json(self.h, view, buf, n.value, C.byref(n)), "gx_local_state_json")
        return buf.raw[:n.value]

    def decode_state_json(self, data: bytes, cap: Optional[int] = None):
        """catalog.Decode(): (rc, records in document order, decode stats)."""
        cap = (len(data) // 64 + 16) if cap is None else cap
        out = (GxService * max(1, cap))()
        n = C.c_uint32()
        ds = GxDecodeStats()
        rc = self.lib.gx_decode_state_json(self.h, data, len(data), out, cap, C.byref(n), C.byref(ds))
        return rc, [out[i].tup() for i in range(min(n.value, cap))], ds.as_dict()

    def merge_remote_state_json(self, view: int, data: bytes):
        """MergeRemoteState(buf): (rc, decode stats)."""
        ds = GxDecodeStats()
        rc = self.lib.gx_merge_remote_state_json(self.h, view, data, len(data), C.byref(ds))
        return rc, ds.as_dict()

    def notify_leave(self, view: int, node: int):
        check(self.lib.gx_notify_leave(self.h, view, node))

    # read-back -------------------------------------------------------------------------
    def read_views(self, lo: Optional[int] = None, hi: Optional[int] = None) -> np.ndarray:
        lo = self.lo if lo is None else lo
        hi = self.hi if hi is None else hi
        out = np.empty((hi - lo, self.H * self.S), dtype=np.uint64)
        check(self.lib.gx_read_views(self.h, lo, hi, out.ctypes.data_as(C.c_void_p)), "gx_read_views")
        return out

    def write_views(self, words: np.ndarray, lo: int = 0):
        words = np.ascontiguousarray(words, dtype=np.uint64)
        hi = lo + words.shape[0]
        check(self.lib.gx_write_views(self.h, lo, hi, words.ctypes.data_as(C.c_void_p)), "gx_write_views")

    def write_slot(self, view: int, item):
        check(self.lib.gx_write_slot(self.h, view, svc_array([item])), "gx_write_slot")

    def slot(self, view: int, host: int, s: int):
        """(updated_ns, status) of one slot, or None if absent."""
        row = self.read_views(view, view + 1)[0]
        w = int(row[host * self.S + s])
        if w & 7 == ABSENT:
            return None
        return (self.word_time(w), w & 7)

    def hosts(self, lo=None, hi=None):
        lo = self.lo if lo is None else lo
        hi = self.hi if hi is None else hi
        out = (GxHostState * max(1, hi - lo))()
        check(self.lib.gx_read_hosts(self.h, lo, hi, out))
        return [out[i] for i in range(hi - lo)]

    def queue(self, host: int):
        n = C.c_uint32()
        check(self.lib.gx_read_queue(self.h, host, None, 0, C.byref(n)))
        out = (GxJob * max(1, n.value))()
        check(self.lib.gx_read_queue(self.h, host, out, n.value, C.byref(n)))
        return [out[i] for i in range(n.value)]

    def sleepers(self, host: int):
        n = C.c_uint32()
        check(self.lib.gx_read_sleepers(self.h, host, None, 0, C.byref(n)))
        out = (GxSleeper * max(1, n.value))()
        check(self.lib.gx_read_sleepers(self.h, host, out, n.value, C.byref(n)))
        return [out[i] for i in range(n.value)]

    def pending(self, host: int):
        out = (GxService * 1024)()
        n = C.c_uint32()
        check(self.lib.gx_read_pending(self.h, host, out, 1024, C.byref(n)))
        return [out[i] for i in range(min(n.value, 1024))]

    def read_list(self, host: int, slot: int):
        out = (GxService * 1024)()
        n = C.c_uint32()
        check(self.lib.gx_read_list(self.h, host, slot, out, 1024, C.byref(n)))
        return [out[i] for i in range(min(n.value, 1024))]

    def each_service_sorted(self, view: int, owner: int = ALL_OWNERS) -> list:
        """EachServiceSorted (catalog/view.go:14-26), or one server's SortedServices (:48-58)."""
        n = C.c_uint32()
        check(self.lib.gx_each_service_sorted(self.h, view, owner, None, 0, C.byref(n)), "gx_each_service_sorted")
        out = (GxService * max(1, n.value))()
        check(self.lib.gx_each_service_sorted(self.h, view, owner, out, n.value, C.byref(n)), "gx_each_service_sorted")
        return [out[i] for i in range(n.value)]

    def set_service_names(self, names) -> None:
        """Service.Name of every record r = host * S + svc (a list of R str/bytes)."""
        bs = [x.encode() if isinstance(x, str) else bytes(x) for x in names]
        assert len(bs) == self.H * self.S
        off = np.zeros(len(bs) + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(b) for b in bs])
        blob = b"".join(bs) or b"\0"
        check(self.lib.gx_set_service_names(self.h, blob, off.ctypes.data_as(C.POINTER(C.c_uint64))),
              "gx_set_service_names")

    def by_service(self, view: int):
        """ByService (services_state.go:738-748): [(group, record)] in group order."""
        n = C.c_uint32()
        check(self.lib.gx_by_service(self.h, view, None, None, 0, C.byref(n)), "gx_by_service")
        out = (GxService * max(1, n.value))()
        grp = (C.c_uint32 * max(1, n.value))()
        check(self.lib.gx_by_service(self.h, view, out, grp, n.value, C.byref(n)), "gx_by_service")
        return [(grp[i], out[i]) for i in range(n.value)]

    def server_times(self, view: int, lo: int = 0, hi: Optional[int] = None) -> np.ndarray:
        """Server.LastUpdated / LastChanged of owners [lo, hi) in `view`: int64 [n, 2]."""
        hi = self.H if hi is None else hi
        out = np.empty((hi - lo, 2), dtype=np.int64)
        check(self.lib.gx_read_server_times(self.h, view, lo, hi, out.ctypes.data_as(C.c_void_p)),
              "gx_read_server_times")
        return out

    def last_changed(self, lo: Optional[int] = None, hi: Optional[int] = None) -> np.ndarray:
        """state.LastChanged of views [lo, hi)."""
        lo = self.lo if lo is None else lo
        hi = self.hi if hi is None else hi
        out = np.empty(hi - lo, dtype=np.int64)
        check(self.lib.gx_read_last_changed(self.h, lo, hi, out.ctypes.data_as(C.c_void_p)),
              "gx_read_last_changed")
        return out

    def add_listener(self, view: int, lid: int, capacity: int):
        check(self.lib.gx_add_listener(self.h, view, lid, capacity), "gx_add_listener")

    def remove_listener(self, view: int, lid: int) -> int:
        return self.lib.gx_remove_listener(self.h, view, lid)

    def drain_listener(self, view: int, lid: int, cap: int = 4096):
        out = (GxChangeEvent * max(1, cap))()
        n = C.c_uint32()
        check(self.lib.gx_listener_drain(self.h, view, lid, out, cap, C.byref(n)), "gx_listener_drain")
        return [out[i] for i in range(n.value)]

    def digests(self) -> np.ndarray:
        out = np.empty(self.hi - self.lo, dtype=np.uint64)
        check(self.lib.gx_host_digests(self.h, out.ctypes.data_as(C.c_void_p)), "gx_host_digests")
        return out

    def stats(self) -> dict:
        s = GxStats()
        check(self.lib.gx_stats_get(self.h, C.byref(s)))
        return s.as_dict()

    def timing(self) -> dict:
        t = GxTiming()
        check(self.lib.gx_timing_get(self.h, C.byref(t)))
        return t.as_dict()

    # sharded rounds (phase API; buffers are addresses: device memory for the HIP engine) -----
    def round_send(self):
        check(self.lib.gx_round_send(self.h), "gx_round_send")

    def outbox_bytes(self) -> np.ndarray:
        out = np.zeros(self.G, dtype=np.uint64)
        check(self.lib.gx_outbox_bytes(self.h, out.ctypes.data_as(C.c_void_p)), "gx_outbox_bytes")
        return out

    def exchange_plan(self) -> np.ndarray:
        """(G, G) bytes shard s sends shard g this round in the planned exchange (gx.h)."""
        G = max(1, self.params.n_shards)
        out = np.zeros(G * G, dtype=np.uint64)
        check(self.lib.gx_exchange_plan(self.h, out.ctypes.data_as(C.c_void_p)), "gx_exchange_plan")
        return out.reshape(G, G)

    def xplan_waits(self):
        """(calls of gx_exchange_plan that waited on the host for their batch, all calls): a
        diagnostics symbol of the HIP engine, not in gx.h."""
        out = (C.c_uint64 * 2)()
        check(self.lib.gx_xplan_waits(self.h, out), "gx_xplan_waits")
        return int(out[0]), int(out[1])

    def outbox_pack_planned(self, ptr: int, cap: int):
        check(self.lib.gx_outbox_pack_planned(self.h, C.c_void_p(ptr), C.c_uint64(cap)), "gx_outbox_pack_planned")

    def outbox_sizes_async(self, ptr: int):
        """Per-shard outbox bytes into engine memory at ptr (device memory on the HIP engine)."""
        check(self.lib.gx_outbox_sizes_async(self.h, C.c_void_p(ptr)), "gx_outbox_sizes_async")

    def outbox_pack(self, ptr: int, cap: int):
        check(self.lib.gx_outbox_pack(self.h, C.c_void_p(ptr), cap), "gx_outbox_pack")

    def inbox_unpack(self, ptr: int, nbytes: int):
        check(self.lib.gx_inbox_unpack(self.h, C.c_void_p(ptr), nbytes), "gx_inbox_unpack")

    def round_merge(self):
        check(self.lib.gx_round_merge(self.h), "gx_round_merge")

    def round_gossip_begin(self, plan: np.ndarray, ptr: int, cap: int):
        """round_send + exchange_plan (into `plan`, G*G uint64) + outbox_pack_planned in one call."""
        check(self.lib.gx_round_gossip_begin(self.h, plan.ctypes.data_as(C.c_void_p), C.c_void_p(ptr),
                                             C.c_uint64(cap)), "gx_round_gossip_begin")

    def round_gossip_end(self, ptr: int, nbytes: int) -> bool:
        """inbox_unpack + round_merge, then round_end unless this is a push-pull round (returns True:
        the caller runs the push-pull steps and round_end)."""
        ae = C.c_int(0)
        check(self.lib.gx_round_gossip_end(self.h, C.c_void_p(ptr), C.c_uint64(nbytes), C.byref(ae)),
              "gx_round_gossip_end")
        return bool(ae.value)

    def ae_bytes(self) -> np.ndarray:
        out = np.zeros(self.G, dtype=np.uint64)
        check(self.lib.gx_ae_bytes(self.h, out.ctypes.data_as(C.c_void_p)), "gx_ae_bytes")
        return out

    def ae_pack(self, ptr: int, cap: int):
        check(self.lib.gx_ae_pack(self.h, C.c_void_p(ptr), cap), "gx_ae_pack")

    def ae_delta_bytes(self, ptr: int, nbytes: int) -> np.ndarray:
        """Compare the received push-pull digests with this shard's; lead-message sizes per shard."""
        out = np.zeros(self.G, dtype=np.uint64)
        check(self.lib.gx_ae_delta_bytes(self.h, C.c_void_p(ptr), nbytes, out.ctypes.data_as(C.c_void_p)),
              "gx_ae_delta_bytes")
        return out

    def ae_delta_pack(self, ptr: int, cap: int):
        check(self.lib.gx_ae_delta_pack(self.h, C.c_void_p(ptr), cap), "gx_ae_delta_pack")

    def ae_return_bytes(self, ptr: int, nbytes: int) -> np.ndarray:
        """Received lead blocks -> sizes of the return messages per shard."""
        out = np.zeros(self.G, dtype=np.uint64)
        check(self.lib.gx_ae_return_bytes(self.h, C.c_void_p(ptr), nbytes, out.ctypes.data_as(C.c_void_p)),
              "gx_ae_return_bytes")
        return out

    def ae_return_pack(self, lead_ptr: int, lead_bytes: int, ptr: int, cap: int):
        check(self.lib.gx_ae_return_pack(self.h, C.c_void_p(lead_ptr), lead_bytes, C.c_void_p(ptr), cap),
              "gx_ae_return_pack")

    def ae_merge(self, lead_ptr: int = 0, lead_bytes: int = 0, ret_ptr: int = 0, ret_bytes: int = 0):
        check(self.lib.gx_ae_merge(self.h, C.c_void_p(lead_ptr), lead_bytes, C.c_void_p(ret_ptr), ret_bytes),
              "gx_ae_merge")

    def is_ae_round(self) -> bool:
        """This round is a push-pull round (every shard agrees: the schedule is global)."""
        p = self.params
        return bool(p.ae_period_rounds) and self.round % p.ae_period_rounds == p.ae_phase

    def set_stream(self, stream_ptr, async_phases: bool):
        """Run this engine's device work on the caller's HIP stream (0 = the default stream; None =
        the engine's own); with async_phases the sharded phase calls return once queued (gx.h)."""
        mode = (1 | (2 if async_phases else 0)) if stream_ptr is not None else 0  # gx.h GX_STREAM_*
        check(self.lib.gx_set_stream(self.h, C.c_void_p(stream_ptr or None), mode), "gx_set_stream")

    def ae_merge_local(self):
        """Start this shard's local push-pull pairs (asynchronous; overlaps the row exchange)."""
        check(self.lib.gx_ae_merge_local(self.h), "gx_ae_merge_local")

    def round_end(self):
        check(self.lib.gx_round_end(self.h), "gx_round_end")

    def lock_census(self) -> int:
        """This shard's hosts that do not hold the ServicesState lock this round (gx_lock_census)."""
        n = C.c_uint32(0)
        check(self.lib.gx_lock_census(self.h, C.byref(n)), "gx_lock_census")
        return int(n.value)

    def ae_skip_locked(self):
        """A push-pull round with every host of the cluster locked: its counts only (gx_ae_skip_locked)."""
        check(self.lib.gx_ae_skip_locked(self.h), "gx_ae_skip_locked")

    def view_minmax(self, ptr_min: int, ptr_max: int):
        check(self.lib.gx_view_minmax(self.h, C.c_void_p(ptr_min), C.c_void_p(ptr_max)), "gx_view_minmax")

    def owner_words(self, ptr: int):
        """R words at ptr (device memory for the HIP engine): each record's word in its owner's view."""
        check(self.lib.gx_owner_words(self.h, C.c_void_p(ptr)), "gx_owner_words")

    # memberlist failure detection ---------------------------------------------
    def fd_members(self, host: int, lo: int = 0, hi: Optional[int] = None) -> bytes:
        hi = self.H if hi is None else hi
        out = (GxMember * max(1, hi - lo))()
        check(self.lib.gx_fd_read_members(self.h, host, lo, hi, out), "gx_fd_read_members")
        return bytes(out)[:C.sizeof(GxMember) * (hi - lo)]

    def fd_member(self, host: int, node: int) -> GxMember:
        m = GxMember()
        check(self.lib.gx_fd_read_members(self.h, host, node, node + 1, C.byref(m)), "gx_fd_read_members")
        return m

    def fd_hosts(self, lo: int = 0, hi: Optional[int] = None):
        hi = self.H if hi is None else hi
        out = (GxFdHost * max(1, hi - lo))()
        check(self.lib.gx_fd_read_hosts(self.h, lo, hi, out), "gx_fd_read_hosts")
        return [out[i] for i in range(hi - lo)]

    def fd_queue(self, host: int, cap: int = 65536):
        out = (GxFdMsg * cap)()
        tx = (C.c_uint8 * cap)()
        n = C.c_uint32()
        check(self.lib.gx_fd_read_queue(self.h, host, out, tx, cap, C.byref(n)), "gx_fd_read_queue")
        return [(out[i].tup(), tx[i]) for i in range(min(n.value, cap))]

    def fd_notify(self, host: int, msgs: Sequence):
        arr = (GxFdMsg * max(1, len(msgs)))(*[m if isinstance(m, GxFdMsg) else fd_msg(*m) for m in msgs])
        check(self.lib.gx_fd_notify(self.h, host, arr, len(msgs)), "gx_fd_notify")

    def fd_get_broadcasts(self, host: int, limit: int):
        out = (GxFdMsg * max(1, limit))()
        n = C.c_uint32()
        check(self.lib.gx_fd_get_broadcasts(self.h, host, limit, out, C.byref(n)), "gx_fd_get_broadcasts")
        return [out[i].tup() for i in range(n.value)]

    def fd_probe(self, host: int):
        t, ack = C.c_uint32(), C.c_int()
        check(self.lib.gx_fd_probe(self.h, host, C.byref(t), C.byref(ack)), "gx_fd_probe")
        return (None if t.value == FD_NONE else t.value), bool(ack.value)

    def fd_timers(self, host: int):
        check(self.lib.gx_fd_timers(self.h, host), "gx_fd_timers")

    def fd_merge_state(self, host: int, remote: Sequence):
        """pushPull's mergeState on `host`; remote[m] = (state, incarnation) or None (not listed)."""
        arr = np.array([0xFF if x is None else (int(x[1]) << 32) | int(x[0]) for x in remote], dtype=np.uint64)
        assert arr.size == self.H
        check(self.lib.gx_fd_merge_state(self.h, host, arr.ctypes.data), "gx_fd_merge_state")

    def fd_converged(self):
        c = C.c_int()
        n = C.c_uint64()
        check(self.lib.gx_fd_converged(self.h, C.byref(c), C.byref(n)), "gx_fd_converged")
        return bool(c.value), n.value

    def converged(self):
        c = C.c_int()
        n = C.c_uint64()
        check(self.lib.gx_converged(self.h, C.byref(c), C.byref(n)))
        return bool(c.value), n.value

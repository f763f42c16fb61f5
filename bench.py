"""Benchmark: record-merges/sec and rounds-to-converge wall time of the gossip-convergence engine.

A step is one gossip round of the seeded schedule (DESIGN.md "Round model"). The default workload
is BASELINE.json's headline configuration, H=32768 hosts x S=16 services (cfg 5): a converged
catalog is split into two halves for 50 rounds, every host NotifyLeave()s the other half after 5
rounds (ExpireServer storm), the partition heals, and memberlist push-pull anti-entropy runs every
10 rounds. All state is resident in HBM; the timed region is `gx_run_rounds(K)`.

  python bench.py [--gpus N --steps K --warmup W] [--config cfg5|cfg2|cfg3|cfg4] [--no-converge]

Prints ONE JSON line (rank 0). N>1 runs one process per GPU (torch.distributed.run): the same
cluster is sharded by host block over the N GPUs. Every round's cross-shard packets,
and on push-pull rounds the row digests and the differing row blocks, move by RCCL all-to-all over
xGMI, so the total work is fixed (strong scaling); `exchange` reports the bytes moved. Results are
bit-identical to the 1-GPU run.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "record-merges/sec (whole node) + rounds-to-converge wall time, H=32768 S=16"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)

# queue_cap: the broadcast FIFO's stored window per host (gx.h gx_job). The reference's queue is
# unbounded; the engine stores the first queue_cap jobs and counts the rest in place, and a run stays
# faithful to the reference's queue while no deferred job reaches the head, which takes at least
# queue_cap / (fanout * GossipMessages) rounds after the window first fills: 16384 / 3 = 5461 rounds,
# 20480 / 3 = 6826 (cfg 5 also stores the storm's 16384 ExpireServer jobs per host), 139264 / 45 =
# 3094 rounds at GossipMessages 15 (71 GB at H = 32768), all past --converge-max 3000.
Q_GM1 = 16384
# uniformly random 8-B gathers over a 137 GB table on MI355X (profiles/r04/gather_bench.hip; a
# read-modify-write of the slot runs at the same rate, a blind scatter at 2.8e10/s)
# 128-B view lines per second when every access is a run of 16 consecutive 8-B slots of a random
# line (profiles/r04/gather_bench.jsonl, gather_run16: 6.379e11 words/s over a 137 GB table)
LINE_CEILING_PER_S = 6.379e11 / 16
CONFIGS = {
    # BASELINE.json configs[4]: 32768 x 16, 2-way partition for 50 rounds, departure storm, heal
    "cfg5": dict(desc="32768 hosts x 16 services, fanout 3, cap 32 records/msg, 2-way partition rounds "
                      "[0,50) + ExpireServer storm at round 5 + heal",
                 p=dict(n_hosts=32768, n_services=16, fanout=3, packet_cap=32, pending_cap=100,
                        queue_cap=20480, list_slots=32, init_mode=2, partition_start=0,
                        partition_end=50, storm_round=5, ae_period_rounds=10),
                 # to ~12,000 rounds: past the first unlock (~5,460) and the relock, inside the stored
                 # window's lossless horizon (~12,300)
                 converge=dict(max_rounds=12000),
                 ref_variant="cfg5_ref"),
    # cfg 5 at the reference's own anti-entropy cadence: PushPullInterval 20 s (config/config.go:45,
    # main.go:252-256) = 100 rounds of GossipInterval 200 ms; reported beside cfg5 for its
    # rounds-to-converge
    "cfg5_ref": dict(desc="cfg5 at Sidecar's default PushPullInterval 20 s: 32768 hosts x 16 services, fanout 3, "
                          "cap 32 records/msg, 2-way partition rounds [0,50) + ExpireServer storm at round 5 + heal",
                     p=dict(n_hosts=32768, n_services=16, fanout=3, packet_cap=32, pending_cap=100,
                            queue_cap=20480, list_slots=32, init_mode=2, partition_start=0,
                            partition_end=50, storm_round=5, ae_period_rounds=100)),
    # cfg 5 at Sidecar's own defaults (config/config.go:45-47, main.go:252-259): PushPullInterval 20 s
    # (100 rounds) and GossipMessages 15 (up to 15 GetBroadcasts packets per gossip target per round)
    "cfg5_defaults": dict(desc="cfg5 at Sidecar's defaults (PushPullInterval 20 s, GossipMessages 15): 32768 hosts "
                               "x 16 services, fanout 3, cap 32 records/msg, 2-way partition rounds [0,50) + "
                               "ExpireServer storm at round 5 + heal",
                          p=dict(n_hosts=32768, n_services=16, fanout=3, packet_cap=32, pending_cap=100,
                                 queue_cap=139264, list_slots=32, init_mode=2, partition_start=0,
                                 partition_end=50, storm_round=5, ae_period_rounds=100, gossip_messages=15)),
    # configs[1]: 4096 x 16, fanout 3, cap 32, one GPU (cold start: every view knows its own records)
    "cfg2": dict(desc="4096 hosts x 16 services, fanout 3, cap 32 records/msg, own-records start, "
                      "push-pull every 10 rounds",
                 p=dict(n_hosts=4096, n_services=16, fanout=3, packet_cap=32, queue_cap=Q_GM1,
                        list_slots=32, init_mode=1, ae_period_rounds=10),
                 converge=dict(max_rounds=60000, over=dict(queue_cap=1 << 20))),
    # configs[2]: 16384 x 16 with 5% churn/round and alive-lifespan expiry
    "cfg3": dict(desc="16384 hosts x 16 services, 5% of owners start/stop a service per round, 5% of "
                      "records aged U[0,100s] (alive-lifespan expiry), push-pull every 10 rounds",
                 p=dict(n_hosts=16384, n_services=16, fanout=3, queue_cap=Q_GM1, list_slots=32, init_mode=2,
                        churn_ppm=50000, aged_ppm=50000, ae_period_rounds=10)),
    # configs[3]: 8192 x 64, push-pull every 10 rounds
    "cfg4": dict(desc="8192 hosts x 64 services, push-pull full-state merge every 10 rounds",
                 p=dict(n_hosts=8192, n_services=64, fanout=3, queue_cap=Q_GM1, list_slots=32, init_mode=1,
                        ae_period_rounds=10),
                 converge=dict(max_rounds=60000, over=dict(queue_cap=1 << 20))),
    # cfg 5 driven by memberlist's failure detector instead of the scripted storm:
    # the partition drops packets, SWIM probes suspect the other half, Lifeguard timers decide
    # (for a 10 s partition at this size they do not expire: refutations win after the heal)
    "cfg5fd": dict(desc="cfg5 with memberlist failure detection: 32768 hosts x 16 services, 2-way network "
                        "partition rounds [0,50), SWIM probes + Lifeguard suspicion, NotifyLeave -> "
                        "ExpireServer, push-pull every 10 rounds",
                   p=dict(n_hosts=32768, n_services=16, fanout=3, packet_cap=32, pending_cap=100,
                          queue_cap=20480, list_slots=32, init_mode=2, partition_start=0,
                          partition_end=50, ae_period_rounds=10, fd_enable=1)),
    # host crashes detected by the failure detector: 2% of 16384 hosts crash at round 5
    "fd_depart": dict(desc="16384 hosts x 16 services, 2% of hosts crash at round 5, memberlist failure "
                           "detection (SWIM + Lifeguard) -> NotifyLeave -> ExpireServer, push-pull every 10 rounds",
                      p=dict(n_hosts=16384, n_services=16, fanout=3, queue_cap=Q_GM1, list_slots=32, init_mode=2,
                             ae_period_rounds=10, fd_enable=1, depart_round=5, depart_ppm=20000)),
    # plumbing case of the failure detector (CPU rehearsal of the sharded path)
    "cfg1fd": dict(desc="64 hosts x 8 services, fanout 3, 10% of hosts crash at round 5, memberlist failure "
                        "detection, push-pull every 10 rounds",
                   p=dict(n_hosts=64, n_services=8, fanout=3, queue_cap=4096, init_mode=2, ae_period_rounds=10,
                          fd_enable=1, depart_round=5, depart_ppm=100000)),
    # small plumbing case (configs[0]); also the CPU-baseline scale model
    "cfg1": dict(desc="64 hosts x 8 services, fanout 3", p=dict(n_hosts=64, n_services=8, fanout=3,
                                                                queue_cap=4096, init_mode=0)),
}

KNAMES = ["owner", "scan", "storm", "send", "route", "merge", "ae", "converge", "encode", "decode", "fd"]
GOSSIP_KERNELS = ("owner", "scan", "send", "merge")  # the kernels every gossip round runs


def workload_text(cfg):
    """Config description with the anti-entropy cadence and pairing spelled out."""
    c = CONFIGS[cfg]
    p = c["p"]
    ae = p.get("ae_period_rounds", 0)
    if ae:
        pairing = ("per-node initiation (every live host starts one exchange with a random peer)"
                   if p.get("push_pull_mode", 0) else
                   "seeded perfect matching (every host in exactly one exchange per push-pull round)")
        cad = f"push-pull every {ae} rounds ({ae * 0.2:g} s), {pairing}"
    else:
        cad = "no push-pull"
    gm = p.get("gossip_messages", 0)
    gms = f", GossipMessages {gm}" if gm > 1 else ""
    return f"{cfg}: {c['desc']}; {cad}{gms}"


def make_engine(lib, cfg, seed, device, **over):
    from sidecar_amd.abi import Engine, default_params
    p = default_params(lib, **dict(CONFIGS[cfg]["p"], **over))
    p.seed = seed
    p.device = device
    return Engine(p, lib=lib)


def merges(st):
    return st["gossip_merges"] + st["ae_merges"] + st["local_merges"]


def queue_report(cfg, st0, st1, queue_cap=None):
    """The broadcast queues over a run (gx.h gx_job): jobs deferred past the stored window, jobs LOST
    (deferred jobs GetBroadcasts reached: the reference would have sent them), the first round of a
    LOST dequeue, SendServices lists that did not fit, sleep-ring overflow, and the reference's own
    MAX_PENDING_LENGTH truncation (services_delegate.go:109-120, not a deviation). faithful: no job
    the reference would deliver was lost (every packet and looper state is the reference's)."""
    p = dict(CONFIGS[cfg]["p"])
    if queue_cap:
        p["queue_cap"] = queue_cap  # the run's own stored window (a converge run may widen it)
    ke = p.get("fanout", 3) * max(1, p.get("gossip_messages", 0))
    d = {k: st1[k] - (st0[k] if st0 else 0) for k in ("queue_deferred", "queue_drops", "list_drops", "sleep_drops",
                                                       "pending_drops", "retransmits", "dequeues",
                                                       "locked_merges")}
    # faithful: no job the reference would deliver was lost, and no merge ran on a host whose
    # looper held the ServicesState lock (locked_merges, only with lock_model = 0; gx.h)
    return {"window_jobs_per_host": p["queue_cap"], "lossless_rounds_after_fill": p["queue_cap"] // ke,
            "retransmits": d["retransmits"], "dequeues": d["dequeues"], "deferred": d["queue_deferred"],
            "lost": d["queue_drops"], "first_lost_round": st1["first_drop_round"], "list_drops": d["list_drops"],
            "sleep_drops": d["sleep_drops"], "pending_truncated": d["pending_drops"],
            "locked_merges": d["locked_merges"],
            "faithful": d["queue_drops"] == 0 and d["sleep_drops"] == 0 and d["locked_merges"] == 0}


def expiry_report(st0, st1):
    """Alive-lifespan expiries over a run (TombstoneOthersServices, services_state.go:655-679), and
    the false ones: expiries of records whose owner host is live (gx.h false_expiries). A faithful
    steady-state figure where the catalog never agrees bit for bit: live owners restamp every 60 s
    (services_state.go:547) and a view that has not heard a refresh for ALIVE_LIFESPAN (80 s) tombstones
    the record."""
    return {k: st1[k] - (st0[k] if st0 else 0) for k in ("expired", "false_expiries")}


def merges_by_source(st0, st1):
    """Record-merges of the window by where the record came from: gossip packets merged on arrival,
    records that waited in a locked host's inbound pipeline (merged at its unlock), push-pull Merge of
    a partner's full state, and the owners' own TrackNewServices merges."""
    d = {k: st1[k] - st0[k] for k in ("gossip_merges", "ae_merges", "local_merges", "lock_drained")}
    return {"gossip_packets": d["gossip_merges"] - d["lock_drained"], "lock_pipeline_drained": d["lock_drained"],
            "push_pull": d["ae_merges"], "owner_local": d["local_merges"]}


def device_time_share(kern):
    """Each kernel class's share of the window's device time (the per-launch-event pass); says what
    the headline's wall time is spent on (e.g. the ExpireServer storm, not merging)."""
    if not kern:
        return None
    tot = sum(v["ms"] for v in kern.values())
    return {k: round(v["ms"] / tot, 4) for k, v in sorted(kern.items(), key=lambda kv: -kv[1]["ms"])} if tot else None


def lock_report(p, st0, st1, hosts=None, rnd=None):
    """The ServicesState lock held by a blocked looper (gx.h lock_model) over a run:
    records held in locked hosts' inbound pipelines, dropped at a full pipeline (memberlist's handoff
    queue), merged at unlock; push-pull exchanges that did not run; ExpireServer calls that waited;
    with lock_model = 0, the merges that ran on locked hosts anyway (the rounds-1..4 model)."""
    d = {k: st1[k] - (st0[k] if st0 else 0) for k in ("locked_merges", "lock_buffered", "lock_drops",
                                                       "lock_drained", "ae_locked", "expire_deferred")}
    out = {"lock_model": int(p.lock_model), "pipeline_records": int(p.lock_buffer), **d,
           "first_locked_round": st1["first_locked_round"]}
    if hosts is not None:
        out["hosts_locked_at_end"] = sum(h.locked_at(rnd) for h in hosts)
        out["records_held_at_end"] = sum(h.lock_buffered for h in hosts)
    return out


class Cluster:
    """The benchmarked cluster: one engine (N=1) or this rank's shard (N>1, sidecar_amd.dist)."""

    def __init__(self, lib, cfg, seed, rank, world, local_rank, barrier, device=None, **over):
        self.world = world
        self.barrier = barrier
        if world == 1:
            self.e = make_engine(lib, cfg, seed, local_rank, **over)
            self.shard = None
        else:
            from sidecar_amd.dist import DistShard
            kw = dict(CONFIGS[cfg]["p"], **over)
            kw["seed"] = seed
            self.shard = DistShard(lib, rank, world, device or f"cuda:{local_rank}", **kw)
            self.e = self.shard.e

    @property
    def round(self):
        return self.e.round

    def run_rounds(self, n):
        if self.shard is None:
            self.e.run_rounds(n)
        else:
            self.shard.run_rounds(n)

    def stats(self):
        return self.e.stats() if self.shard is None else self.shard.stats()

    def converged(self):
        if self.shard is not None:
            return self.shard.converged()
        ok, n = self.e.converged()
        if ok and self.e.params.fd_enable:
            # with the failure detector, converged also means every live host sees the truth:
            # crashed hosts dead, live hosts alive (no pending suspicion, no false death)
            ok, n = self.e.fd_converged()
        return ok, n

    def exchange_bytes(self):
        """Bytes moved between GPUs by the whole job (summed over ranks); None at N = 1."""
        if self.shard is None:
            return None
        w = self.shard.wire.as_dict()
        keys = sorted(w)
        import torch
        t = torch.tensor([w[k] for k in keys], dtype=torch.int64, device=self.shard.device)
        self.shard._all_reduce(t, self.shard.dist.ReduceOp.SUM)
        return dict(zip(keys, [int(x) for x in t.tolist()]))

    def close(self):
        if self.shard is not None:
            self.shard.close()  # drains the engine's streams before the process group goes
        else:
            self.e.close()


def gossip_stretch_start(cfg, accepting=False):
    """First round of a stretch of 9 gossip-only rounds (no storm, no push-pull): by default the
    second such stretch after the storm (rounds 21..29 of cfg 5: every record gossiped there is
    already held, the senders' filter drops all of it); `accepting`: the first stretch after the
    heal (rounds 51..59 of cfg 5), where the heal's push-pull accepts are retransmitted and gossip
    records are live. None when the config has no partition (accepting)."""
    p = CONFIGS[cfg]["p"]
    period = p.get("ae_period_rounds", 0)
    phase = p.get("ae_phase", 0)
    p10 = min(period or 10, 10)

    def has_ae(r0):
        return period and any(r % period == phase for r in range(r0, r0 + p10 - 1))

    if accepting:
        if not p.get("partition_end", 0):
            return None
        s = p["partition_end"] + 1
    else:
        s = phase + 1  # the round after a push-pull round, past the storm, then one stretch later
        while s <= p.get("storm_round", -1):
            s += p10
        s += p10
    while has_ae(s):
        s += 1
    return s


def gossip_round_span(lib, cfg, seed, local_rank, start=None, **over):
    """Device time per gossip round without per-launch instrumentation: a stretch of period - 1
    gossip-only rounds from `start` (gossip_stretch_start), bracketed by two events on the engine's
    stream (the caller's torch stream). The per-class split above records an event pair around
    every launch, which adds about 10 us per round. `over`: parameter overrides (lock_model)."""
    import torch
    p = CONFIGS[cfg]["p"]
    period = min(p.get("ae_period_rounds", 0) or 10, 10)
    if start is None:
        start = gossip_stretch_start(cfg)
    e = make_engine(lib, cfg, seed, local_rank, **over)
    e.run_rounds(start - period)
    st = torch.cuda.Stream()  # a stream of its own (launches on the legacy default stream are slower)
    e.set_stream(st.cuda_stream, False)
    n = period - 1
    e.run_rounds(period)  # the first stretch on a new stream starts with ~0.15 ms of queue set-up
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0, u0 = e.stats(), e.timing()["send"]["units"]
    a.record(st)
    e.run_rounds(n)  # (run_rounds ends with one wake-up kernel, ~8 us, inside the span)
    b.record(st)
    b.synchronize()
    s1, u1 = e.stats(), e.timing()["send"]["units"]
    us = 1e3 * a.elapsed_time(b) / n
    e_lock = e.params.lock_model
    e.set_stream(None, False)
    e.close()
    # SURVEY §8(d) algorithmic bytes of a gossip record-merge: 22 B (inbound record 13 + slot 9)
    # + 9 B per accept + 13 B per retransmit queued; the stretch holds gossip rounds only. With the
    # ServicesState lock (gx.h lock_model) a locked receiver's records are not merged that round:
    # each one appended to its inbound pipeline is 13 B read + 13 B written, each one that finds the
    # pipeline full 13 B read (sent, then dropped), so a locked stretch's roofline is not 0 by
    # construction
    m, acc, rx, buf, drop = (s1[k] - s0[k] for k in ("gossip_merges", "gossip_accepts", "retransmits",
                                                       "lock_buffered", "lock_drops"))
    byts = (22 * m + 9 * acc + 13 * rx + 26 * buf + 13 * drop) / n
    gbs = byts / (us * 1e3)
    # Against the lines the round touches: the senders' filter reads each packet's receiver slots,
    # a run of consecutive slots per batch (an ExpireServer batch is one owner's 16 services, one
    # 128-B line of the receiver's row); k_send counts a line wherever a filtered record leaves the
    # previous record's line (gx_timing units). Floor: those lines at the measured rate of random
    # 16-slot runs (gather_run16)
    lines = (u1 - u0) / n
    us_ceil = 1e6 * lines / LINE_CEILING_PER_S
    return round(us, 2), {"bound": "hbm", "scope": "whole gossip round (send + merge kernels), SURVEY 8(d) bytes",
                          "rounds": [start, start + n - 1],
                          "bytes_per_round": int(byts), "merges_per_round": m // n,
                          "accepts_per_round": acc // n, "accept_fraction": round(acc / m, 4) if m else None,
                          "pipeline_appends_per_round": buf // n, "pipeline_drops_per_round": drop // n,
                          "achieved": round(gbs, 1),
                          "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                          "lock_model": int(e_lock),
                          "line_ceiling": {"view_lines_per_round": int(lines),
                                           "ceiling_lines_per_s": LINE_CEILING_PER_S,
                                           "source": "profiles/r04/gather_bench.jsonl (gather_run16)",
                                           "us_per_round_at_ceiling": round(us_ceil, 2),
                                           "frac": round(us_ceil / us, 4) if us and lines else None}}


def dissemination(lib, cfg, seed, local_rank, start=100, rounds=300):
    """Rounds for a catalog change to reach every view (README.md:13-15 "a few seconds"), measured
    on the device from per-record min/max words (gx_view_minmax) after every round of
    [start, start + rounds): a record's version is born in the round its newest word (the max over
    all views) changes, and has spread once every view holds it (min == max). Latency = rounds from
    the birth round to the round after which all views agree. A version replaced by a newer one
    before it spread is counted as superseded; one still spreading at the end, as unfinished."""
    import torch
    e = make_engine(lib, cfg, seed, local_rank)
    try:
        e.run_rounds(start)
        R = e.H * e.S
        dev = torch.device(f"cuda:{local_rank}")
        mn = torch.empty(R, dtype=torch.int64, device=dev)
        mx = torch.empty(R, dtype=torch.int64, device=dev)
        e.view_minmax(mn.data_ptr(), mx.data_ptr())
        prev = mx.clone()
        born = torch.full((R,), -1, dtype=torch.int64, device=dev)
        lats, superseded = [], 0
        for _ in range(rounds):
            r = e.round
            e.run_rounds(1)
            e.view_minmax(mn.data_ptr(), mx.data_ptr())
            new = mx != prev
            superseded += int((new & (born >= 0)).sum().item())
            born = torch.where(new, torch.full_like(born, r), born)
            done = (mn == mx) & (born >= 0)
            lats.append((r - born[done]).cpu())
            born = torch.where(done, torch.full_like(born, -1), born)
            prev.copy_(mx)
        lat = torch.cat(lats).double() if lats else torch.empty(0, dtype=torch.float64)
        out = {"rounds_measured": [start, start + rounds - 1], "changes_spread": int(lat.numel()),
               "superseded": superseded, "unfinished": int((born >= 0).sum().item()),
               "round_s": 0.2, "definition": "rounds from a version's birth round to the round after which "
                                              "every view holds it (per-record min == max over all views)"}
        if lat.numel():
            q = torch.quantile(lat, torch.tensor([0.5, 0.99], dtype=torch.float64))
            out.update({"p50_rounds": float(q[0]), "p99_rounds": float(q[1]), "max_rounds": float(lat.max()),
                        "mean_rounds": round(float(lat.mean()), 2)})
        return out
    finally:
        e.close()


def version_spread(e, dev, heal, end, check_every=10, slots=16):
    """Convergence figure that stays defined while owners keep restamping (Sidecar's 60 s refresh,
    services_state.go:547) and expiry keeps re-tombstoning (:655-679): per record, how long an owner's
    version takes to reach every live view. A view "holds" version T of record r when its word for r
    has Updated >= T (a view's slot time only grows, services_state.go:321, so this is monotone).
      heal:  T = the owner's own word at the heal round; rounds from the heal until every live view
             holds it.
      born:  every version an owner stamps itself after the heal (TrackNewServices / TombstoneServices
             restamp Updated = now, services_state.go:446-453,703): rounds from the check that saw it
             until every live view holds it. A version not held everywhere by `end` is unfinished.
    Checked every `check_every` rounds (per-record min over live views, gx_view_minmax, and the
    owners' words, gx_owner_words), so latencies are multiples of check_every."""
    import torch
    R = e.H * e.S
    i64 = torch.int64
    own = torch.empty(R, dtype=i64, device=dev)
    mn = torch.empty(R, dtype=i64, device=dev)
    mx = torch.empty(R, dtype=i64, device=dev)
    SIGN = -(1 << 63)
    M61 = (1 << 61) - 1

    def ts(w):  # slot time of packed words held in int64 (a logical shift)
        return torch.where((w & 7) == 7, torch.full_like(w, -1), (w >> 3) & M61)  # absent: no version

    def min_ts():
        e.view_minmax(mn.data_ptr(), mx.data_ptr())
        return ts(mn ^ SIGN)  # the min word itself

    e.run_rounds(heal - e.round)
    e.owner_words(own.data_ptr())
    prev = own.clone()
    heal_T = ts(own)
    heal_lat = torch.full((R,), -1, dtype=i64, device=dev)
    pend_T = torch.full((R, slots), 1 << 62, dtype=i64, device=dev)
    pend_b = torch.zeros((R, slots), dtype=i64, device=dev)
    nxt = torch.zeros(R, dtype=i64, device=dev)
    lats, overflow, born = [], 0, 0
    rows = torch.arange(R, device=dev)
    mt = min_ts()
    heal_lat = torch.where((heal_T >= 0) & (mt >= heal_T), torch.zeros_like(heal_lat), heal_lat)
    while e.round < end:
        r0 = e.round
        e.run_rounds(min(check_every, end - e.round))
        e.owner_words(own.data_ptr())
        t0_window = e.params.t0_ns - e.epoch + (r0 + 1) * e.params.round_ns  # stamped by the owner in the window
        new = (own != prev) & (ts(own) >= t0_window)
        prev.copy_(own)
        if bool(new.any()):
            idx = rows[new]
            born += int(idx.numel())
            full = pend_T[idx, nxt[idx] % slots] < (1 << 62)
            overflow += int(full.sum())
            pend_T[idx, nxt[idx] % slots] = ts(own[idx])
            pend_b[idx, nxt[idx] % slots] = e.round
            nxt[idx] += 1
        mt = min_ts()
        done = pend_T <= mt[:, None]
        if bool(done.any()):
            lats.append((e.round - pend_b[done]).cpu())
            pend_T[done] = 1 << 62
        hl = (heal_T >= 0) & (heal_lat < 0) & (mt >= heal_T)
        heal_lat = torch.where(hl, torch.full_like(heal_lat, e.round - heal), heal_lat)

    def q(x):
        if not x.numel():
            return None
        x = x.double()
        qs = torch.quantile(x, torch.tensor([0.5, 0.99], dtype=torch.float64)) if x.numel() < (1 << 24) else \
            torch.tensor([float(x.median()), float(x.kthvalue(max(1, int(0.99 * x.numel())))[0])])
        return {"p50_rounds": float(qs[0]), "p99_rounds": float(qs[1]), "max_rounds": float(x.max())}

    hv = heal_lat[heal_T >= 0].cpu()
    lat = torch.cat(lats) if lats else torch.empty(0, dtype=i64)
    return {"definition": "a view holds version T of a record when its slot's Updated >= T; latency = rounds "
                          "until every live view holds it (checked every %d rounds)" % check_every,
            "rounds": [heal, end],
            "heal_version": dict(q(hv[hv >= 0]) or {}, records=int(hv.numel()), unfinished=int((hv < 0).sum())),
            "born_after_heal": dict(q(lat) or {}, versions=born, spread=int(lat.numel()),
                                    unfinished=int((pend_T < (1 << 62)).sum()), ring_overflow=overflow)}


def run_converge(lib, cfg, seed, rank, world, local_rank, barrier, max_rounds, check_every, device=None,
                 **over):
    """Fresh cluster from round 0: chunks of `check_every` rounds (100 past round 1000; the round is
    taken from the engine's last-change round, so the chunk only bounds when agreement is seen),
    catalog agreement checked between chunks (check time excluded). Returns (rounds_to_converge or
    None, wall_s, rounds run, disagreement samples, queue report, lock report): the samples are the
    records some live views disagree on, every 100 rounds (every 1000 past round 10000). Without
    agreement the lock report carries `steady_state` (steady_state())."""
    c = Cluster(lib, cfg, seed, rank, world, local_rank, barrier, device, **over)
    wall = 0.0
    conv = None
    samples, state = [], []
    st_end = None
    try:
        while c.round < max_rounds:
            barrier()
            t0 = time.perf_counter()
            c.run_rounds(min(check_every if c.round < 1000 else max(check_every, 100), max_rounds - c.round))
            barrier()
            wall += time.perf_counter() - t0
            ok, bad = c.converged()
            if (c.round % 100 == 0 and (c.round <= 10000 or c.round % 1000 == 0)) or ok:
                samples.append([c.round, int(bad)])
                if world == 1 and not ok:
                    hs = c.e.hosts()
                    st = c.stats()
                    depth = [h.fifo_tail - h.fifo_head for h in hs]
                    state.append({"round": c.round, "disagreeing": int(bad),
                                  "hosts_locked": sum(h.locked_at(c.round) for h in hs),
                                  "mean_fifo_depth": sum(depth) / len(depth), "max_fifo_depth": max(depth),
                                  "false_expiries": st["false_expiries"], "ae_exchanges": st["ae_exchanges"],
                                  "queue_drops": st["queue_drops"]})
            if ok:
                lc = c.stats()["last_change_round"]
                conv = lc + 1  # the catalog stopped changing after round lc and agrees
                if CONFIGS[cfg]["p"].get("fd_enable"):
                    conv = max(conv, c.round)  # membership agreement is known at check granularity
                # wall to convergence: the rounds past the convergence point are excluded pro rata
                wall = wall * conv / c.round if c.round else wall
                break
        st_end = c.stats()
        hosts = (c.e.hosts(), c.round) if world == 1 else (None, None)
        lr = lock_report(c.e.params, None, st_end, *hosts)
        lr["expiries"] = expiry_report(None, st_end)
        if conv is None and state:
            lr["steady_state"] = steady_state(state, c.e.params.n_hosts)
        return conv, wall, c.round, samples, queue_report(cfg, None, st_end, c.e.params.queue_cap), lr
    finally:
        c.close()


def steady_state(state, n_hosts):
    """What a run that never agrees settles into, from the samples of its second half: the share of
    hosts whose looper holds the ServicesState lock, broadcast-queue depth, records the views disagree
    on, and the false-expiry and push-pull rates, with each quantity's change between the third and the
    fourth quarter of the run (`drift`, relative): a stationary regime (|drift| small) whose sampled
    state never reaches agreement is the documented answer where rounds-to-converge does not exist."""
    last = state[-1]["round"]
    half = [r for r in state if r["round"] >= last // 2]  # the second half of the run's rounds
    if len(half) < 4:
        return None
    q3, q4 = half[:len(half) // 2], half[len(half) // 2:]

    def mean(rows, k):
        return sum(r[k] for r in rows) / len(rows)

    def rate(rows, k):
        return (rows[-1][k] - rows[0][k]) / max(1, rows[-1]["round"] - rows[0]["round"])

    out = {"rounds": [half[0]["round"], half[-1]["round"]], "samples": len(half),
           "hosts_locked_frac": round(mean(half, "hosts_locked") / n_hosts, 4),
           "hosts_locked_min": min(r["hosts_locked"] for r in half),
           "mean_fifo_depth": round(mean(half, "mean_fifo_depth"), 1),
           "max_fifo_depth": max(r["max_fifo_depth"] for r in half),
           "disagreeing_min": min(r["disagreeing"] for r in half),
           "false_expiries_per_round": round(rate(half, "false_expiries"), 2),
           "push_pull_exchanges_per_round": round(rate(half, "ae_exchanges"), 4),
           "queue_drops": half[-1]["queue_drops"]}
    drift = {}
    for k, f in (("hosts_locked", mean), ("mean_fifo_depth", mean), ("disagreeing", mean)):
        a, b = f(q3, k), f(q4, k)
        drift[k] = round((b - a) / a, 4) if a else None
    a, b = rate(q3, "false_expiries"), rate(q4, "false_expiries")
    drift["false_expiries_per_round"] = round((b - a) / a, 4) if a else None
    out["drift_q3_to_q4"] = drift
    return out


def _oracle_rate(lib, cfg, h_sample, warmup, steps):
    """Merges/s of the oracle over rounds [warmup, warmup + steps) of cfg's schedule at H = h_sample
    (the GPU bench's own round window, so both see the same storm / push-pull / gossip mix)."""
    from sidecar_amd.abi import Engine, default_params
    p = dict(CONFIGS[cfg]["p"])
    p["n_hosts"] = min(p["n_hosts"], h_sample)
    e = Engine(default_params(lib, **p), lib=lib)
    if warmup:
        e.run_rounds(warmup)
    st0 = e.stats()
    t0 = time.perf_counter()
    e.run_rounds(steps)
    dt = time.perf_counter() - t0
    m = merges(e.stats()) - merges(st0)
    e.close()
    return m / dt, dt, p


def cpu_baseline(cfg, warmup, steps, h_mt=16384, h_single=4096):
    """The CPU oracle on a bounded sample of the same workload: the bench's round window of cfg's
    schedule with H scaled down (about 10 s each). The multi-threaded build (per-host phase loops
    on every core this process may use, OpenMP) is the reported baseline; the serial build (the
    reference's one merge goroutine per node, services_state.go:129-135) is reported beside it."""
    import ctypes
    from tests.oracle_lib import load_oracle
    omp = load_oracle(omp=True)
    omp.gx_oracle_threads.restype = ctypes.c_int
    threads = int(omp.gx_oracle_threads())
    v_mt, dt_mt, p = _oracle_rate(omp, cfg, h_mt, warmup, steps)
    v_1, dt_1, p1 = _oracle_rate(load_oracle(), cfg, h_single, warmup, steps)
    win = f"rounds [{warmup}, {warmup + steps})"
    return {"value": v_mt, "unit": "record-merges/s", "cores": threads, "kind": "port",
            "sample": f"oracle/gx_oracle.c built with OpenMP ({threads} threads over hosts), same {cfg} "
                      f"schedule at H={p['n_hosts']} (S={p['n_services']}), {win} in {dt_mt:.1f}s; "
                      f"Go reference unavailable (no Go toolchain on the box)",
            "single_thread": {"value": v_1, "cores": 1,
                              "sample": f"serial oracle at H={p1['n_hosts']}, {win} in {dt_1:.1f}s"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="cfg5", choices=sorted(CONFIGS))
    ap.add_argument("--seed", type=int, default=0x5EED)
    ap.add_argument("--no-converge", action="store_true")
    ap.add_argument("--converge-max", type=int, default=3000)
    ap.add_argument("--check-every", type=int, default=10)
    ap.add_argument("--spread-max", type=int, default=3000, help="last round of the version-spread run")
    ap.add_argument("--no-lock-off", action="store_true",
                    help="skip the same window with lock_model = 0 (the rounds-1..4 model, for comparison)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-split", action="store_true", help="skip the instrumented per-kernel pass")
    ap.add_argument("--cpu-hosts", type=int, default=16384, help="H of the multi-threaded CPU sample")
    # HBM bytes per launch of each kernel class over the window's own launches (profiles/r06/pmc_window.py)
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "r06", "pmc_window.json"))
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    backend = os.environ.get("GX_BENCH_BACKEND", "nccl")  # gloo: rehearsal of N ranks on one GPU
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "gloo":  # ranks share the visible GPUs (collectives staged through the host)
            local_rank %= max(1, torch.cuda.device_count())
        torch.cuda.set_device(local_rank)
        dist.init_process_group(backend)

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    from sidecar_amd.abi import load_product
    lib = load_product()
    seed = args.seed

    # headline window: no per-launch instrumentation inside it (event records are host
    # work inside the wall-clock window)
    c = Cluster(lib, args.config, seed, rank, world, local_rank, barrier)
    if args.warmup:
        c.run_rounds(args.warmup)
    st0 = c.stats()
    x0 = c.exchange_bytes()
    barrier()
    t0 = time.perf_counter()
    c.run_rounds(args.steps)
    barrier()
    dt = time.perf_counter() - t0
    st1 = c.stats()
    x1 = c.exchange_bytes()
    xfer = {k: x1[k] - x0[k] for k in x1} if x1 else None
    lock = lock_report(c.e.params, st0, st1, *((c.e.hosts(), c.round) if world == 1 else (None, None)))
    c.close()

    split = {k: st1[k] - st0[k] for k in ("gossip_merges", "ae_merges", "local_merges")}
    tot_merges = merges(st1) - merges(st0)  # whole cluster (summed over shards)
    dt_max = dt
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt_max = float(t.item())

    # the same window without the ServicesState lock (lock_model = 0, the rounds-1..4 model): merges
    # proceed on hosts whose looper holds the lock; reported for comparison, never the headline
    lock_off = None
    if world == 1 and not args.no_lock_off and c.e.params.lock_model:
        c = Cluster(lib, args.config, seed, rank, world, local_rank, barrier, lock_model=0)
        if args.warmup:
            c.run_rounds(args.warmup)
        s0 = c.stats()
        barrier()
        t0 = time.perf_counter()
        c.run_rounds(args.steps)
        barrier()
        dto = time.perf_counter() - t0
        s1 = c.stats()
        c.close()
        lock_off = {"value": (merges(s1) - merges(s0)) / dto, "ms_per_step": dto * 1000.0 / args.steps,
                    "merges": {k: s1[k] - s0[k] for k in ("gossip_merges", "ae_merges", "local_merges")},
                    "locked_merges": s1["locked_merges"] - s0["locked_merges"],
                    "faithful": s1["locked_merges"] == s0["locked_merges"],
                    "note": "lock_model = 0: merges run on hosts whose BroadcastServices / BroadcastTombstones looper "
                            "holds the ServicesState lock (services_state.go:535,569 / :610,628); not the reference"}

    # per-kernel split: the same window again on a fresh cluster, with HIP events around every
    # launch on the engine's stream (device time per kernel class and algorithmic bytes)
    def kernel_split(**over):
        c = Cluster(lib, args.config, seed, rank, world, local_rank, barrier, **over)
        if args.warmup:
            c.run_rounds(args.warmup)
        c.e.enable_timing(True)
        tm0 = c.e.timing()
        c.run_rounds(args.steps)
        tm1 = c.e.timing()
        c.close()
        out = {}
        for k in KNAMES:
            ms = tm1[k]["ms"] - tm0[k]["ms"]
            nl = tm1[k]["launches"] - tm0[k]["launches"]
            b = tm1[k]["bytes"] - tm0[k]["bytes"]
            if nl:
                out[k] = {"ms": round(ms, 4), "launches": nl, "bytes": b,
                          "GBps": round(b / (ms * 1e6), 1) if ms > 0 else None}
        return out

    kern, kern_off = {}, None
    if not args.no_kernel_split:
        kern = kernel_split()
        if world == 1 and not args.no_lock_off and lock["lock_model"]:
            # the same window without the lock: every push-pull pair and every gossip receiver runs
            # the merge path the locked reference hosts skip (kernel measurement, not the reference)
            kern_off = kernel_split(lock_model=0)
    pmc = {}
    try:
        pmc = json.load(open(args.pmc)).get(args.config, {})
    except Exception:
        pass

    def roofline(k, kern=kern, with_pmc=True):
        if k not in kern or not kern[k]["ms"]:
            return None
        ach = kern[k]["GBps"] or 0.0
        # PMC traffic is measured on the N = 1 run (profiles/r06/pmc_window.json): per launch of the
        # whole engine, so only comparable with this line at N = 1
        traffic = (pmc.get(k) or {}).get("hbm_bytes_per_launch") if world == 1 and with_pmc else None
        return {"bound": "hbm", "kernel": k, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4),
                "bytes_per_launch": kern[k]["bytes"] // max(1, kern[k]["launches"]),
                "us_per_launch": round(1e3 * kern[k]["ms"] / kern[k]["launches"], 2),
                "traffic": traffic}

    dom = max(kern, key=lambda k: kern[k]["ms"]) if kern else None
    roof = roofline(dom) if dom else None
    roof_off = None
    if kern_off:
        dom_off = max(kern_off, key=lambda k: kern_off[k]["ms"])
        roof_off = {"dominant": roofline(dom_off, kern_off, False),
                    **{k: roofline(k, kern_off, False) for k in ("ae", "scan", "send", "merge") if k in kern_off},
                    "note": "lock_model = 0 window: kernel measurement on merges the locked reference hosts "
                            "skip (not the reference)"}
    gossip = None
    if kern:
        gms = sum(kern[k]["ms"] for k in GOSSIP_KERNELS if k in kern)
        gossip = {"kernels": list(GOSSIP_KERNELS), "device_us_per_round": round(1e3 * gms / args.steps, 2),
                  "gossip_merges": split["gossip_merges"],
                  "record_merges_per_s": split["gossip_merges"] / (gms * 1e-3) if gms else None}
        if world == 1:  # without per-launch events: the span of a stretch of gossip-only rounds
            gossip["round_span_us"], gossip["roofline"] = gossip_round_span(lib, args.config, seed, local_rank)
            acc0 = gossip_stretch_start(args.config, accepting=True)
            if acc0 is not None:  # the post-heal stretch, where gossip records are live without the lock
                gossip["round_span_us_accepting"], gossip["roofline_accepting"] = gossip_round_span(
                    lib, args.config, seed, local_rank, start=acc0)
            if not args.no_lock_off and lock["lock_model"]:
                # The same stretches without the lock: where the reference's hosts are locked (their
                # receivers only queue or drop) the kernels still run the whole merge path, which is
                # what these measure (the rounds-1..4 comparison); never the headline
                lo = {"note": "lock_model = 0: kernel measurement on the merge path the locked reference "
                              "hosts skip; not the reference"}
                lo["round_span_us"], lo["roofline"] = gossip_round_span(lib, args.config, seed, local_rank,
                                                                        lock_model=0)
                if acc0 is not None:
                    lo["round_span_us_accepting"], lo["roofline_accepting"] = gossip_round_span(
                        lib, args.config, seed, local_rank, start=acc0, lock_model=0)
                gossip["lock_off"] = lo

    conv = None
    conv_lock_off = None
    if not args.no_converge:
        # a config may follow its converge run further, with a stored FIFO window that keeps it
        # lossless that long (CONFIGS[...]["converge"]; the window's size does not change any result
        # while no job is LOST, gx.h gx_job)
        cv = CONFIGS[args.config].get("converge", {})
        cmax = args.converge_max if args.converge_max != 3000 else cv.get("max_rounds", 3000)
        r, w, ran, dis_s, qr, lr = run_converge(lib, args.config, seed, rank, world, local_rank, barrier,
                                                cmax, args.check_every, **cv.get("over", {}))
        conv = {"rounds_to_converge": r, "converge_wall_s": round(w, 3) if r else None,
                "rounds_run": ran, "simulated_s": (r * 0.2) if r else None, "queues": qr, "lock": lr}
        if r is None:  # how far from agreement the catalog stays (records some live views disagree on)
            conv["disagreeing_records"] = {"min": min(x[1] for x in dis_s) if dis_s else None,
                                           "every_100_rounds": dis_s}
        if world == 1 and not args.no_lock_off and lr["lock_model"]:  # the rounds-1..4 figure, for comparison
            r, w, ran, _, qr, lr = run_converge(lib, args.config, seed, rank, world, local_rank, barrier,
                                                min(args.converge_max, 3000), args.check_every, lock_model=0)
            conv_lock_off = {"rounds_to_converge": r, "converge_wall_s": round(w, 3) if r else None,
                             "rounds_run": ran, "locked_merges": qr["locked_merges"], "faithful": qr["faithful"],
                             "note": "lock_model = 0 (not the reference: merges run on locked hosts)"}
    conv_ref = None
    ref = CONFIGS[args.config].get("ref_variant")
    if ref and not args.no_converge:
        r, w, ran, _, qr, lr = run_converge(lib, ref, seed, rank, world, local_rank, barrier, args.converge_max,
                                            args.check_every)
        conv_ref = {"config": workload_text(ref), "rounds_to_converge": r,
                    "converge_wall_s": round(w, 3) if r else None, "rounds_run": ran,
                    "simulated_s": (r * 0.2) if r else None, "queues": qr, "lock": lr}
    spread = None
    # per-version spread after the heal, or from round 0 where there is no partition (defined at any
    # cadence, on every line)
    heal = CONFIGS[args.config]["p"].get("partition_end", 0)
    if world == 1 and not args.no_converge:
        e = make_engine(lib, args.config, seed, local_rank)
        try:
            spread = version_spread(e, torch.device(f"cuda:{local_rank}"), heal, max(heal + 10, args.spread_max))
            if not spread["born_after_heal"]["versions"]:
                # no owner stamped a version after the heal (its loopers held the lock throughout):
                # a spread figure would be defined over nothing
                spread = {"rounds": spread["rounds"], "versions_born_after_heal": 0,
                          "hosts_locked_at_end": sum(h.locked_at(e.round) for h in e.hosts()),
                          "note": "no owner refreshed after the heal: BroadcastServices never ran on a host "
                                  "whose looper held the ServicesState lock (services_state.go:535,569)"}
        finally:
            e.close()
    dis = None
    if world == 1 and CONFIGS[args.config]["p"].get("churn_ppm") and not args.no_converge:
        dis = dissemination(lib, args.config, seed, local_rank)  # churn never converges: spread latency
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.config, args.warmup, args.steps, h_mt=args.cpu_hosts)

    if rank == 0:
        cfgp = CONFIGS[args.config]["p"]
        out = {
            "metric": METRIC, "value": tot_merges / dt_max, "unit": "record-merges/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": dt_max * 1000.0 / args.steps, "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None, "dtype": "int64", "data": "synthetic (seeded gossip schedule)",
            "config": {"workload": workload_text(args.config),
                       "hosts": cfgp["n_hosts"], "services": cfgp["n_services"],
                       "fanout": cfgp.get("fanout", 3),
                       "parallelism": (f"host-sharded over {world} ranks ("
                                       + ("RCCL all-to-all)" if backend == "nccl" else "gloo, host-staged all-to-all)")
                                       if world > 1 else "single GPU")},
            "gossip_merges_per_s": split["gossip_merges"] / dt_max, "ae_merges_per_s": split["ae_merges"] / dt_max,
            "merges": split, "merges_by_source": merges_by_source(st0, st1),
            "device_time_share": device_time_share(kern),
            "expiries": expiry_report(st0, st1),
            "queues": queue_report(args.config, st0, st1), "lock": lock,
            "lock_off": lock_off,
            "gossip": gossip, "converge": conv, "converge_lock_off": conv_lock_off,
            "converge_ref_cadence": conv_ref,
            "dissemination": dis, "version_spread": spread,
            "roofline": roof, "roofline_merge": roofline("merge"), "roofline_send": roofline("send"),
            "roofline_lock_off": roof_off,
            "cpu_baseline": cpu, "kernels": kern, "kernels_lock_off": kern_off,
            "kernels_scope": "whole engine" if world == 1 else "rank 0's shard (device time and bytes of its launches)",
            "exchange": xfer,
        }
        if cfgp.get("fd_enable") or cfgp.get("depart_ppm"):
            out["failure_detection"] = {k: st1[k] - st0[k] for k in st1 if k.startswith("fd_") or k in (
                "lost_packets", "expire_server")}
        print(json.dumps(out), flush=True)
    if dist is not None:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

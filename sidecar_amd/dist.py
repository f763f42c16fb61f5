"""Host sharding across engines: one round = send phase, packet exchange, merge phase,
push-pull digest exchange, push-pull delta exchange, end.

Each engine owns the contiguous host block [g*H/G, (g+1)*H/G). The exchange moves the wire
formats of include/gx.h between shards:
  * ``DistShard`` — one process per GPU, ``torch.distributed`` all-to-all (RCCL over xGMI for
    the HIP engine with backend "nccl"; gloo for the CPU oracle in tests);
  * ``LocalShards`` — every shard in this process (one GPU or the CPU); the exchange is a
    device-side concatenation. Used to check the sharded kernels against the unsharded engine.
Exchange buffers are torch uint8 tensors on the engine's device: the HIP engine reads and
writes them as device memory.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np
import torch

from .abi import Engine, GxParams, default_params

# stats that hold the earliest round something happened (-1: never): the minimum over shards
FIRST_ROUND_STATS = ("first_drop_round", "first_locked_round")


def planned_exchange(p: GxParams) -> bool:
    """A gossip round exchanges fixed, seeded slot counts (gx_exchange_plan: no size collective, no
    host wait) iff the failure detector is off and GossipMessages is at most one message per target
    (0 and 1 both mean one). Past one message the plan reserves GossipMessages slots per sampled peer
    and ships mostly padding (GM 15: ~85 MB per rank per round at cfg 5, G = 8), so the exact sizes
    are gathered instead."""
    return not p.fd_enable and p.gossip_messages <= 1


def lock_shortcut(p: GxParams) -> bool:
    """A push-pull round may be replaced by gx_ae_skip_locked when every host holds the lock: the
    lock model on, no failure detector (its membership half runs regardless), no departures."""
    return bool(p.lock_model) and not p.fd_enable and not (p.depart_round >= 0 and p.depart_ppm)


def _ptr(t: torch.Tensor) -> int:
    return t.data_ptr() if t.numel() else 0


class WireBytes:
    """Bytes each exchange moved between shards (this process's shards, sent side)."""

    def __init__(self, e: Engine):
        p = e.params
        self.R = e.H * e.S
        # one digest message per cross-shard pair (gx.h "digest")
        self.dig_msg = 16 + 16 * ((self.R + 511) // 512) + (8 * e.H if p.fd_enable and p.fd_push_pull_state else 0)
        self.packets = self.ae_digest = self.ae_delta = self.ae_lead = self.ae_return = self.ae_full_rows = 0

    def add_ae(self, digest_sizes, lead_sizes, return_sizes):
        dig = int(np.asarray(digest_sizes).sum())
        n_msgs = dig // self.dig_msg
        self.ae_digest += dig
        lead, ret = int(np.asarray(lead_sizes).sum()), int(np.asarray(return_sizes).sum())
        self.ae_lead += lead
        self.ae_return += ret
        self.ae_delta += lead + ret
        self.ae_full_rows += n_msgs * (16 + 8 * self.R)  # the same pairs' full rows

    def as_dict(self):
        return {"packets": self.packets, "ae_digest": self.ae_digest, "ae_delta": self.ae_delta,
                "ae_lead": self.ae_lead, "ae_return": self.ae_return, "ae_full_rows_equivalent": self.ae_full_rows}


class _Shard:
    def __init__(self, params: GxParams, lib, device: torch.device):
        self.e = Engine(params, lib=lib)
        self.device = device
        if device.type == "cuda":
            # the engine queues its work on torch's stream, so packing, the collectives and
            # unpacking are ordered by the stream; only calls that return sizes wait
            self.e.set_stream(torch.cuda.current_stream(device).cuda_stream, True)

    def sync(self):
        pass  # stream-ordered (CUDA) or synchronous (CPU oracle)

    def pack(self, sizes: np.ndarray, packer) -> torch.Tensor:
        buf = torch.empty(int(sizes.sum()), dtype=torch.uint8, device=self.device)
        packer(_ptr(buf), buf.numel())
        return buf


class LocalShards:
    """G shards of one cluster driven in one process."""

    def __init__(self, lib, G: int, device="cpu", **kw):
        self.device = torch.device(device)
        self.G = G
        self.shards: List[_Shard] = []
        for g in range(G):
            p = default_params(lib, **kw)
            p.n_shards = G
            p.shard_id = g
            if self.device.type == "cuda":
                p.device = self.device.index or 0
            self.shards.append(_Shard(p, lib, self.device))
        self.wire = WireBytes(self.shards[0].e)
        self.exchange_paths = {"planned": 0, "sized": 0}  # gossip rounds per exchange path (planned_exchange)
        self.trace_ae = False  # keep each push-pull round's digest and delta inboxes (host copies)
        self.ae_trace = []
        self.ae_skipped = 0  # push-pull rounds with every host locked (gx_ae_skip_locked)
        self.skip_locked = True  # False: run the whole exchange even then (wire tests)

    @property
    def engines(self) -> List[Engine]:
        return [s.e for s in self.shards]

    def _exchange(self, sizes_fn, pack_fn, after_pack=None) -> List[torch.Tensor]:
        """Every shard packs per destination; returns each shard's inbox (sources ascending)."""
        sizes = [sizes_fn(s) for s in self.shards]  # sizes[src][dst]
        self.last_sizes = sizes
        bufs = [s.pack(sz, lambda p, n, e=s.e: pack_fn(e, p, n)) for s, sz in zip(self.shards, sizes)]
        if after_pack is not None:
            for s in self.shards:
                after_pack(s.e)
        for s in self.shards:
            s.sync()
        inboxes = []
        for dst in range(self.G):
            parts = []
            for src in range(self.G):
                off = int(sizes[src][:dst].sum())
                parts.append(bufs[src][off:off + int(sizes[src][dst])])
            inboxes.append(torch.cat(parts) if parts else torch.empty(0, dtype=torch.uint8, device=self.device))
        for s in self.shards:
            s.sync()
        return inboxes

    def _outbox_sizes(self, s) -> np.ndarray:
        """The shard's outbox sizes through gx_outbox_sizes_async (written by the device)."""
        t = torch.zeros(self.G, dtype=torch.int64, device=self.device)
        s.e.outbox_sizes_async(_ptr(t))
        return t.cpu().numpy().astype(np.uint64)

    def _planned_bufs(self):
        """Each shard's send buffer of the planned exchange, allocated once at its bound (DistShard)."""
        if getattr(self, "_pb", None) is None:
            e = self.shards[0].e
            p = e.params
            slot = 16 + 16 * p.packet_cap
            self._pb = [torch.empty((s.e.hi - s.e.lo) * p.fanout * slot, dtype=torch.uint8, device=self.device)
                        for s in self.shards]
        return self._pb

    def _gossip_planned(self) -> bool:
        """A planned gossip round through gx_round_gossip_begin / _end, as DistShard runs it; True
        when it is a push-pull round (round_end is then the caller's)."""
        G = self.G
        bufs = self._planned_bufs()
        plan = np.zeros(G * G, dtype=np.uint64)
        for s, b in zip(self.shards, bufs):
            s.e.round_gossip_begin(plan, _ptr(b), b.numel())
        m = plan.reshape(G, G)
        self.last_sizes = [m[g].copy() for g in range(G)]
        ae = []
        for dst, s in enumerate(self.shards):
            parts = [bufs[src][int(m[src][:dst].sum()):int(m[src][:dst + 1].sum())] for src in range(G)]
            x = torch.cat(parts)
            ae.append(s.e.round_gossip_end(_ptr(x), x.numel()))
        assert all(a == ae[0] for a in ae)
        return ae[0]

    def run_rounds(self, n: int):
        planned = planned_exchange(self.shards[0].e.params)
        for _ in range(n):
            self.exchange_paths["planned" if planned else "sized"] += 1
            if planned:
                ae = self._gossip_planned()
                self.wire.packets += int(sum(int(x.sum()) for x in self.last_sizes))
                if not ae:
                    continue
            else:
                for s in self.shards:
                    s.e.round_send()
                inb = self._exchange(self._outbox_sizes, lambda e, p, c: e.outbox_pack(p, c))
                self.wire.packets += int(sum(int(x.sum()) for x in self.last_sizes))
                for s, x in zip(self.shards, inb):
                    s.e.inbox_unpack(_ptr(x), x.numel())
                for s in self.shards:
                    s.e.round_merge()
            # push-pull: digests, the blocks each side leads, the partners' return blocks (gx.h);
            # shard-local pairs overlap the exchanges. Every shard agrees on the AE rounds. With
            # every host of the cluster locked, every pair fails: the counts only (gx_ae_skip_locked)
            if self.shards[0].e.is_ae_round() and self.G > 1 and self.skip_locked and lock_shortcut(self.shards[0].e.params) and \
                    sum(s.e.lock_census() for s in self.shards) == 0:
                for s in self.shards:
                    s.e.ae_skip_locked()
                self.ae_skipped += 1
            elif self.shards[0].e.is_ae_round():
                dig = self._exchange(lambda s: s.e.ae_bytes(), lambda e, p, c: e.ae_pack(p, c),
                                     after_pack=lambda e: e.ae_merge_local())
                dig_sizes = self.last_sizes
                lead_sizes = {id(s.e): s.e.ae_delta_bytes(_ptr(x), x.numel()) for s, x in zip(self.shards, dig)}
                lead = self._exchange(lambda s: lead_sizes[id(s.e)], lambda e, p, c: e.ae_delta_pack(p, c))
                lead_sz = self.last_sizes
                ret_sizes = {id(s.e): s.e.ae_return_bytes(_ptr(x), x.numel()) for s, x in zip(self.shards, lead)}
                lead_of = {id(s.e): x for s, x in zip(self.shards, lead)}
                ret = self._exchange(lambda s: ret_sizes[id(s.e)],
                                     lambda e, p, c: e.ae_return_pack(_ptr(lead_of[id(e)]), lead_of[id(e)].numel(), p, c))
                for a, b, c in zip(dig_sizes, lead_sz, self.last_sizes):
                    self.wire.add_ae(a, b, c)
                if self.trace_ae and any(x.numel() for x in dig):
                    self.ae_trace.append(([x.cpu().numpy().tobytes() for x in dig],
                                          [x.cpu().numpy().tobytes() for x in lead],
                                          [x.cpu().numpy().tobytes() for x in ret]))
                for s, x, y in zip(self.shards, lead, ret):
                    s.e.ae_merge(_ptr(x), x.numel(), _ptr(y), y.numel())
            for s in self.shards:
                s.e.round_end()

    def stats(self) -> dict:
        tot = {}
        for s in self.shards:
            for k, v in s.e.stats().items():
                if k in FIRST_ROUND_STATS:  # the earliest over shards (-1: none)
                    tot[k] = min(x for x in (tot.get(k, -1), v) if x >= 0) if max(tot.get(k, -1), v) >= 0 else -1
                else:
                    tot[k] = max(tot.get(k, v), v) if k in ("round", "last_change_round") else tot.get(k, 0) + v
        return tot

    def converged(self):
        R = self.shards[0].e.H * self.shards[0].e.S
        mn = torch.empty(R, dtype=torch.int64, device=self.device)
        mx = torch.empty(R, dtype=torch.int64, device=self.device)
        gmn = gmx = None
        for s in self.shards:
            s.e.view_minmax(_ptr(mn), _ptr(mx))
            gmn = mn.clone() if gmn is None else torch.minimum(gmn, mn)
            gmx = mx.clone() if gmx is None else torch.maximum(gmx, mx)
        bad = int((gmn != gmx).sum().item())
        if bad == 0 and self.shards[0].e.params.fd_enable:  # membership agrees with the truth too
            bad = sum(s.e.fd_converged()[1] for s in self.shards)
        return bad == 0, bad


class DistShard:
    """This process's shard; the others are peers in torch.distributed's default group."""

    def __init__(self, lib, rank: int, world: int, device, group=None, **kw):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank, self.world = rank, world
        self.device = torch.device(device)
        p = default_params(lib, **kw)
        p.n_shards = world
        p.shard_id = rank
        if self.device.type == "cuda":
            p.device = self.device.index or 0
        self.s = _Shard(p, lib, self.device)
        self.e = self.s.e
        self.wire = WireBytes(self.e)
        self.exchange_paths = {"planned": 0, "sized": 0}  # gossip rounds per exchange path (planned_exchange)
        self.ae_skipped = 0  # push-pull rounds with every host locked (gx_ae_skip_locked)
        self.skip_locked = True  # False: run the whole exchange even then
        # gloo has no device all-to-all / all-gather: a gloo group over device shards (the one-GPU
        # rehearsal of the RCCL path in tests/test_gpu_dist.py) stages collectives through the host
        self.stage = self.device.type == "cuda" and dist.get_backend(group) == "gloo"

    def _host(self, t: torch.Tensor) -> torch.Tensor:
        return t.cpu() if self.stage else t

    def _a2a(self, recv, send, rs, ss):
        if not self.stage:
            self.dist.all_to_all_single(recv, send, output_split_sizes=rs, input_split_sizes=ss, group=self.group)
            return
        r = torch.empty(recv.numel(), dtype=recv.dtype)
        self.dist.all_to_all_single(r, send.cpu(), output_split_sizes=rs, input_split_sizes=ss, group=self.group)
        recv.copy_(r)

    def _all_reduce(self, t: torch.Tensor, op):
        h = self._host(t)
        self.dist.all_reduce(h, op=op, group=self.group)
        if h is not t:
            t.copy_(h)

    CHUNK = 256 << 20  # bytes per peer per all-to-all call

    def _exchange(self, sizes, packer, after_pack=None) -> torch.Tensor:
        """all-to-all of this shard's per-destination messages; returns the inbox (sources ascending).
        `sizes`: host array, or a device tensor the engine filled (gx_outbox_sizes_async), which
        then travels in the size all-gather without a host wait of its own."""
        dist = self.dist
        # every rank learns the whole size matrix in one collective: its receive sizes, and the
        # number of chunked calls all ranks make
        if isinstance(sizes, torch.Tensor):
            mine = sizes
        else:
            mine = torch.tensor(sizes.astype(np.int64), device=self.device)
        mine = self._host(mine)
        rows = [torch.empty_like(mine) for _ in range(self.world)]
        dist.all_gather(rows, mine, group=self.group)
        m = torch.stack(rows).tolist()  # m[src][dst]: the one host wait of the exchange
        ss = [int(x) for x in m[self.rank]]
        rs = [int(m[src][self.rank]) for src in range(self.world)]
        self.last_sizes = np.array(ss, dtype=np.uint64)
        send = self.s.pack(self.last_sizes, packer)
        if after_pack is not None:
            after_pack()  # shard-local pairs on the engine's side stream, beside the collective
        recv = torch.empty(sum(rs), dtype=torch.uint8, device=self.device)
        self._a2a_chunked(recv, send, rs, ss, max(max(r) for r in m))
        self.s.sync()
        return recv

    def _a2a_chunked(self, recv, send, rs, ss, largest):
        """all_to_all_single of per-peer segments, split into calls of at most CHUNK bytes per peer.
        `largest`: the largest segment between any two ranks (every rank knows the whole size
        matrix), so every rank makes the same number of calls, ceil(largest / CHUNK)."""
        calls = (int(largest) + self.CHUNK - 1) // self.CHUNK
        if calls <= 1:
            self._a2a(recv, send, rs, ss)
            return
        soff = np.concatenate([[0], np.cumsum(ss)])
        roff = np.concatenate([[0], np.cumsum(rs)])
        for c in range(calls):
            lo = c * self.CHUNK
            s_part = [max(0, min(self.CHUNK, n - lo)) for n in ss]
            r_part = [max(0, min(self.CHUNK, n - lo)) for n in rs]
            s_buf = torch.cat([send[int(soff[p]) + lo:int(soff[p]) + lo + s_part[p]] for p in range(self.world)])
            r_buf = torch.empty(sum(r_part), dtype=torch.uint8, device=self.device)
            self._a2a(r_buf, s_buf, r_part, s_part)
            o = 0
            for p in range(self.world):
                if r_part[p]:
                    recv[int(roff[p]) + lo:int(roff[p]) + lo + r_part[p]].copy_(r_buf[o:o + r_part[p]])
                o += r_part[p]

    def _planned_bufs(self):
        """The send buffer of the planned exchange, allocated once at its bound (k_send writes the
        slots straight into it, before the round's counts reach the host: a shard sends at most
        fanout packet slots per host, gx.h gx_exchange_plan), and the plan matrix."""
        if getattr(self, "_pb", None) is None:
            p = self.e.params
            slot = 16 + 16 * p.packet_cap
            hl = self.e.hi - self.e.lo
            send = torch.empty(hl * p.fanout * slot, dtype=torch.uint8, device=self.device)
            self._pb = (send, np.zeros(self.world * self.world, dtype=np.uint64))
            self._precv = torch.empty(0, dtype=torch.uint8, device=self.device)
        return self._pb

    def _planned_recv(self, nr: int) -> torch.Tensor:
        """The receive buffer, grown to this round's planned size when a round needs more (with a
        quarter of headroom); the bound, every other shard's fanout slots per host, is only reached
        when every packet of the cluster comes here."""
        if nr > self._precv.numel():
            self._precv = torch.empty(nr + nr // 4, dtype=torch.uint8, device=self.device)
        return self._precv

    def _gossip_planned(self) -> bool:
        """One planned gossip round in two engine calls around the all-to-all; True when it is a
        push-pull round (the caller runs the push-pull steps and round_end). A per-peer segment over
        CHUNK goes in several calls, like _exchange's."""
        e = self.e
        send, plan = self._planned_bufs()
        e.round_gossip_begin(plan, _ptr(send), send.numel())
        m = plan.reshape(self.world, self.world)
        ss = [int(x) for x in m[self.rank]]
        rs = [int(m[src][self.rank]) for src in range(self.world)]
        self.last_sizes = m[self.rank].copy()
        ns, nr = sum(ss), sum(rs)
        if ns > send.numel():
            raise RuntimeError("planned exchange larger than its bound")  # cannot happen (gx.h)
        recv = self._planned_recv(nr)
        self._a2a_chunked(recv[:nr], send[:ns], rs, ss, int(m.max()))
        return e.round_gossip_end(_ptr(recv), nr)

    def _all_locked(self) -> bool:
        """Every host of every shard holds the ServicesState lock this round (gx_lock_census)."""
        if self.world < 2 or not (self.skip_locked and lock_shortcut(self.e.params)):
            return False
        t = torch.tensor([self.e.lock_census()], dtype=torch.int64, device=self.device)
        self._all_reduce(t, self.dist.ReduceOp.SUM)
        return int(t.item()) == 0

    def run_rounds(self, n: int):
        e = self.e
        planned = planned_exchange(e.params)  # sizes from the seeded plan: no host wait
        for _ in range(n):
            self.exchange_paths["planned" if planned else "sized"] += 1
            if planned:
                ae = self._gossip_planned()
            else:
                e.round_send()
                ob = torch.zeros(self.world, dtype=torch.int64, device=self.device)
                e.outbox_sizes_async(_ptr(ob))  # no host wait: the sizes join the size all-gather
                x = self._exchange(ob, e.outbox_pack)
                e.inbox_unpack(_ptr(x), x.numel())
                e.round_merge()
                ae = e.is_ae_round()
            self.wire.packets += int(self.last_sizes.sum())
            # push-pull: digests, lead blocks, return blocks (local pairs overlap the exchanges);
            # with every host of the cluster locked (one census collective) every pair fails
            if ae and self._all_locked():
                e.ae_skip_locked()
                e.round_end()
                self.ae_skipped += 1
            elif ae:
                dsz = e.ae_bytes()
                dig = self._exchange(dsz, e.ae_pack, after_pack=e.ae_merge_local)
                lsz = e.ae_delta_bytes(_ptr(dig), dig.numel())
                lead = self._exchange(lsz, e.ae_delta_pack)
                rsz = e.ae_return_bytes(_ptr(lead), lead.numel())
                ret = self._exchange(rsz, lambda p, c: e.ae_return_pack(_ptr(lead), lead.numel(), p, c))
                self.wire.add_ae(dsz, lsz, rsz)
                e.ae_merge(_ptr(lead), lead.numel(), _ptr(ret), ret.numel())
                e.round_end()
            elif not planned:
                e.round_end()

    def close(self):
        """Wait for the engine's work (its stream and the planned exchange's look-ahead stream) and
        free it, before the caller tears the process group down: RCCL's communicator teardown
        must not race the engine's kernels or buffers."""
        if getattr(self, "e", None) is None:
            return
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        self.e.close()
        self._pb = None
        self._precv = None
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def stats(self) -> dict:
        st = self.e.stats()
        keys = sorted(st)
        t = torch.tensor([st[k] for k in keys], dtype=torch.int64, device=self.device)
        mx = t.clone()
        mn = torch.tensor([int(st[k]) if st[k] >= 0 else 1 << 62 for k in FIRST_ROUND_STATS],
                          dtype=torch.int64, device=self.device)
        self._all_reduce(t, self.dist.ReduceOp.SUM)
        self._all_reduce(mx, self.dist.ReduceOp.MAX)
        self._all_reduce(mn, self.dist.ReduceOp.MIN)  # the earliest LOST dequeue / lock over shards
        out = dict(zip(keys, t.tolist()))
        for k in ("round", "last_change_round"):
            out[k] = int(mx[keys.index(k)].item())
        for k, x in zip(FIRST_ROUND_STATS, mn.tolist()):
            out[k] = int(x) if x < 1 << 62 else -1
        return out

    def converged(self):
        """(agreed, n) as LocalShards.converged: n = catalog records on which the live views disagree
        (all shards); once they agree, with the failure detector, the sum over shards of the nodes
        some of the shard's live views misjudge (a node misjudged in several shards counts once
        per shard). Every rank takes the same branch: `bad` is all-reduced first."""
        R = self.e.H * self.e.S
        mn = torch.empty(R, dtype=torch.int64, device=self.device)
        mx = torch.empty(R, dtype=torch.int64, device=self.device)
        self.e.view_minmax(_ptr(mn), _ptr(mx))
        self._all_reduce(mn, self.dist.ReduceOp.MIN)
        self._all_reduce(mx, self.dist.ReduceOp.MAX)
        bad = int((mn != mx).sum().item())
        if bad == 0 and self.e.params.fd_enable:  # membership agrees with the truth on every shard too
            t = torch.tensor([self.e.fd_converged()[1]], dtype=torch.int64, device=self.device)
            self._all_reduce(t, self.dist.ReduceOp.SUM)
            bad = int(t.item())
        return bad == 0, bad

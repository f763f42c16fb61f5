// gx_fd.hpp — memberlist failure detection on the device.
//
// memberlist (github.com/NinesStack/memberlist v0.0.0-20170522194404-cfac2b5cf519, reference
// go.mod:6; a fork of hashicorp/memberlist, absent from the reference tree) runs SWIM + Lifeguard
// on every Sidecar node; Sidecar only reacts to NotifyLeave -> go ExpireServer(node)
// (services_delegate.go:173-176). Per simulated host the engine keeps memberlist's member list
// (gx_member per (host, node), suspicion deadlines in fd_dl for coalesced timer scans) and its
// TransmitLimitedQueue as per-transmit-count stacks linked through the member rows.
//
// Kernels (one host per thread or wave; the work is pointer-chasing integer logic, latency-
// bound, not bandwidth-bound):
//   k_fd_tick   one wave per host: suspicion timers due -> deadNode on the due nodes' lanes,
//               then ExpireServer in node order on lane 0 (NotifyLeave), the due deadlines found
//               by a coalesced scan of the host's fd_dl row (only when its exact lower bound
//               min_deadline has passed); then probe() on the host's probe tick (lane 0)
//   k_fd_send   one thread per host: kRandomNodes gossip targets, then the memberlist messages
//               of every packet (TransmitLimitedQueue.GetBroadcasts)
//   k_fd_recv   one thread per receiver, after the catalog merge: the packets' memberlist
//               messages in sender order -> aliveNode / suspectNode / deadNode
// Handlers follow the restatement in oracle/gx_oracle_fd.c (the CPU checker) rule for rule.

struct FdAcc {
  unsigned c[C_NCTR_ALL - C_NCTR];
  GXD FdAcc() {
#pragma unroll
    for (int i = 0; i < C_NCTR_ALL - C_NCTR; i++) c[i] = 0;
  }
  GXD void inc(int k, unsigned v = 1) { c[k - C_NCTR] += v; }
};
GXD void fd_flush(const Dev &d, const FdAcc &f) {
  for (int i = 0; i < C_NCTR_ALL - C_NCTR; i++) {
    unsigned long long x = wave_sum((unsigned long long)f.c[i]);
    if ((threadIdx.x & 63) == 0) ctr_atomic(d, C_NCTR + i, x);
  }
}


// Reaped at the host's last resetNodes: dead for more than GossipToTheDeadTime.
GXD bool fd_reaped(const Dev &d, uint32_t v, const gx_member *x) {
  return x->state == GX_M_DEAD &&
         (int64_t)fdhp(d, v)->wrap_round - (int64_t)x->change_round > (int64_t)d.p.fd_gossip_dead_rounds;
}

// ----------------------------------------------------------------- TransmitLimitedQueue --
GXD void q_unlink(const Dev &d, uint32_t v, uint32_t m) {
  gx_member *x = memp(d, v, m);
  gx_fd_host *h = fdhp(d, v);
  const uint16_t pv = x->q_prev, nx = x->q_next;
  if (pv != GX_FD_NONE) memp(d, v, pv)->q_next = nx;
  else h->q_head[x->tx - 1] = nx;
  if (nx != GX_FD_NONE) memp(d, v, nx)->q_prev = pv;
  x->q_prev = x->q_next = GX_FD_NONE;
  x->tx = 0;
  h->q_len--;
}
GXD void q_push(const Dev &d, uint32_t v, uint32_t m, uint32_t b) {  // newest of bucket b
  gx_member *x = memp(d, v, m);
  gx_fd_host *h = fdhp(d, v);
  const uint16_t top = h->q_head[b];
  x->q_prev = GX_FD_NONE;
  x->q_next = top;
  if (top != GX_FD_NONE) memp(d, v, top)->q_prev = (uint16_t)m;
  h->q_head[b] = (uint16_t)m;
  x->tx = (uint8_t)(b + 1);
  h->q_len++;
}
// encodeAndBroadcast -> QueueBroadcast: invalidates the queued message about m. With `defer`
// (the membership merge's lanes), only the message is written and *defer set: the caller moves
// the flagged nodes to the queue's front afterwards, in node order.
GXD void fd_broadcast(const Dev &d, uint32_t v, uint32_t m, int kind, uint32_t inc, uint32_t from,
                      bool *defer = nullptr) {
  gx_member *x = memp(d, v, m);
  if (!defer && x->tx) q_unlink(d, v, m);
  x->msg_kind = (uint8_t)kind;
  x->msg_incarnation = inc;
  x->msg_from = (uint16_t)from;
  if (defer) *defer = true;
  else q_push(d, v, m, 0);
}
// The deferred half of fd_broadcast (unlink if queued, push on stack 0) for every node base + k
// with bit k of qm set, in node order, by the lanes of one wave
// (`mine` = this lane's bit). Sequential requeues unlink each node from its stack and push it on
// stack 0, so the result is: every stack minus the set, with the set on top of stack 0 in
// descending node order. Unlink: the lane that starts a run of set nodes in a stack (its q_prev is
// not in the set) splices prev <-> s, s the run's first successor outside the set (found by
// pointer jumping over the lanes' links in registers); runs are disjoint, so no two lanes write
// the same link. Push: each set lane links to its
// neighbours in the set by lane order, the lowest onto the old top of stack 0.
GXD void fd_requeue_chunk(const Dev &d, uint32_t v, uint32_t base, unsigned long long qm, bool mine) {
  const uint32_t lane = threadIdx.x & 63, m = base + lane;
  gx_fd_host *h = fdhp(d, v);
  auto in_set = [&](uint32_t y) { return y != GX_FD_NONE && y - base < 64u && ((qm >> (y - base)) & 1ull); };
  uint32_t tx = 0, pv = GX_FD_NONE, s = GX_FD_NONE;
  if (mine) {
    const gx_member *x = memp(d, v, m);
    tx = x->tx;
    pv = x->q_prev;
    s = x->q_next;
  }
  const bool queued = mine && tx != 0;
  // each queued lane's first successor outside the set, by pointer jumping over the lanes'
  // successors (a run has at most 64 nodes, so 6 doublings reach its end)
#pragma unroll
  for (int i = 0; i < 6; i++) {
    const bool jump = queued && in_set(s);
    const uint32_t t = (uint32_t)__shfl((int)s, jump ? (int)(s - base) : (int)lane, 64);
    if (jump) s = t;
  }
  if (queued && !in_set(pv)) {  // a run starts here: splice its predecessor to s
    if (pv != GX_FD_NONE) memp(d, v, pv)->q_next = (uint16_t)s;
    else h->q_head[tx - 1] = (uint16_t)s;
    if (s != GX_FD_NONE) memp(d, v, s)->q_prev = (uint16_t)pv;
  }
  const unsigned long long qq = __ballot(queued);
  __threadfence_block();  // every splice is done before stack 0's top is read
  const uint32_t top = h->q_head[0];
  if (mine) {
    gx_member *x = memp(d, v, m);
    const unsigned long long below = qm & ((1ull << lane) - 1), above = lane == 63 ? 0ull : qm & (~0ull << (lane + 1));
    x->q_next = below ? (uint16_t)(base + 63 - __builtin_clzll(below)) : (uint16_t)top;
    x->q_prev = above ? (uint16_t)(base + __ffsll((long long)above) - 1) : (uint16_t)GX_FD_NONE;
    x->tx = 1;
    if (!below && top != GX_FD_NONE) memp(d, v, top)->q_prev = (uint16_t)m;
    if (!above) h->q_head[0] = (uint16_t)m;
  }
  if (lane == 0) h->q_len += (uint32_t)__popcll(qm) - (uint32_t)__popcll(qq);
}
// TransmitLimitedQueue.GetBroadcasts with a message budget (<= 64): the messages are taken from
// the tops of the stacks in transmit-count order, then requeued one transmit count up (dropped at
// the retransmit limit). As a sequence of unlinks in take order and pushes in reverse take order
// (the oracle's restatement), stack b ends as: the segment taken from stack b - 1 (links kept)
// followed by what stack b kept. So one walk does it: each visited stack is spliced as soon as its
// taken prefix is known, and each taken node is read once (message fields and link in one row).
GXD void q_splice(const Dev &d, gx_fd_host *h, uint32_t v, uint32_t b, uint32_t first, uint32_t last, uint32_t rest) {
  if (first != GX_FD_NONE) {
    h->q_head[b] = (uint16_t)first;
    memp(d, v, last)->q_next = (uint16_t)rest;
    if (rest != GX_FD_NONE) memp(d, v, rest)->q_prev = (uint16_t)last;
  } else {
    h->q_head[b] = (uint16_t)rest;
    if (rest != GX_FD_NONE) memp(d, v, rest)->q_prev = GX_FD_NONE;
  }
}
GXD uint32_t fd_get_broadcasts(const Dev &d, FdAcc &f, uint32_t v, uint32_t limit, gx_fd_msg *out) {
  gx_fd_host *h = fdhp(d, v);
  uint32_t n = 0, dropped = 0, pf = GX_FD_NONE, pl = GX_FD_NONE;  // segment taken from stack b - 1
  const uint32_t L = d.p.fd_retransmit_limit;
  if (limit > 64) limit = 64;
  uint32_t b = 0;
  for (; b < L && n < limit; b++) {
    uint32_t first = GX_FD_NONE, last = GX_FD_NONE, m = h->q_head[b];
    while (m != GX_FD_NONE && n < limit) {
      gx_member *x = memp(d, v, m);
      const uint32_t nx = x->q_next;
      gx_fd_msg g;
      g.incarnation = x->msg_incarnation;
      g.node = (uint16_t)m;
      g.from = x->msg_from;
      g.kind = x->msg_kind;
      g.pad[0] = g.pad[1] = g.pad[2] = 0;
      out[n++] = g;
      if (b + 1 < L) {
        x->tx = (uint8_t)(b + 2);
      } else {  // transmitted the limit: leaves the queue
        x->tx = 0;
        x->q_prev = x->q_next = GX_FD_NONE;
        dropped++;
      }
      if (first == GX_FD_NONE) first = m;
      last = m;
      m = nx;
    }
    q_splice(d, h, v, b, pf, pl, m);  // stack b := segment of stack b - 1 ++ what b kept
    pf = b + 1 < L ? first : GX_FD_NONE;
    pl = last;
  }
  if (b < L && pf != GX_FD_NONE) q_splice(d, h, v, b, pf, pl, h->q_head[b]);
  h->q_len -= dropped;
  f.inc(C_FD_SENT, n);
  return n;
}

// --------------------------------------------------------------------- message handlers --
GXD void fd_set_deadline(const Dev &d, uint32_t v, uint32_t m, int64_t dl, bool lanes = false) {
  if (dl > GX_FD_NO_DEADLINE - 1) dl = GX_FD_NO_DEADLINE - 1;
  *dlp(d, v, m) = (int32_t)dl;
  if (lanes) atomicMin(&fdhp(d, v)->min_deadline, (int32_t)dl);  // several lanes of one host
  else if ((int32_t)dl < fdhp(d, v)->min_deadline) fdhp(d, v)->min_deadline = (int32_t)dl;
}
GXD void fd_refute(const Dev &d, FdAcc &f, uint32_t v, uint32_t accused, bool *defer = nullptr) {
  gx_member *me = memp(d, v, v);
  uint32_t inc = me->incarnation + 1;
  if (accused >= inc) inc = accused + 1;
  me->incarnation = inc;
  fd_broadcast(d, v, v, GX_M_ALIVE, inc, v, defer);
  f.inc(C_FD_REFUTE);
}
// deadNode; NotifyLeave -> ExpireServer (services_delegate.go:173-176).
// With `defer` (the timer scan's lanes), the queue move is deferred as in fd_broadcast and, on a
// death, *died is set instead of running ExpireServer, which the caller then runs in node order.
GXD void fd_dead_node(const Dev &d, Acc &a, FdAcc &f, uint32_t v, const gx_fd_msg &g, bool *defer = nullptr,
                      bool *died = nullptr) {
  const uint32_t m = g.node;
  gx_member *x = memp(d, v, m);
  if (fd_reaped(d, v, x)) return;
  if (g.incarnation < x->incarnation) return;
  *dlp(d, v, m) = GX_FD_NO_DEADLINE;  // delete(m.nodeTimers, d.Node)
  if (x->state == GX_M_DEAD) return;
  if (m == v) {
    fd_refute(d, f, v, g.incarnation, defer);
    return;
  }
  fd_broadcast(d, v, m, GX_M_DEAD, g.incarnation, g.from, defer);
  x->incarnation = g.incarnation;
  x->state = GX_M_DEAD;
  x->change_round = (int32_t)d.round;
  f.inc(C_FD_DEATH);
  if (died) *died = true;
  else notify_leave(d, a, v, m);
}
GXD bool fd_confirm(const Dev &d, FdAcc &f, uint32_t v, uint32_t m, gx_member *x, uint32_t from,
                    bool lanes = false) {
  if (x->n_conf >= d.p.fd_suspicion_k) return false;
  for (uint32_t i = 0; i <= x->n_conf; i++)
    if (x->susp_from[i] == from) return false;
  x->susp_from[1 + x->n_conf] = (uint16_t)from;
  x->n_conf++;
  *dlp(d, v, m) = GX_FD_NO_DEADLINE;
  fd_set_deadline(d, v, m, (int64_t)x->change_round + d.p.fd_suspicion_rounds[x->n_conf], lanes);
  f.inc(C_FD_CONFIRM);
  return true;
}
GXD void fd_suspect_node(const Dev &d, FdAcc &f, uint32_t v, const gx_fd_msg &g, bool *defer = nullptr) {
  const uint32_t m = g.node;
  gx_member *x = memp(d, v, m);
  if (fd_reaped(d, v, x)) return;
  if (g.incarnation < x->incarnation) return;
  if (x->state == GX_M_SUSPECT) {
    if (fd_confirm(d, f, v, m, x, g.from, defer != nullptr))
      fd_broadcast(d, v, m, GX_M_SUSPECT, g.incarnation, g.from, defer);
    return;
  }
  if (x->state != GX_M_ALIVE) return;
  if (m == v) {
    fd_refute(d, f, v, g.incarnation, defer);
    return;
  }
  fd_broadcast(d, v, m, GX_M_SUSPECT, g.incarnation, g.from, defer);
  x->incarnation = g.incarnation;
  x->state = GX_M_SUSPECT;
  x->change_round = (int32_t)d.round;
  x->n_conf = 0;
  x->susp_from[0] = (uint16_t)g.from;
  x->susp_from[1] = x->susp_from[2] = GX_FD_NONE;
  fd_set_deadline(d, v, m, d.round + (int64_t)d.p.fd_suspicion_rounds[0], defer != nullptr);
  f.inc(C_FD_SUSPECT);
}
GXD void fd_alive_node(const Dev &d, FdAcc &f, uint32_t v, const gx_fd_msg &g, bool *defer = nullptr) {
  const uint32_t m = g.node;
  gx_member *x = memp(d, v, m);
  if (fd_reaped(d, v, x)) {  // unknown node: re-added as dead, incarnation 0
    x->state = GX_M_DEAD;
    x->incarnation = 0;
    x->change_round = INT32_MIN;
  }
  if (m == v) {
    if (g.incarnation <= x->incarnation) return;
    uint32_t inc = x->incarnation + 1;
    if (g.incarnation >= inc) inc = g.incarnation + 1;
    x->incarnation = inc;
    fd_broadcast(d, v, v, GX_M_ALIVE, inc, v, defer);
    f.inc(C_FD_REFUTE);
    return;
  }
  if (g.incarnation <= x->incarnation) return;
  *dlp(d, v, m) = GX_FD_NO_DEADLINE;
  fd_broadcast(d, v, m, GX_M_ALIVE, g.incarnation, g.from, defer);
  x->incarnation = g.incarnation;
  if (x->state != GX_M_ALIVE) {
    x->state = GX_M_ALIVE;
    x->change_round = (int32_t)d.round;
  }
  x->n_conf = 0;
  f.inc(C_FD_ALIVE);
}
GXD void fd_handle(const Dev &d, Acc &a, FdAcc &f, uint32_t v, const gx_fd_msg &g) {
  if (g.node >= d.H) return;
  if (g.kind == GX_M_ALIVE) fd_alive_node(d, f, v, g);
  else if (g.kind == GX_M_SUSPECT) fd_suspect_node(d, f, v, g);
  else if (g.kind == GX_M_DEAD) fd_dead_node(d, a, f, v, g);
  f.inc(C_FD_RECV);
}

// ---------------------------------------------------------------------------- probes ------
// probe() + probeNode(): returns the target (GX_FD_NONE if none), *ack its outcome.
GXD uint32_t fd_probe_host(const Dev &d, FdAcc &f, uint32_t v, bool *ack_out) {
  gx_fd_host *h = fdhp(d, v);
  const uint32_t H = d.H;
  uint32_t t = GX_FD_NONE, num_check = 0;
  *ack_out = false;
  while (num_check < H) {
    if (h->probe_index >= H) {  // resetNodes: reap, reshuffle
      h->probe_pass++;
      h->probe_index = 0;
      h->wrap_round = (int32_t)d.round;
      num_check++;
      continue;
    }
    uint32_t c = feistel_perm(rng4(d.p.seed, ST_FD_PERM, v, h->probe_pass, 0), h->probe_index, H);
    h->probe_index++;
    if (c == v || memp(d, v, c)->state == GX_M_DEAD) {
      num_check++;
      continue;
    }
    t = c;
    break;
  }
  if (t == GX_FD_NONE) return t;
  f.inc(C_FD_PROBES);
  bool ack = reach(d, v, t);
  if (!ack) {  // IndirectChecks relays: kRandomNodes over alive nodes other than us and the target
    uint32_t relays[16], nr = 0;
    const uint32_t want = d.p.fd_indirect_checks;
    for (uint32_t a = 0; nr < want && a < 3u * H; a++) {
      uint32_t r = unif(rng4(d.p.seed, ST_FD_RELAY, (uint64_t)d.round, v, a), H);
      if (r == v || r == t || memp(d, v, r)->state != GX_M_ALIVE) continue;
      bool dup = false;
      for (uint32_t i = 0; i < nr; i++) dup |= relays[i] == r;
      if (!dup) relays[nr++] = r;
    }
    for (uint32_t i = 0; i < nr; i++)
      if (reach(d, v, relays[i]) && reach(d, relays[i], t)) ack = true;
  }
  if (!ack) {
    f.inc(C_FD_PROBE_FAIL);
    gx_fd_msg s;
    s.incarnation = memp(d, v, t)->incarnation;
    s.node = (uint16_t)t;
    s.from = (uint16_t)v;
    s.kind = GX_M_SUSPECT;
    fd_suspect_node(d, f, v, s);
  }
  *ack_out = ack;
  return t;
}
GXD bool fd_probe_tick(const Dev &d, uint32_t v) {
  const uint32_t P = d.p.fd_probe_rounds;
  return (uint64_t)d.round % P == rng4(d.p.seed, ST_FD_PHASE, v, 0, 0) % P;
}

// Suspicion timers of host v due this round, one wave: coalesced scan of the fd_dl row, the due
// nodes declared dead with the effects of sequential handlers in node order; the new exact
// min_deadline is the wave minimum of the rest.
GXD void fd_timers_wave(const Dev &d, Acc &a, FdAcc &f, uint32_t v) {
  const uint32_t lane = threadIdx.x & 63;
  if (fdhp(d, v)->min_deadline > d.round) return;  // uniform
  if (lane == 0) kbytes(d, GX_K_FD, 4ull * d.H, d.H);  // the deadline row
  int32_t mn = GX_FD_NO_DEADLINE;
  for (uint32_t base = 0; base < d.H; base += 64) {
    const uint32_t m = base + lane;
    const int32_t dl = m < d.H ? *dlp(d, v, m) : GX_FD_NO_DEADLINE;
    const bool due = dl <= d.round;
    if (!due) mn = dl < mn ? dl : mn;
    // the due nodes' deadNode handlers run side by side (each touches only its node's row and
    // deadline); their queue moves follow in node order (fd_requeue_chunk), then lane 0 runs
    // ExpireServer for the new deaths in node order (the catalog side never reads member rows)
    bool bc = false, died = false;
    if (due) {
      gx_fd_msg g;
      g.incarnation = memp(d, v, m)->incarnation;
      g.node = (uint16_t)m;
      g.from = (uint16_t)v;
      g.kind = GX_M_DEAD;
      g.pad[0] = g.pad[1] = g.pad[2] = 0;
      fd_dead_node(d, a, f, v, g, &bc, &died);
    }
    const unsigned long long qm = __ballot(bc);
    if (qm) {
      __threadfence_block();
      fd_requeue_chunk(d, v, base, qm, bc);
      __threadfence_block();
    }
    unsigned long long dm = __ballot(died);
    if (lane == 0)
      while (dm) {
        const uint32_t k = (uint32_t)__ffsll((long long)dm) - 1;
        dm &= dm - 1;
        notify_leave(d, a, v, base + k);
      }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    int32_t y = __shfl_xor(mn, o, 64);
    mn = y < mn ? y : mn;
  }
  if (lane == 0) fdhp(d, v)->min_deadline = mn;
}

// gossip(): kRandomNodes(GossipNodes) skipping us and nodes dead beyond GossipToTheDeadTime.
GXD uint32_t fd_sample_peers(const Dev &d, uint32_t u, uint32_t *peers) {
  const uint32_t H = d.H;
  uint32_t cnt = 0;
  if (H < 2) return 0;
  for (uint32_t a = 0; cnt < d.K && a < 3u * H; a++) {
    uint32_t p = unif(rng4(d.p.seed, ST_PEER, (uint64_t)d.round, u, a), H);
    if (p == u) continue;
    const gx_member *x = memp(d, u, p);
    if (x->state == GX_M_DEAD && d.round - (int64_t)x->change_round > (int64_t)d.p.fd_gossip_dead_rounds) continue;
    bool dup = false;
    for (uint32_t i = 0; i < cnt; i++) dup |= peers[i] == p;
    if (!dup) peers[cnt++] = p;
  }
  return cnt;
}
GXD uint32_t fd_budget(const Dev &d) {
  uint32_t b = d.p.fd_msg_cap;
  if (d.p.limit_bytes) {
    uint32_t x = d.p.limit_bytes / (d.p.fd_msg_bytes + 2);
    b = x < b ? x : b;
  }
  return b;
}

// ------------------------------------------------- push-pull membership (mergeState) ------
// The member list pushPull sends: incarnation << 32 | state per node, FD_SNAP_ABSENT if reaped.
#define FD_SNAP_ABSENT 0xffull
GXD uint64_t fd_snap_word(const Dev &d, uint32_t v, uint32_t m) {
  const gx_member *x = memp(d, v, m);
  if (fd_reaped(d, v, x)) return FD_SNAP_ABSENT;
  return ((uint64_t)x->incarnation << 32) | x->state;
}
// state.go mergeState into host v, node order: alive -> aliveNode, suspect or dead ->
// suspectNode{From: v}. One wave: the lanes test 64 nodes at a time for an effect (a superset of
// the nodes whose handler changes anything; a node's test reads only that node's row, which the
// handlers of other nodes do not change), run the flagged nodes' handlers side by side (each
// touches only its node's row), and lane 0 then moves the broadcast nodes in the queue in order.
// One 64-node chunk of the merge into host v: w = the remote list's word for node base + lane,
// lo/hi = the node's row fields in v's list (read before any handler of this chunk ran).
GXD void fd_merge_chunk(const Dev &d, FdAcc &f, uint32_t v, uint32_t base, uint64_t w, uint4 lo, uint4 hi,
                        int64_t wrap, int64_t dead_rounds, unsigned &present_n) {
  const uint32_t lane = threadIdx.x & 63;
  const bool present = base + lane < d.H && (w & 0xffu) != FD_SNAP_ABSENT;
  bool flag = false;
  if (present) {
    present_n++;
    const uint32_t inc_l = lo.x, state = hi.x & 0xffu, n_conf = (hi.x >> 8) & 0xffu;
    const bool reaped = state == GX_M_DEAD && wrap - (int64_t)(int32_t)lo.z > dead_rounds;
    const uint32_t inc = (uint32_t)(w >> 32);
    if ((w & 0xffu) == GX_M_ALIVE) {
      flag = reaped || inc > inc_l;
    } else {
      const uint32_t from[3] = {hi.y >> 16, hi.z & 0xffffu, hi.z >> 16};
      bool confirm = state == GX_M_SUSPECT && n_conf < d.p.fd_suspicion_k;
      for (uint32_t i = 0; i < 3 && confirm; i++)
        if (i <= n_conf && from[i] == v) confirm = false;
      flag = !reaped && inc >= inc_l && (state == GX_M_ALIVE || confirm);
    }
  }
  // each flagged lane runs its node's handler (node-local state, deadline, counters); the
  // queue moves (unlink, push to the front of bucket 0) follow on lane 0 in node order, which
  // is the order the sequential handlers would have queued them in
  bool bc = false;
  if (flag) {
    gx_fd_msg g;
    g.incarnation = (uint32_t)(w >> 32);
    g.node = (uint16_t)(base + lane);
    g.pad[0] = g.pad[1] = g.pad[2] = 0;
    if ((w & 0xffu) == GX_M_ALIVE) {
      g.from = (uint16_t)(base + lane);
      g.kind = GX_M_ALIVE;
      fd_alive_node(d, f, v, g, &bc);
    } else {
      g.from = (uint16_t)v;
      g.kind = GX_M_SUSPECT;
      fd_suspect_node(d, f, v, g, &bc);
    }
  }
  const unsigned long long qm = __ballot(bc);
  if (qm) {
    __threadfence_block();  // the lanes' row writes before other lanes read those rows
    fd_requeue_chunk(d, v, base, qm, bc);
    __threadfence_block();
  }
}
GXD void fd_row_fields(const Dev &d, uint32_t v, uint32_t m, uint4 &lo, uint4 &hi) {
  const uint4 *x = reinterpret_cast<const uint4 *>(memp(d, v, m));
  lo = x[0];  // incarnation, msg_incarnation, change_round, deadline
  hi = x[1];  // state, n_conf, tx, msg_kind | msg_from, susp_from[0] | susp_from[1], susp_from[2] | q_prev, q_next
}
// state.go mergeState into host v, node order: alive -> aliveNode, suspect or dead ->
// suspectNode{From: v}. One wave: the lanes test 64 nodes at a time for an effect (a superset of
// the nodes whose handler changes anything; a node's test reads only that node's row, which the
// handlers of other nodes do not change), run the flagged nodes' handlers side by side (each
// touches only its node's row), and lane 0 then moves the broadcast nodes in the queue in order.
GXD void fd_merge_state_wave(const Dev &d, FdAcc &f, uint32_t v, const uint64_t *remote) {
  const uint32_t lane = threadIdx.x & 63;
  const int64_t wrap = fdhp(d, v)->wrap_round, dead_rounds = d.p.fd_gossip_dead_rounds;
  unsigned present_n = 0;
  // the next chunk's remote words and row fields are loaded while this chunk is tested and handled
  // (the handlers touch only flagged nodes' rows and queue links, never the fields tested here)
  auto load = [&](uint32_t base, uint64_t &w, uint4 &lo, uint4 &hi) {
    const uint32_t m = base + lane;
    w = m < d.H ? remote[m] : FD_SNAP_ABSENT;
    if (m < d.H && (w & 0xffu) != FD_SNAP_ABSENT) fd_row_fields(d, v, m, lo, hi);
  };
  uint64_t w = 0, wn = 0;
  uint4 lo = make_uint4(0, 0, 0, 0), hi = lo, lon = lo, hin = lo;
  load(0, w, lo, hi);
  for (uint32_t base = 0; base < d.H; base += 64) {
    if (base + 64 < d.H) load(base + 64, wn, lon, hin);
    fd_merge_chunk(d, f, v, base, w, lo, hi, wrap, dead_rounds, present_n);
    w = wn;
    lo = lon;
    hi = hin;
  }
  f.inc(C_FD_STATE_MERGE, present_n);
  if (lane == 0) kbytes(d, GX_K_FD, 24ull * d.H, d.H);  // remote word + the node's row fields, per node
}
// Both directions of a push-pull pair (a, b) in one workgroup, chunk by chunk: wave 0 merges b's
// list into a's, wave 1 a's into b's. Each wave reads its own host's rows of a chunk, hands the
// partner the round-start words (incarnation << 32 | state, reaped = absent) through LDS, and the
// barrier keeps every read of a chunk ahead of both waves' handlers for it, so neither side
// needs a snapshot of the other's list (the handlers of a chunk touch only its nodes' rows).
GXD void fd_merge_pair_lockstep(const Dev &d, FdAcc &f, uint32_t a, uint32_t b, uint64_t *s_w) {
  const uint32_t lane = threadIdx.x & 63, side = threadIdx.x >> 6;
  const uint32_t v = side ? b : a;
  const int64_t wrap = fdhp(d, v)->wrap_round, dead_rounds = d.p.fd_gossip_dead_rounds;
  unsigned present_n = 0;
  uint4 lo = make_uint4(0, 0, 0, 0), hi = lo, lon = lo, hin = lo;
  if (lane < d.H) fd_row_fields(d, v, lane, lo, hi);
  for (uint32_t base = 0; base < d.H; base += 64) {
    const uint32_t m = base + lane;
    uint64_t mine = FD_SNAP_ABSENT;  // fd_snap_word of v's row for m
    if (m < d.H) {
      const uint32_t state = hi.x & 0xffu;
      const bool reaped = state == GX_M_DEAD && wrap - (int64_t)(int32_t)lo.z > dead_rounds;
      mine = reaped ? FD_SNAP_ABSENT : ((uint64_t)lo.x << 32) | state;
    }
    s_w[side * 64 + lane] = mine;
    __syncthreads();
    const uint64_t w = s_w[(1 - side) * 64 + lane];
    if (base + 64 + lane < d.H) fd_row_fields(d, v, base + 64 + lane, lon, hin);
    fd_merge_chunk(d, f, v, base, w, lo, hi, wrap, dead_rounds, present_n);
    __syncthreads();  // both waves are done with s_w
    lo = lon;
    hi = hin;
  }
  f.inc(C_FD_STATE_MERGE, present_n);
  if (lane == 0) kbytes(d, GX_K_FD, 32ull * d.H, d.H);  // the node's row fields, per node and side
}

// ---------------------------------------------------------------------------- kernels -----
__global__ void k_fd_init(Dev d) {
  const size_t n = (size_t)d.Hl * d.H;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    gx_member x;
    x.incarnation = 0;
    x.msg_incarnation = 0;
    x.change_round = 0;
    x.deadline = GX_FD_NO_DEADLINE;
    x.state = GX_M_ALIVE;
    x.n_conf = 0;
    x.tx = 0;
    x.msg_kind = 0;
    x.msg_from = GX_FD_NONE;
    x.susp_from[0] = x.susp_from[1] = x.susp_from[2] = GX_FD_NONE;
    x.q_prev = x.q_next = GX_FD_NONE;
    d.mem[i] = x;
    d.fd_dl[i] = GX_FD_NO_DEADLINE;
  }
  for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < d.Hl; v += (size_t)gridDim.x * blockDim.x) {
    gx_fd_host h;
    h.probe_pass = 0;
    h.probe_index = 0;
    h.wrap_round = INT32_MIN;
    h.min_deadline = GX_FD_NO_DEADLINE;
    h.q_len = 0;
    h.departed = 0;
    h.hq_len = 0;
    for (int b = 0; b < GX_FD_MAX_TX; b++) h.q_head[b] = GX_FD_NONE;
    d.fdh[v] = h;
  }
}

__global__ __launch_bounds__(64) void k_fd_tick(Dev d) {  // one wave per host of this engine
  Acc a;
  FdAcc f;
  const uint32_t v = d.lo + blockIdx.x;
  if (!departed(d, v)) {
    fd_timers_wave(d, a, f, v);
    if (threadIdx.x == 0 && fd_probe_tick(d, v)) {
      bool ack;
      fd_probe_host(d, f, v, &ack);
    }
  }
  acc_flush(d, a);
  fd_flush(d, f);
}

__global__ __launch_bounds__(64) void k_fd_send(Dev d) {  // one thread per host of this engine
  FdAcc f;
  const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x, u = d.lo + idx;
  if (idx < d.Hl) {
    const uint32_t K = d.K, KE = d.KE, NG = d.NG, cap = d.p.fd_msg_cap;
    for (uint32_t j = 0; j < KE; j++) d.fd_len[(size_t)idx * KE + j] = 0;
    uint32_t np = 0;
    if (!departed(d, u)) {
      uint32_t peers[16];
      np = fd_sample_peers(d, u, peers);
      const uint32_t budget = fd_budget(d);
      for (uint32_t j = 0; j < np; j++) {
        d.fd_peers[(size_t)idx * K + j] = peers[j];
        // GossipMessages: each of the target's gathers (packet entry j * NG + n) takes memberlist's
        // messages first; the queue only shrinks during the gathers, so once a gather finds it
        // empty the later ones do too (and the target's gathering goes on only while the
        // delegate's part is not empty, k_send)
        for (uint32_t n = 0; n < NG; n++) {
          const size_t x = (size_t)idx * KE + (size_t)j * NG + n;
          const uint32_t l = fd_get_broadcasts(d, f, u, budget, &d.fdm[x * cap]);
          d.fd_len[x] = l;
          if (!l) break;
        }
      }
    }
    d.fd_np[idx] = np;
  }
  fd_flush(d, f);
}

// gx.h fd_handoff_shared: a receiver whose catalog lock blocks NotifyMsg takes its packets' items
// in arrival order, memberlist's messages of a packet before its records (k_merge_seg leaves such
// receivers to this kernel): a memberlist message is handled at once while the handler is not yet
// blocked (fewer than GX_LOCK_HANDLER_AT items held), else it queues in the handoff queue or is
// dropped at a full pipeline; records go to the pipeline as in k_merge_seg. Oracle: ph_receive.
GXD void fd_handoff_locked(const Dev &d, Acc &a, FdAcc &f, uint32_t vi, uint32_t lw) {
  const uint32_t v = d.lo + vi, cnt = d.in_cnt[vi], capv = pipe_cap(d, vi, lw), fcap = d.p.fd_msg_cap;
  const bool now_ok = !departed(d, v);
  uint32_t nb = GX_LOCK_BUF(lw), nq = d.fdh[vi].hq_len;
  grec *lkb = &d.lkb[(size_t)vi * d.C];
  gx_fd_msg *q = &d.fdq[(size_t)vi * d.HQ];
  int64_t after = -1;
  for (uint32_t n = 0; n < cnt; n++) {
    const uint4 hx = inbox_next(d, vi, after);
    after = hx.x;
    const uint32_t nf = d.fd_len[hx.y];
    const gx_fd_msg *pk = &d.fdm[(size_t)hx.y * fcap];
    if (nb + nq < GX_LOCK_HANDLER_AT) {
      if (now_ok)
        for (uint32_t y = 0; y < nf; y++) fd_handle(d, a, f, v, pk[y]);
    } else {
      for (uint32_t y = 0; y < nf; y++) {
        if (nb + nq < capv) {
          q[nq++] = pk[y];
          f.inc(C_FD_HQ);
        } else {
          f.inc(C_FD_HQ_DROP);
        }
      }
    }
    const grec *pr = packet_recs(d, vi, hx.w, hx.y);
    for (uint32_t x = 0; x < hx.z; x++) {
      if (nb + nq < capv) {
        lkb[nb++] = pr[x];
        a.c[C_LOCK_BUF]++;
      } else {
        a.c[C_LOCK_DROP]++;
      }
    }
  }
  if (cnt) {  // (a deadNode handled above may have set the waiting-ExpireServer bit: reread the word)
    d.hs[vi].lock = (d.hs[vi].lock & ((1u << GX_LOCK_BUF_SHIFT) - 1u)) | nb << GX_LOCK_BUF_SHIFT;
    d.fdh[vi].hq_len = nq;
  }
}
__global__ __launch_bounds__(64) void k_fd_recv(Dev d) {  // one thread per receiver of this engine
  Acc a;
  FdAcc f;
  const uint32_t vi = blockIdx.x * blockDim.x + threadIdx.x, v = d.lo + vi;
  const uint32_t lw = vi < d.Hl && d.p.fd_handoff_shared ? d.hs[vi].lock : 0u;
  if (vi < d.Hl && d.p.fd_handoff_shared && locked_in(d, lw)) {
    fd_handoff_locked(d, a, f, vi, lw);
  } else if (vi < d.Hl && !departed(d, v)) {
    const uint32_t cap = d.p.fd_msg_cap;
    if (d.p.fd_handoff_shared && d.fdh[vi].hq_len) {  // the handoff queue drains first (unlocked now)
      const uint32_t n = d.fdh[vi].hq_len;
      d.fdh[vi].hq_len = 0;
      for (uint32_t k = 0; k < n; k++) fd_handle(d, a, f, v, d.fdq[(size_t)vi * d.HQ + k]);
    }
    // the packets' messages are read-only here: the next one is loaded before the current
    // message's handler runs, so its load is not ordered behind the handler's row writes
    // the inbox in sender order (a selection walk over the few headers)
    const uint32_t cnt = d.in_cnt[vi];
    int64_t after = -1;
    for (uint32_t x = 0; x < cnt; x++) {
      const uint4 hx = inbox_next(d, vi, after);
      after = hx.x;
      const uint32_t e = hx.y, n = d.fd_len[e];
      const gx_fd_msg *pk = &d.fdm[(size_t)e * cap];
      gx_fd_msg cur = n ? pk[0] : gx_fd_msg{};
      for (uint32_t y = 0; y < n; y++) {
        const gx_fd_msg nxt = y + 1 < n ? pk[y + 1] : cur;
        fd_handle(d, a, f, v, cur);
        cur = nxt;
      }
    }
  }
  acc_flush(d, a);
  fd_flush(d, f);
}

// Round-start member lists of this engine's hosts (push-pull), one thread per (host, node).
__global__ void k_fd_snap(Dev d) {
  const size_t n = (size_t)d.Hl * d.H;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    d.fd_snap[i] = fd_snap_word(d, d.lo + (uint32_t)(i / d.H), (uint32_t)(i % d.H));
  if (blockIdx.x == 0 && threadIdx.x == 0) kbytes(d, GX_K_FD, 20ull * n, n);  // 12 B of row read, 8 B written
}
GXD const uint64_t *snap_row(const Dev &d, uint32_t v) { return &d.fd_snap[(size_t)li(d, v) * d.H]; }
// pushPull runs when both are up, the path exists and the initiator a sees b alive at round start
GXD bool pp_runs(const Dev &d, uint32_t a, uint32_t b) {
  return !departed(d, a) && !departed(d, b) && reach(d, a, b) && (snap_row(d, a)[b] & 0xffu) == GX_M_ALIVE;
}
// Unsharded push-pull round: pair t as k_ae derives it; wave 2t merges b's list into a, 2t+1 a's into b.
// Unsharded push-pull membership: one 128-thread workgroup per pair, both directions in lockstep.
__global__ __launch_bounds__(128) void k_fd_pushpull_pair(Dev d, uint64_t key0, uint64_t key1) {
  __shared__ uint64_t s_w[128];
  __shared__ uint32_t s_run;
  FdAcc f;
  const uint32_t t = blockIdx.x;
  uint32_t base = 0, m = d.H, q = t;
  uint64_t key = key0;
  if (d.pair_split) {
    uint32_t m0 = d.H / 2, np0 = m0 / 2;
    if (t < np0) {
      m = m0;
    } else {
      base = m0;
      m = d.H - m0;
      q = t - np0;
      key = key1;
    }
  }
  const uint32_t a = base + feistel_perm(key, 2 * q, m), b = base + feistel_perm(key, 2 * q + 1, m);
  if (threadIdx.x == 0)  // pp_runs on the lists as this phase starts (nothing merged yet); a side that
    // holds the ServicesState lock fails the whole exchange (gx.h lock_model) unless only readers
    // hold it (lock_readers: ro_flag, cleared by k_ae_ro after this launch)
    s_run = !departed(d, a) && !departed(d, b) && reach(d, a, b) && (fd_snap_word(d, a, b) & 0xffu) == GX_M_ALIVE &&
            !(d.p.lock_model && (host_locked(d, a) || host_locked(d, b)) && !(d.p.lock_readers && d.ro_flag[t]));
  __syncthreads();
  if (s_run) fd_merge_pair_lockstep(d, f, a, b, s_w);
  fd_flush(d, f);
}
// Sharded push-pull round over the plan (ae_plan): a local pair merges both ways from the local
// lists; a cross pair merges the partner's list received with the digests (rsnap row k) into this
// side's host unless the pair does not run.
__global__ __launch_bounds__(64) void k_fd_pushpull_plan(Dev d, const uint32_t *pa, const uint32_t *pb,
                                                          const int32_t *prow, const uint8_t *skip,
                                                          const uint64_t *rsnap) {
  FdAcc f;
  const uint32_t i = blockIdx.x >> 1, side = blockIdx.x & 1;
  const int32_t k = prow[i];
  if (k < 0) {
    if (pp_runs(d, pa[i], pb[i]) && !(d.p.lock_model && (host_locked(d, pa[i]) || host_locked(d, pb[i]))))
      fd_merge_state_wave(d, f, side ? pb[i] : pa[i], snap_row(d, side ? pa[i] : pb[i]));
  } else if (side == 0 && !(skip[k] & 1u)) {
    fd_merge_state_wave(d, f, pa[i], &rsnap[(size_t)k * d.H]);
  }
  fd_flush(d, f);
}
// The partner lists of this round's cross pairs, out of the digest inbox (message k).
__global__ void k_fd_rsnap(Dev d, const uint8_t *in, size_t dig_bytes, uint32_t nblk, uint32_t n, uint64_t *rsnap) {
  const size_t tot = (size_t)n * d.H;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (size_t)gridDim.x * blockDim.x) {
    const size_t k = i / d.H, x = i % d.H;
    rsnap[i] = *reinterpret_cast<const uint64_t *>(in + k * dig_bytes + 16 + 16ull * nblk + 8 * x);
  }
}

// Single-host ABI kernels (one wave; lane 0 runs the handler logic).
__global__ __launch_bounds__(64) void k_fd_api_notify(Dev d, uint32_t v, const gx_fd_msg *msgs, uint32_t n) {
  Acc a;
  FdAcc f;
  if (threadIdx.x == 0)
    for (uint32_t i = 0; i < n; i++) fd_handle(d, a, f, v, msgs[i]);
  acc_flush(d, a);
  fd_flush(d, f);
}
__global__ __launch_bounds__(64) void k_fd_api_getb(Dev d, uint32_t v, uint32_t limit, gx_fd_msg *out, uint32_t *n_out) {
  FdAcc f;
  if (threadIdx.x == 0) *n_out = fd_get_broadcasts(d, f, v, limit, out);
  fd_flush(d, f);
}
__global__ __launch_bounds__(64) void k_fd_api_probe(Dev d, uint32_t v, uint32_t *out) {
  FdAcc f;
  if (threadIdx.x == 0) {
    bool ack;
    out[0] = fd_probe_host(d, f, v, &ack);
    out[1] = ack;
  }
  fd_flush(d, f);
}
__global__ __launch_bounds__(64) void k_fd_api_timers(Dev d, uint32_t v) {
  Acc a;
  FdAcc f;
  fd_timers_wave(d, a, f, v);
  acc_flush(d, a);
  fd_flush(d, f);
}

// Membership agreement with the truth (gx_fd_converged): one thread per node m reads column m of
// the member lists (adjacent threads, adjacent nodes: coalesced rows).
__global__ void k_fd_converged(Dev d, unsigned long long *bad) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  bool dis = false;
  if (m < d.H) {  // over this engine's live hosts
    const uint8_t want = departed(d, m) ? GX_M_DEAD : GX_M_ALIVE;
    for (uint32_t v = d.lo; v < d.lo + d.Hl && !dis; v++)
      dis = !departed(d, v) && memp(d, v, m)->state != want;
  }
  unsigned long long c = wave_sum(dis ? 1ull : 0ull);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(bad, c);
}
__global__ __launch_bounds__(64) void k_fd_api_merge_state(Dev d, uint32_t v, const uint64_t *remote) {
  FdAcc f;
  fd_merge_state_wave(d, f, v, remote);
  fd_flush(d, f);
}

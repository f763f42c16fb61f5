/*
 * gx_oracle_fd.c — CPU ORACLE of memberlist failure detection. TEST
 * INFRASTRUCTURE ONLY; #included by gx_oracle.c (one translation unit).
 *
 * memberlist is absent from the reference tree: github.com/NinesStack/memberlist
 * v0.0.0-20170522194404-cfac2b5cf519 (reference go.mod:6, go.sum:8-9), a fork of
 * hashicorp/memberlist. Sidecar configures it with DefaultLANConfig (main.go:243-261) and only
 * reacts to NotifyLeave -> go ExpireServer(node) (services_delegate.go:173-176); NotifyJoin and
 * NotifyUpdate log (:169-171, :178-180). This file restates the published algorithm of that
 * library, sequentially, per simulated host:
 *   probe()/probeNode()         state.go: round-robin over a shuffled node list, skipping self
 *                               and dead nodes; direct probe, then IndirectChecks relays picked
 *                               by kRandomNodes among alive nodes; no ack -> suspectNode
 *   suspectNode/deadNode/aliveNode/refute   state.go message handlers, incarnation rules
 *   suspicion                    suspicion.go (Lifeguard): timeout max, shrinking towards min
 *                               with log(c+1)/log(k+1) over c independent confirmations
 *   TransmitLimitedQueue         queue.go: one queued message per node (newer invalidates),
 *                               fewest transmits first, newest first among equals, each message
 *                               sent retransmitLimit times
 *   kRandomNodes / gossip filter util.go, state.go gossip(): alive, suspect, and dead nodes
 *                               within GossipToTheDeadTime
 *   resetNodes                  state.go: at each wrap of the probe list, dead nodes older than
 *                               GossipToTheDeadTime are reaped (here: lazily, via wrap_round)
 * The round-model resolutions (phase order, fixed n, reaping, push-pull pairing) are in
 * DESIGN.md §3b. Parity against the fork itself is unpinned: no reference test exercises it.
 */

enum { ST_FD_PHASE = 8, ST_FD_PERM = 9, ST_FD_RELAY = 10, ST_DEPART = 11 };

#define MEM(e, v, m) (&(e)->mem[(size_t)(v) * (e)->H + (m)])

static int departed_at(const gx_params *p, int64_t round, uint32_t u) {
  if (p->depart_round < 0 || round < p->depart_round || !p->depart_ppm) return 0;
  return (uint32_t)(rng4(p->seed, ST_DEPART, u, 0, 0) % 1000000ull) < p->depart_ppm;
}
static int departed(const gx_engine *e, uint32_t u) { return departed_at(&e->p, e->round, u); }

/* Network reachability a -> b this round: a crashed host sends and answers nothing; with the
 * failure detector on, the partition is a network property (packets across it are lost). */
static int reach(const gx_engine *e, uint32_t a, uint32_t b) {
  if (departed(e, a) || departed(e, b)) return 0;
  if (partitioned(e) && ((a < e->H / 2) != (b < e->H / 2))) return 0;
  return 1;
}

/* util.go suspicionTimeout / suspicion.go remainingSuspicionTime / util.go retransmitLimit. */
int gx_fd_defaults(gx_params *p) {
  if (!p || p->n_hosts < 1 || p->fd_probe_rounds < 1 || p->round_ns <= 0) return GX_EINVAL;
  const int mult = 4, max_mult = 6, retransmit_mult = 4;
  double n = (double)p->n_hosts;
  p->fd_retransmit_limit = (uint32_t)(retransmit_mult * (int)ceil(log10(n + 1.0)));
  if (p->fd_retransmit_limit > GX_FD_MAX_TX) p->fd_retransmit_limit = GX_FD_MAX_TX;
  double scale = fmax(1.0, log10(fmax(1.0, n)));
  int64_t interval = (int64_t)p->fd_probe_rounds * p->round_ns;
  int64_t min_ns = (int64_t)mult * (int64_t)(scale * 1000.0) * interval / 1000;
  int64_t max_ns = (int64_t)max_mult * min_ns;
  int k = mult - 2;
  if ((int)p->n_hosts - 2 < k) k = 0;
  p->fd_suspicion_k = (uint32_t)k;
  for (int c = 0; c < 8; c++) {
    int64_t t;
    if (c == 0) {
      t = k < 1 ? min_ns : max_ns;
    } else if (c > k) {
      t = min_ns;
    } else {
      double frac = log((double)c + 1.0) / log((double)k + 1.0);
      double raw = (double)max_ns / 1e9 - frac * ((double)max_ns / 1e9 - (double)min_ns / 1e9);
      t = (int64_t)floor(1000.0 * raw) * 1000000ll;
      if (t < min_ns) t = min_ns;
    }
    p->fd_suspicion_rounds[c] = (uint32_t)((t + p->round_ns - 1) / p->round_ns);
  }
  return GX_OK;
}

/* A dead node older than GossipToTheDeadTime at the host's last resetNodes is no longer in its
 * member list: messages about it are ignored, an alive message re-adds it (aliveNode). */
static int fd_reaped(const gx_engine *e, uint32_t v, const gx_member *x) {
  return x->state == GX_M_DEAD &&
         (int64_t)e->fdh[v].wrap_round - (int64_t)x->change_round > (int64_t)e->p.fd_gossip_dead_rounds;
}

/* ------------------------------------------------------------ TransmitLimitedQueue -------- */
static void q_unlink(gx_engine *e, uint32_t v, uint32_t m) {
  gx_member *x = MEM(e, v, m);
  gx_fd_host *h = &e->fdh[v];
  if (x->q_prev != GX_FD_NONE) MEM(e, v, x->q_prev)->q_next = x->q_next;
  else h->q_head[x->tx - 1] = x->q_next;
  if (x->q_next != GX_FD_NONE) MEM(e, v, x->q_next)->q_prev = x->q_prev;
  x->q_prev = x->q_next = GX_FD_NONE;
  x->tx = 0;
  h->q_len--;
}
static void q_push(gx_engine *e, uint32_t v, uint32_t m, uint32_t b) { /* newest of bucket b */
  gx_member *x = MEM(e, v, m);
  gx_fd_host *h = &e->fdh[v];
  x->q_prev = GX_FD_NONE;
  x->q_next = h->q_head[b];
  if (h->q_head[b] != GX_FD_NONE) MEM(e, v, h->q_head[b])->q_prev = (uint16_t)m;
  h->q_head[b] = (uint16_t)m;
  x->tx = (uint8_t)(b + 1);
  h->q_len++;
}
/* encodeAndBroadcast -> QueueBroadcast: the new message about m invalidates the queued one. */
static void fd_broadcast(gx_engine *e, uint32_t v, uint32_t m, int kind, uint32_t inc, uint32_t from) {
  gx_member *x = MEM(e, v, m);
  if (x->tx) q_unlink(e, v, m);
  x->msg_kind = (uint8_t)kind;
  x->msg_incarnation = inc;
  x->msg_from = (uint16_t)from;
  q_push(e, v, m, 0);
}
/* TransmitLimitedQueue.GetBroadcasts with a message budget: the first `limit` messages in queue
 * order; each moves to the newest end of the next transmit count (keeping their order), or
 * leaves the queue once sent fd_retransmit_limit times. */
static uint32_t fd_get_broadcasts(gx_engine *e, uint32_t v, uint32_t limit, gx_fd_msg *out) {
  uint16_t taken[64];
  uint8_t from_b[64];
  uint32_t n = 0, L = e->p.fd_retransmit_limit;
  if (limit > 64) limit = 64;
  for (uint32_t b = 0; b < L && n < limit; b++)
    for (uint32_t m = e->fdh[v].q_head[b]; m != GX_FD_NONE && n < limit; m = MEM(e, v, m)->q_next) {
      taken[n] = (uint16_t)m;
      from_b[n] = (uint8_t)b;
      n++;
    }
  for (uint32_t i = 0; i < n; i++) {
    const gx_member *x = MEM(e, v, taken[i]);
    out[i].incarnation = x->msg_incarnation;
    out[i].node = taken[i];
    out[i].from = x->msg_from;
    out[i].kind = x->msg_kind;
    out[i].pad[0] = out[i].pad[1] = out[i].pad[2] = 0;
    q_unlink(e, v, taken[i]);
  }
  for (uint32_t i = n; i-- > 0;)
    if ((uint32_t)from_b[i] + 1 < L) q_push(e, v, taken[i], from_b[i] + 1u);
  e->st.fd_msgs_sent += n;
  return n;
}

/* ------------------------------------------------------------------- message handlers ----- */
static void fd_set_deadline(gx_engine *e, uint32_t v, gx_member *x, int64_t dl) {
  if (dl > GX_FD_NO_DEADLINE - 1) dl = GX_FD_NO_DEADLINE - 1;
  x->deadline = (int32_t)dl;
  if (x->deadline < e->fdh[v].min_deadline) e->fdh[v].min_deadline = x->deadline;
}

/* refute(): beat the accusation with a higher own incarnation and broadcast alive. */
static void fd_refute(gx_engine *e, uint32_t v, uint32_t accused) {
  gx_member *me = MEM(e, v, v);
  uint32_t inc = me->incarnation + 1;
  if (accused >= inc) inc = accused + 1;
  me->incarnation = inc;
  fd_broadcast(e, v, v, GX_M_ALIVE, inc, v);
  e->st.fd_refutes++;
}

/* deadNode (state.go); NotifyLeave -> ExpireServer (services_delegate.go:173-176). */
static void fd_dead_node(gx_engine *e, uint32_t v, const gx_fd_msg *d, int64_t now) {
  uint32_t m = d->node;
  gx_member *x = MEM(e, v, m);
  if (fd_reaped(e, v, x)) return;
  if (d->incarnation < x->incarnation) return;
  x->deadline = GX_FD_NO_DEADLINE; /* delete(m.nodeTimers, d.Node) */
  if (x->state == GX_M_DEAD) return;
  if (m == v) {
    fd_refute(e, v, d->incarnation);
    return;
  }
  fd_broadcast(e, v, m, GX_M_DEAD, d->incarnation, d->from);
  x->incarnation = d->incarnation;
  x->state = GX_M_DEAD;
  x->change_round = (int32_t)e->round;
  e->st.fd_deaths++;
  notify_leave(e, v, m, now);
}

/* suspicion.Confirm: one confirmation per distinct accuser, at most k; the deadline moves to
 * start + timeout(c). A deadline already past fires at the next timer phase. */
static int fd_confirm(gx_engine *e, uint32_t v, gx_member *x, uint32_t from) {
  if (x->n_conf >= e->p.fd_suspicion_k) return 0;
  for (uint32_t i = 0; i <= x->n_conf; i++)
    if (x->susp_from[i] == from) return 0;
  x->susp_from[1 + x->n_conf] = (uint16_t)from;
  x->n_conf++;
  x->deadline = GX_FD_NO_DEADLINE;
  fd_set_deadline(e, v, x, (int64_t)x->change_round + e->p.fd_suspicion_rounds[x->n_conf]);
  e->st.fd_confirmations++;
  return 1;
}

/* suspectNode (state.go). A suspicion timer exists exactly while the node is SUSPECT. */
static void fd_suspect_node(gx_engine *e, uint32_t v, const gx_fd_msg *s) {
  uint32_t m = s->node;
  gx_member *x = MEM(e, v, m);
  if (fd_reaped(e, v, x)) return;
  if (s->incarnation < x->incarnation) return;
  if (x->state == GX_M_SUSPECT) {
    if (fd_confirm(e, v, x, s->from)) fd_broadcast(e, v, m, GX_M_SUSPECT, s->incarnation, s->from);
    return;
  }
  if (x->state != GX_M_ALIVE) return;
  if (m == v) {
    fd_refute(e, v, s->incarnation);
    return;
  }
  fd_broadcast(e, v, m, GX_M_SUSPECT, s->incarnation, s->from);
  x->incarnation = s->incarnation;
  x->state = GX_M_SUSPECT;
  x->change_round = (int32_t)e->round;
  x->n_conf = 0;
  x->susp_from[0] = (uint16_t)s->from;
  x->susp_from[1] = x->susp_from[2] = GX_FD_NONE;
  fd_set_deadline(e, v, x, e->round + (int64_t)e->p.fd_suspicion_rounds[0]);
  e->st.fd_suspicions++;
}

/* aliveNode (state.go). An unknown (reaped) node is re-added as dead with incarnation 0 first. */
static void fd_alive_node(gx_engine *e, uint32_t v, const gx_fd_msg *a) {
  uint32_t m = a->node;
  gx_member *x = MEM(e, v, m);
  if (fd_reaped(e, v, x)) {
    x->state = GX_M_DEAD;
    x->incarnation = 0;
    x->change_round = INT32_MIN;
  }
  if (m == v) { /* about us: ignore the same incarnation, refute a newer one */
    if (a->incarnation <= x->incarnation) return;
    uint32_t inc = x->incarnation + 1;
    if (a->incarnation >= inc) inc = a->incarnation + 1;
    x->incarnation = inc;
    fd_broadcast(e, v, v, GX_M_ALIVE, inc, v);
    e->st.fd_refutes++;
    return;
  }
  if (a->incarnation <= x->incarnation) return;
  x->deadline = GX_FD_NO_DEADLINE; /* delete(m.nodeTimers, a.Node) */
  fd_broadcast(e, v, m, GX_M_ALIVE, a->incarnation, a->from);
  x->incarnation = a->incarnation;
  if (x->state != GX_M_ALIVE) {
    x->state = GX_M_ALIVE;
    x->change_round = (int32_t)e->round;
  }
  x->n_conf = 0;
  e->st.fd_alive_updates++; /* dead -> alive: NotifyJoin, which Sidecar only logs */
}

static void fd_handle(gx_engine *e, uint32_t v, const gx_fd_msg *g, int64_t now) {
  if (g->node >= e->H) return;
  if (g->kind == GX_M_ALIVE) fd_alive_node(e, v, g);
  else if (g->kind == GX_M_SUSPECT) fd_suspect_node(e, v, g);
  else if (g->kind == GX_M_DEAD) fd_dead_node(e, v, g, now);
  e->st.fd_msgs_received++;
}

/* ------------------------------------------------- push-pull membership (mergeState) ------ */
/* A host's member list as pushPull sends it (round-start snapshot): incarnation << 32 | state per
 * node, FD_SNAP_ABSENT for a reaped node (no longer in its list). */
#define FD_SNAP_ABSENT 0xffull
static uint64_t fd_snap_word(const gx_engine *e, uint32_t v, uint32_t m) {
  const gx_member *x = MEM(e, v, m);
  if (fd_reaped(e, v, x)) return FD_SNAP_ABSENT;
  return ((uint64_t)x->incarnation << 32) | x->state;
}
static void fd_snapshot_row(const gx_engine *e, uint32_t v, uint64_t *out) {
  for (uint32_t m = 0; m < e->H; m++) out[m] = fd_snap_word(e, v, m);
}
/* state.go mergeState, node order: alive -> aliveNode; suspect or dead -> suspectNode{From: us}
 * ("we prefer to suspect that node instead of declaring it dead instantly"). */
static void fd_merge_state(gx_engine *e, uint32_t v, const uint64_t *remote) {
  for (uint32_t m = 0; m < e->H; m++) {
    uint64_t w = remote[m];
    if ((w & 0xffu) == FD_SNAP_ABSENT) continue;
    gx_fd_msg g = {(uint32_t)(w >> 32), (uint16_t)m, (uint16_t)m, GX_M_ALIVE, {0, 0, 0}};
    e->st.fd_state_merges++;
    if ((w & 0xffu) == GX_M_ALIVE) {
      fd_alive_node(e, v, &g);
    } else {
      g.kind = GX_M_SUSPECT;
      g.from = (uint16_t)v;
      fd_suspect_node(e, v, &g);
    }
  }
}

/* ------------------------------------------------------------------ timers and probes ----- */
/* Suspicion timers due this round, in node order: deadNode{incarnation, node, From: self}. */
static void fd_timers_host(gx_engine *e, uint32_t v, int64_t now) {
  gx_fd_host *h = &e->fdh[v];
  if (h->min_deadline > e->round) return;
  int32_t mn = GX_FD_NO_DEADLINE;
  for (uint32_t m = 0; m < e->H; m++) {
    gx_member *x = MEM(e, v, m);
    if (x->deadline <= e->round) {
      gx_fd_msg d = {x->incarnation, (uint16_t)m, (uint16_t)v, GX_M_DEAD, {0, 0, 0}};
      fd_dead_node(e, v, &d, now);
    } else if (x->deadline < mn) {
      mn = x->deadline;
    }
  }
  h->min_deadline = mn;
}

/* probe(): the next node of the shuffled list that is neither us nor dead (numCheck bounds the
 * walk); probeNode(): direct probe, then IndirectChecks relays (kRandomNodes over alive nodes
 * other than us and the target, at most 3n draws); no ack -> suspectNode{inc, node, From: us}. */
static uint32_t fd_probe_host(gx_engine *e, uint32_t v, int *acked) {
  gx_fd_host *h = &e->fdh[v];
  uint32_t H = e->H, t = GX_FD_NONE, num_check = 0;
  *acked = 0;
  while (num_check < H) {
    if (h->probe_index >= H) { /* resetNodes: reap, reshuffle */
      h->probe_pass++;
      h->probe_index = 0;
      h->wrap_round = (int32_t)e->round;
      num_check++;
      continue;
    }
    uint32_t c = feistel_perm(rng4(e->p.seed, ST_FD_PERM, v, h->probe_pass, 0), h->probe_index, H);
    h->probe_index++;
    if (c == v || MEM(e, v, c)->state == GX_M_DEAD) {
      num_check++;
      continue;
    }
    t = c;
    break;
  }
  if (t == GX_FD_NONE) return t;
  e->st.fd_probes++;
  int ack = reach(e, v, t);
  if (!ack) {
    uint32_t relays[16], nr = 0, want = e->p.fd_indirect_checks;
    for (uint32_t a = 0; nr < want && a < 3u * H; a++) {
      uint32_t r = unif(rng4(e->p.seed, ST_FD_RELAY, (uint64_t)e->round, v, a), H);
      if (r == v || r == t || MEM(e, v, r)->state != GX_M_ALIVE) continue;
      int dup = 0;
      for (uint32_t i = 0; i < nr; i++) dup |= relays[i] == r;
      if (!dup) relays[nr++] = r;
    }
    for (uint32_t i = 0; i < nr; i++)
      if (reach(e, v, relays[i]) && reach(e, relays[i], t)) ack = 1;
  }
  if (!ack) {
    e->st.fd_probe_failures++;
    gx_fd_msg s = {MEM(e, v, t)->incarnation, (uint16_t)t, (uint16_t)v, GX_M_SUSPECT, {0, 0, 0}};
    fd_suspect_node(e, v, &s);
  }
  *acked = ack;
  return t;
}

static int fd_probe_tick(const gx_engine *e, uint32_t v) {
  uint32_t P = e->p.fd_probe_rounds;
  return (uint64_t)e->round % P == rng4(e->p.seed, ST_FD_PHASE, v, 0, 0) % P;
}

/* gossip(): kRandomNodes(GossipNodes) over the member list, skipping us and nodes dead for more
 * than GossipToTheDeadTime (at most 3n draws). */
static uint32_t fd_sample_peers(const gx_engine *e, uint32_t u, uint32_t *peers) {
  uint32_t H = e->H, cnt = 0;
  if (H < 2) return 0;
  for (uint32_t a = 0; cnt < e->K && a < 3u * H; a++) {
    uint32_t p = unif(rng4(e->p.seed, ST_PEER, (uint64_t)e->round, u, a), H);
    if (p == u) continue;
    const gx_member *x = MEM(e, u, p);
    if (x->state == GX_M_DEAD && e->round - (int64_t)x->change_round > (int64_t)e->p.fd_gossip_dead_rounds) continue;
    int dup = 0;
    for (uint32_t i = 0; i < cnt; i++) dup |= peers[i] == p;
    if (!dup) peers[cnt++] = p;
  }
  return cnt;
}

/* memberlist messages one gossip packet can take: fd_msg_cap, and in byte mode what fits the
 * limit at fd_msg_bytes + 2 (compoundOverhead) each. */
static uint32_t fd_budget(const gx_engine *e) {
  uint32_t b = e->p.fd_msg_cap;
  if (e->p.limit_bytes) {
    uint32_t f = e->p.limit_bytes / (e->p.fd_msg_bytes + 2);
    if (f < b) b = f;
  }
  return b;
}

/* Round phases: timers and probes after the owner phase, memberlist messages of
 * the packets after the catalog merge. */
static void ph_fd_tick(gx_engine *e, uint32_t i, void *ctx) {
  int64_t now = *(const int64_t *)ctx;
  uint32_t v = e->lo + i;
  if (departed(e, v)) return;
  fd_timers_host(e, v, now);
  if (fd_probe_tick(e, v)) {
    int acked;
    fd_probe_host(e, v, &acked);
  }
}
static void ph_fd_send(gx_engine *e, uint32_t i, void *ctx) {
  (void)ctx;
  uint32_t u = e->lo + i, K = e->K, KE = e->KE, NG = e->NG, cap = e->p.fd_msg_cap;
  e->fd_np[u] = 0;
  for (uint32_t j = 0; j < KE; j++) e->fd_len[(size_t)u * KE + j] = 0;
  if (departed(e, u)) return;
  uint32_t peers[64];
  uint32_t np = fd_sample_peers(e, u, peers), budget = fd_budget(e);
  e->fd_np[u] = np;
  for (uint32_t j = 0; j < np; j++) {
    e->fd_peers[(size_t)u * K + j] = peers[j];
    /* GossipMessages (the fork's gossip(): up to N gathers per target, memberlist's queue first in
     * each); the queue only shrinks while gathering, so a gather that finds it empty ends its part */
    for (uint32_t n = 0; n < NG; n++) {
      size_t x = (size_t)u * KE + (size_t)j * NG + n;
      uint32_t l = fd_get_broadcasts(e, u, budget, &e->fdm[x * cap]);
      e->fd_len[x] = l;
      if (!l) break;
    }
  }
}
static void ph_fd_receive(gx_engine *e, uint32_t i, void *ctx) {
  int64_t now = *(const int64_t *)ctx;
  uint32_t v = e->lo + i, cap = e->p.fd_msg_cap;
  if (departed(e, v)) return;
  if (e->fdh[v].hq_len && !locked_at(e, v)) { /* gx.h fd_handoff_shared: the handoff queue drains first */
    const uint32_t n = e->fdh[v].hq_len;
    e->fdh[v].hq_len = 0;
    for (uint32_t k = 0; k < n; k++) fd_handle(e, v, &e->fdq[(size_t)v * e->HQ + k], now);
  }
  for (uint32_t x = e->in_cnt[v]; x < e->in_cnt[v + 1]; x++) {
    uint32_t m = e->in_list[x];
    for (uint32_t y = 0; y < e->fd_len[m]; y++) fd_handle(e, v, &e->fdm[(size_t)m * cap + y], now);
  }
}

static void fd_init(gx_engine *e) {
  if (!e->p.fd_enable) return;
  for (size_t i = 0; i < (size_t)e->H * e->H; i++) {
    gx_member *x = &e->mem[i];
    memset(x, 0, sizeof(*x));
    x->deadline = GX_FD_NO_DEADLINE;
    x->msg_from = GX_FD_NONE;
    x->susp_from[0] = x->susp_from[1] = x->susp_from[2] = GX_FD_NONE;
    x->q_prev = x->q_next = GX_FD_NONE;
  }
  for (uint32_t v = 0; v < e->H; v++) {
    gx_fd_host *h = &e->fdh[v];
    memset(h, 0, sizeof(*h));
    h->wrap_round = INT32_MIN;
    h->min_deadline = GX_FD_NO_DEADLINE;
    for (int b = 0; b < GX_FD_MAX_TX; b++) h->q_head[b] = GX_FD_NONE;
  }
}

/* ------------------------------------------------------------------------------ ABI ------ */
static int fd_host_ok(const gx_engine *e, uint32_t host) { return e && e->p.fd_enable && host < e->H && is_local(e, host); }

int gx_fd_read_members(gx_engine *e, uint32_t host, uint32_t lo, uint32_t hi, gx_member *out) {
  if (!fd_host_ok(e, host) || lo > hi || hi > e->H || (!out && hi > lo)) return GX_EINVAL;
  memcpy(out, MEM(e, host, lo), sizeof(gx_member) * (hi - lo));
  return GX_OK;
}
int gx_fd_read_hosts(gx_engine *e, uint32_t lo, uint32_t hi, gx_fd_host *out) {
  if (!e || !e->p.fd_enable || lo > hi || (hi > lo && (!is_local(e, lo) || !is_local(e, hi - 1))) || (!out && hi > lo))
    return GX_EINVAL;
  for (uint32_t v = lo; v < hi; v++) {
    out[v - lo] = e->fdh[v];
    out[v - lo].departed = (uint32_t)departed(e, v);
  }
  return GX_OK;
}
int gx_fd_read_queue(gx_engine *e, uint32_t host, gx_fd_msg *out, uint8_t *transmits, uint32_t cap,
                     uint32_t *n_out) {
  if (!fd_host_ok(e, host) || !n_out) return GX_EINVAL;
  uint32_t n = 0;
  for (uint32_t b = 0; b < e->p.fd_retransmit_limit; b++)
    for (uint32_t m = e->fdh[host].q_head[b]; m != GX_FD_NONE; m = MEM(e, host, m)->q_next) {
      if (n < cap) {
        const gx_member *x = MEM(e, host, m);
        if (out) {
          gx_fd_msg g = {x->msg_incarnation, (uint16_t)m, x->msg_from, x->msg_kind, {0, 0, 0}};
          out[n] = g;
        }
        if (transmits) transmits[n] = (uint8_t)b;
      }
      n++;
    }
  *n_out = n;
  return GX_OK;
}
int gx_fd_notify(gx_engine *e, uint32_t host, const gx_fd_msg *msgs, uint32_t n) {
  if (!fd_host_ok(e, host) || (!msgs && n)) return GX_EINVAL;
  for (uint32_t i = 0; i < n; i++)
    if (msgs[i].node >= e->H || msgs[i].kind > GX_M_DEAD) return GX_EINVAL;
  int64_t now = now_of(e);
  for (uint32_t i = 0; i < n; i++) fd_handle(e, host, &msgs[i], now);
  return GX_OK;
}
int gx_fd_get_broadcasts(gx_engine *e, uint32_t host, uint32_t limit, gx_fd_msg *out, uint32_t *n_out) {
  if (!fd_host_ok(e, host) || !n_out || limit > 64 || (!out && limit)) return GX_EINVAL;
  *n_out = fd_get_broadcasts(e, host, limit, out);
  return GX_OK;
}
int gx_fd_probe(gx_engine *e, uint32_t host, uint32_t *target, int *acked) {
  if (!fd_host_ok(e, host)) return GX_EINVAL;
  int ack = 0;
  uint32_t t = fd_probe_host(e, host, &ack);
  if (target) *target = t;
  if (acked) *acked = ack;
  return GX_OK;
}
int gx_fd_timers(gx_engine *e, uint32_t host) {
  if (!fd_host_ok(e, host)) return GX_EINVAL;
  fd_timers_host(e, host, now_of(e));
  return GX_OK;
}
int gx_fd_converged(gx_engine *e, int *converged, uint64_t *n_disagree) {
  if (!e || !e->p.fd_enable) return GX_EINVAL;
  uint64_t bad = 0;
  for (uint32_t m = 0; m < e->H; m++) {
    int want = departed(e, m) ? GX_M_DEAD : GX_M_ALIVE;
    for (uint32_t v = e->lo; v < e->hi; v++) /* this engine's hosts */
      if (!departed(e, v) && MEM(e, v, m)->state != want) {
        bad++;
        break;
      }
  }
  if (converged) *converged = bad == 0;
  if (n_disagree) *n_disagree = bad;
  return GX_OK;
}
int gx_fd_merge_state(gx_engine *e, uint32_t host, const uint64_t *remote) {
  if (!fd_host_ok(e, host) || !remote) return GX_EINVAL;
  fd_merge_state(e, host, remote);
  return GX_OK;
}

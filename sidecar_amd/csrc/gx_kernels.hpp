// gx_kernels.hpp — round-phase kernels of the sidecar-gx engine (gfx950). Included by
// gx_engine.hip (single translation unit). DESIGN.md §3 (round model) and §6 (kernels).
#pragma once
#include "gx_device.hpp"

// =================================================================== block-level helpers ==
// Ordered block-wide exclusive scan of packed counts (u64 with independent 16-bit fields: every
// field's block total must stay < 65536). Returns this thread's exclusive prefix, `total` = sum.
GXD unsigned long long block_excl_scan64(unsigned long long x, unsigned long long *s_wave,
                                         unsigned long long &total) {
  uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  unsigned long long incl = x;
  for (int o = 1; o < 64; o <<= 1) {
    unsigned long long y = __shfl_up(incl, o, 64);
    if ((int)lane >= o) incl += y;
  }
  if (lane == 63) s_wave[w] = incl;
  __syncthreads();
  unsigned long long off = 0, tot = 0;
  for (uint32_t i = 0; i < nw; i++) {
    unsigned long long c = s_wave[i];
    if (i < w) off += c;
    tot += c;
  }
  __syncthreads();
  total = tot;
  return off + incl - x;
}
GXD uint32_t fld(unsigned long long x, int i) { return (uint32_t)((x >> (16 * i)) & 0xffffu); }

// Diagnostics (Dev::kprof, env GX_KPROF): after k_send's per-wave marks, GX_KPROF_MERGE_N counters
// of the gossip merge's routing (k_merge_seg), accumulated over launches: [0] receivers with live
// records, [1] routed to 16-lane segments, [2] to 32-lane segments, [3] to a whole wave, [4] merged
// by a whole wave after their segment did not fit, [5] live records registered
#define GX_KPROF_MERGE_N 64
GXD unsigned long long *kprof_merge(const Dev &d) {
  return d.kprof ? d.kprof + (size_t)((d.Hl + 63) / 64) * 4 * 8 : nullptr;
}
// Diagnostics: after the merge counters, two marks per push-pull block of the last k_ae launch:
// [2i] start | CU << 48, [2i + 1] end (wall clock, 100 MHz)
GXD unsigned long long *kprof_ae(const Dev &d) { return d.kprof ? kprof_merge(d) + GX_KPROF_MERGE_N : nullptr; }
// ... then two marks per view scanned by the last k_scan launch, by worklist position: [2w] start |
// CU << 48, [2w + 1] end
GXD unsigned long long *kprof_scan(const Dev &d) { return d.kprof ? kprof_ae(d) + d.H : nullptr; }

// OR of p over a 256-thread block (4 waves), one barrier: the waves' votes alternate between the
// two halves of s_any[8] (par flips per call), so a call's votes cannot be overwritten before every
// wave has read them. HIP's __syncthreads_or reads the work-group size with a vector load each
// call, and the wait on that load also waits for every tile load in flight (the streaming kernels
// call it once per tile).
GXD bool block_any256(bool p, uint32_t *s_any, uint32_t &par) {
  const uint32_t b = __ballot(p) != 0;
  if ((threadIdx.x & 63) == 0) s_any[par * 4 + (threadIdx.x >> 6)] = b;
  __syncthreads();
  const uint32_t *q = s_any + par * 4;
  const bool r = (q[0] | q[1] | q[2] | q[3]) != 0;
  par ^= 1u;
  return r;
}

// Block reduction of a counter -> one atomic on this block's shard.
GXD void block_ctr(const Dev &d, int idx, unsigned long long x, unsigned long long *s_red) {
  x = wave_sum(x);
  uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  if (lane == 0) s_red[w] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (uint32_t i = 0; i < nw; i++) t += s_red[i];
    ctr_atomic(d, idx, t);
  }
  __syncthreads();
}
GXD unsigned long long block_min(unsigned long long x, unsigned long long *s_red) {
  x = wave_min(x);
  uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  if (lane == 0) s_red[w] = x;
  __syncthreads();
  unsigned long long m = ~0ull;
  for (uint32_t i = 0; i < nw; i++) m = s_red[i] < m ? s_red[i] : m;
  __syncthreads();
  return m;
}

GXD unsigned long long block_sum(unsigned long long x, unsigned long long *s_red) {
  x = wave_sum(x);
  uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  if (lane == 0) s_red[w] = x;
  __syncthreads();
  unsigned long long m = 0;
  for (uint32_t i = 0; i < nw; i++) m += s_red[i];
  __syncthreads();
  return m;
}

// =================================================================================== init ==
__global__ void k_init_rec(Dev d, uint64_t *rec_word) {
  uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= d.R) return;
  const gx_params &p = d.p;
  int64_t ts = p.t0_ns - (int64_t)(rng4(p.seed, ST_INIT_TS, r, 0, 0) % 1000000000ull);
  if (p.aged_ppm && (rng4(p.seed, ST_INIT_AGE, r, 0, 0) % 1000000ull) < p.aged_ppm && p.aged_max_ns > 0)
    ts = p.t0_ns - (int64_t)(rng4(p.seed, ST_INIT_AGE, r, 1, 0) % (uint64_t)p.aged_max_ns);
  rec_word[r] = pack(ts, GX_ALIVE);
}

__global__ void k_init_views(Dev d, const uint64_t *rec_word) {
  size_t total = (size_t)d.Hl * d.R;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t v = d.lo + (uint32_t)(i / d.R), r = (uint32_t)(i % d.R);
    uint64_t w = GX_SLOT_ABSENT;
    if (d.p.init_mode == GX_INIT_WARM || (d.p.init_mode == GX_INIT_OWN && r / d.S == v)) w = rec_word[r];
    d.view[i] = w;
  }
}

// Initial catalogs count as inserted in key order: LastUpdated = LastChanged = the owner's last
// record, state.LastChanged = the view's last record (no events).
__global__ void k_init_times(Dev d, const uint64_t *rec_word) {
  size_t total = (size_t)d.Hl * d.H;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t vi = (uint32_t)(i / d.H), o = (uint32_t)(i % d.H), v = d.lo + vi;
    gx_server_times t = {0, 0};
    if (d.p.init_mode == GX_INIT_WARM || (d.p.init_mode == GX_INIT_OWN && o == v)) {
      int64_t ts = ts_of(rec_word[(size_t)o * d.S + d.S - 1]);
      t.last_updated_ns = ts;
      t.last_changed_ns = ts;
    }
    d.srvt[i] = t;
    if (o == 0) {
      int64_t lc = 0;
      if (d.p.init_mode == GX_INIT_WARM) lc = ts_of(rec_word[d.R - 1]);
      else if (d.p.init_mode == GX_INIT_OWN) lc = ts_of(rec_word[(size_t)v * d.S + d.S - 1]);
      d.vlc[vi] = lc;
    }
  }
}

// One tile's server times in key order: s_lu[i] / s_lc[i] = 1 + the last key of owner o0 + i
// with an accepted / a status-changing record this tile (0 = none); the slot already holds the
// stored word.
GXD void tile_owner_times(const Dev &d, uint32_t x, const uint64_t *row, uint32_t o0, uint32_t n,
                          const uint32_t *s_lu, const uint32_t *s_lc) {
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    uint32_t ku = s_lu[i], kc = s_lc[i];
    if (!ku && !kc) continue;
    gx_server_times *t = srv_times(d, x, o0 + i);
    if (ku) t->last_updated_ns = ts_of(row[ku - 1]);
    if (kc) t->last_changed_ns = ts_of(row[kc - 1]);
  }
}
#define TILE_OWNERS 1026  // owners a 1024-slot tile can touch (S = 1, plus both ends)

__global__ void k_init_hosts(Dev d) {
  uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= d.Hl) return;
  uint32_t o = d.lo + idx;
  const gx_params &p = d.p;
  gx_host_state h = {};
  h.bs_next = (int64_t)(rng4(p.seed, ST_PHASE_BS, o, 0, 0) % p.alive_interval_rounds);
  h.bt_next = (int64_t)(rng4(p.seed, ST_PHASE_BT, o, 0, 0) % p.tombstone_interval_rounds);
  h.last_bcast_ns = p.init_mode == GX_INIT_WARM ? p.t0_ns : 0;
  h.running = d.S == 64 ? ~0ull : ((1ull << d.S) - 1);
  d.hs[idx] = h;
  for (uint32_t s = 0; s < d.S; s++) d.own_status[(size_t)idx * d.S + s] = GX_ALIVE;
  for (uint32_t w = 0; w < d.AW; w++)  // list slots past list_slots never free
    d.arena_bits[(size_t)idx * d.AW + w] = d.A >= 32 * (w + 1) ? 0u : ~0u << (d.A - 32 * w);
}

// Exact per-view expiry bound (one block per view): used at create and after raw imports.
__global__ __launch_bounds__(256) void k_minexp_recompute(Dev d, uint32_t lo_idx) {
  __shared__ unsigned long long s_red[4];
  uint32_t v = lo_idx + blockIdx.x;  // local index
  const uint64_t *row = &d.view[(size_t)v * d.R];
  unsigned long long m = ~0ull;
  for (uint32_t r = threadIdx.x; r < d.R; r += blockDim.x) {
    unsigned long long x = exp_time(d.p, row[r]);
    m = x < m ? x : m;
  }
  m = block_min(m, s_red);
  if (threadIdx.x == 0) d.minexp[v] = m;
}

// wake_host on a register copy of the host's counters: the counters and the sleep ring's head
// job are the only dependent loads when nothing is due (64-thread blocks: 4x the CUs of 256)
__global__ __launch_bounds__(64) void k_wake(Dev d) {
  Acc a;
  uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < d.Hl && !departed(d, d.lo + idx)) {  // a crashed host stays frozen
    gx_host_state *h = &d.hs[idx];
    {  // the ServicesState lock for this round: the loopers' state (unchanged since the last sends)
      const uint32_t lw = h->lock, nl = lock_snap(lw, h->flags, d.round, d.p.lock_readers != 0);
      if (nl != lw) h->lock = nl;
    }
    const uint4 c = *reinterpret_cast<const uint4 *>(h);  // fifo_head, fifo_tail, sleep_head, sleep_tail
    if (c.z != c.w) {
      gx_host_state hs;
      hs.fifo_head = c.x;
      hs.fifo_tail = c.y;
      hs.sleep_head = c.z;
      hs.sleep_tail = c.w;
      hs.arena_used = h->arena_used;
      hs.fifo_stored = h->fifo_stored;
      const uint32_t au0 = hs.arena_used;
      while (hs.sleep_head != hs.sleep_tail) {  // re-armed passes: SEND / EXPIRE, never a nil
        const gx_sleeper &z = d.sleep[(size_t)idx * d.SQ + (hs.sleep_head & (d.SQ - 1u))];
        if ((int64_t)z.wake > d.round) break;
        const gx_job j = z.job;
        hs.sleep_head++;
        push_job_r(d, a, d.lo + idx, hs, j, true);
      }
      if (hs.sleep_head != c.z) {
        h->fifo_tail = hs.fifo_tail;
        h->fifo_stored = hs.fifo_stored;
        h->sleep_head = hs.sleep_head;
        if (hs.arena_used != au0) h->arena_used = hs.arena_used;
      }
    }
  }
  acc_flush(d, a);
}

// ================================================================= phase 0+1: owner ticks ==
// A team of T >= S lanes per host (lane s = service s): wake re-armed passes, discovery churn,
// the BroadcastServices tick (services_state.go:525-574) with IsNewService (:509-521) and
// TrackNewServices (:446-453), and the BroadcastTombstones tick. The looper state is the team's
// register copy of the host's bookkeeping; the lead lane stores it and the FIFO pushes. The S
// IsNewService reads and the S AddServiceEntry merges of the tick are independent (distinct own
// keys), so they run on their lanes; everything the reference orders (list order, LastUpdated /
// LastChanged, the ChangeEvents) follows from ballots in list order. Every included record is
// restamped `now`, so the server's times all take that value.
// A ticking view whose exact expiry bound is in the future cannot change in
// TombstoneOthersServices (:645-662); the others go to the expiry scan's worklist. Also clears the
// next round's inbox counts (round-parity buffers, Dev::in_cnt_nx).
// The tick of host idx by its team (T lanes inside one wave); sj = the team's T LDS job slots (the
// head of the sleep ring). Lane tl holds services tl + T*i, i < SPL (SPL = 1 when T >= S); a
// team-wide service mask is the OR of each lane's ballot shifted by T*i. Returns, on the lead
// lane, whether the host went on the expiry-scan worklist (its BroadcastTombstones tick then
// finishes after the scan).
// fwd (k_send's planned sends): the tick also loads the FIFO head jobs into fwd->pj (with the
// sleep-ring head, in the same round trip) and hands its register copy of the bookkeeping to the
// sends, which then neither reload it nor wait for the jobs.
// FIFO head jobs a send team keeps in LDS: T (GossipMessages <= 1: a round's calls fit), or
// GX_JPF * T under GossipMessages > 1 (fewer refills: each one waits on a global load)
#define GX_JPF 3
template <int T>
GXD uint32_t pj_window(const Dev &d) { return d.NG > 1 ? (uint32_t)(GX_JPF * T) : (uint32_t)T; }
struct TickFwd {
  gx_job *pj;         // the team's T * GX_JPF LDS job slots (stored FIFO head jobs)
  uint32_t *peers;    // the team's peer slots (count in [16]), sampled while the tick's loads fly
  gx_host_state hs;   // the bookkeeping after the tick
  uint32_t pf0, npf;  // FIFO position of pj[0], jobs loaded
  uint32_t tick;      // d.tick[idx] as the tick set it
};
// SW: the team's LDS sleeper slots (the head of its sleep ring, refilled SW at a time).
template <int T, int SPL = 1, bool FWD = false, int SW = T>
GXD bool owner_tick(const Dev &d, Acc &a, uint32_t idx, gx_sleeper *sj, TickFwd &fwd) {
  const uint32_t lane = threadIdx.x & 63, tl = lane & (T - 1), tw = lane / T;
  const bool lead = tl == 0;
  const uint64_t tmask = T == 64 ? ~0ull : ((1ull << T) - 1ull);
  const bool act = idx < d.Hl && !departed(d, d.lo + idx);
  bool queued = false;
  gx_host_state hs;
  auto team_mask = [&](const bool *p) -> uint64_t {  // bit s = service s's predicate
    uint64_t m = 0;
#pragma unroll
    for (int i = 0; i < SPL; i++) m |= ((__ballot(p[i]) >> (tw * T)) & tmask) << (T * i);
    return m;
  };
  // everything the tick may read is loaded up front: the bookkeeping, the own records' view slots
  // (one 128-B row segment), their local status and the view's expiry bound
  uint64_t cur0[SPL];
  uint8_t ost0[SPL];
#pragma unroll
  for (int i = 0; i < SPL; i++) {
    cur0[i] = GX_SLOT_ABSENT;
    ost0[i] = GX_ALIVE;
  }
  unsigned long long mexp0 = 0;
  if (act) {
    hs = d.hs[idx];
    const uint32_t o = d.lo + idx;
#pragma unroll
    for (int i = 0; i < SPL; i++) {
      const uint32_t sv = tl + T * i;
      if (sv < d.S) {
        cur0[i] = vrow(d, o)[o * d.S + sv];
        ost0[i] = d.own_status[(size_t)idx * d.S + sv];
      }
    }
    if (tl == 0) mexp0 = d.minexp[idx];
    {  // the sleep ring's head: T slots, or SW under GossipMessages > 1 (a round re-arms up to
       // fanout * GossipMessages passes, and they wake together)
      const uint32_t ns = hs.sleep_tail - hs.sleep_head, win = d.NG > 1 ? (uint32_t)SW : (uint32_t)T;
      for (uint32_t x = tl; x < ns && x < win; x += T) sj[x] = d.sleep[(size_t)idx * d.SQ + ((hs.sleep_head + x) & (d.SQ - 1u))];
    }
    if (FWD) {  // the tick pushes at the FIFO tail only: the stored jobs at the head stay where they are
      const uint32_t q = hs.fifo_stored - hs.fifo_head;
      const uint32_t win = pj_window<T>(d), nl = q < win ? q : win;
      for (uint32_t x = tl; x < nl; x += T) fwd.pj[x] = d.fifo[(size_t)idx * d.Q + ((hs.fifo_head + x) % d.Q)];
      fwd.pf0 = hs.fifo_head;
      fwd.npf = nl;
    }
  }
  if (FWD && tl == 0 && idx < d.Hl) {  // the sends' peers: ALU while the loads above are in flight
    const uint64_t h3 = mix64(mix64(mix64(d.p.seed ^ ((uint64_t)ST_PEER * 0xD1B54A32D192ED03ull)) ^ (uint64_t)d.round) ^
                              (uint64_t)(d.lo + idx));
    uint32_t base = 0, m = d.H;
    const uint32_t u = d.lo + idx;
    if (d.partitioned) {
      const uint32_t half = d.H / 2;
      base = u < half ? 0 : half;
      m = u < half ? half : d.H - half;
    }
    uint32_t cnt = 0;
    if (m >= 2) {
      const uint32_t want = d.K < m - 1 ? d.K : m - 1;
      for (uint32_t at = 0; cnt < want && at < 64u * d.K; at++) {  // = sample_peers
        const uint32_t ix = unif(mix64(h3 ^ at), m - 1), self = u - base;
        const uint32_t pp = base + (ix >= self ? ix + 1 : ix);
        bool dup = false;
        for (uint32_t i = 0; i < cnt; i++) dup |= fwd.peers[i] == pp;
        if (!dup) fwd.peers[cnt++] = pp;
      }
    }
    fwd.peers[16] = cnt;
  }
  if (FWD) fwd.tick = 0;
  wave_sync();  // the team's sleep-ring slots
  if (idx < d.Hl) {
    const uint32_t o = d.lo + idx;
    if (lead) d.in_cnt_nx[idx] = 0;
    if (!act) {  // a crashed host runs no loopers
      if (lead) d.tick[idx] = 0;
    } else {
      // TimedLooper re-arm (services_state.go:585-601): due passes re-enter the FIFO in order
      const uint32_t win = d.NG > 1 ? (uint32_t)SW : (uint32_t)T;
      for (uint32_t w = 0; hs.sleep_head != hs.sleep_tail; w++) {
        if (w == win) {  // past the loaded slots: the next window, all its loads in flight together
          const uint32_t ns = hs.sleep_tail - hs.sleep_head;
          wave_sync();
          for (uint32_t x = tl; x < ns && x < win; x += T)
            sj[x] = d.sleep[(size_t)idx * d.SQ + ((hs.sleep_head + x) & (d.SQ - 1u))];
          wave_sync();
          w = 0;
        }
        const gx_sleeper z = sj[w];
        if ((int64_t)z.wake > d.round) break;
        hs.sleep_head++;
        push_job_r(d, a, o, hs, z.job, lead);
      }
      uint8_t ost[SPL];
#pragma unroll
      for (int i = 0; i < SPL; i++) ost[i] = ost0[i];
      if (d.p.churn_ppm) {  // discovery churn: one service starts or stops
        const uint64_t x = rng4(d.p.seed, ST_CHURN, (uint64_t)d.round, o, 0);
        if ((uint32_t)(x & 0xffffffffu) % 1000000u < d.p.churn_ppm) {
          const uint32_t cs = (uint32_t)((x >> 32) % d.S);
          hs.running ^= 1ull << cs;
#pragma unroll
          for (int i = 0; i < SPL; i++)
            if (tl + T * i == cs && ((hs.running >> cs) & 1ull)) {
              ost[i] = GX_ALIVE;
              d.own_status[(size_t)idx * d.S + cs] = GX_ALIVE;
            }
          if (lead) a.c[C_CHURN]++;
        }
      }
      // with the lock modelled, a looper whose tick finds the other one blocked on its nil (holding
      // the ServicesState lock) waits: it ticks at the first owner phase after that nil was taken
      const bool lm = d.p.lock_model != 0;
      if (!(hs.flags & 1u) && !(lm && (hs.flags & 2u)) && hs.bs_next <= d.round) {
        // fn(): the running services in key order, restamped now; lane tl holds services tl + T*i
        const bool refresh = (d.now - d.p.alive_broadcast_interval_ns) > hs.last_bcast_ns;  // (:547)
        bool run[SPL], isnew[SPL], inc[SPL];
        uint64_t sw[SPL], cur[SPL];
#pragma unroll
        for (int i = 0; i < SPL; i++) {
          const uint32_t sv = tl + T * i;
          run[i] = sv < d.S && ((hs.running >> sv) & 1ull);
          sw[i] = pack(d.now, ost[i]);
          cur[i] = run[i] ? cur0[i] : GX_SLOT_ABSENT;  // no other writer of own slots before this
          isnew[i] = run[i] && (st_of(cur[i]) == GX_ABSENT ||
                                (st_of(sw[i]) != GX_TOMBSTONE && st_of(sw[i]) != st_of(cur[i])));
          inc[i] = isnew[i] || (run[i] && refresh);
        }
        const uint64_t newm = team_mask(isnew);
        const uint64_t incm = team_mask(inc);
        if (incm) {
          hs.last_bcast_ns = d.now;
          // SendServices(list, ALIVE_COUNT if anything is new, else 1) (:555-558); a deferred job
          // takes no list, a list that does not fit queues the job LOST
          const uint32_t npass = newm ? d.p.alive_count : 1;
          const uint32_t mlen = (uint32_t)__popcll(incm) < d.L ? (uint32_t)__popcll(incm) : d.L;
          const bool stores = fifo_room(d, hs.fifo_head, hs.fifo_tail, hs.fifo_stored) != 0;
          const int lslot = stores ? list_alloc<T>(d, idx, hs.arena_used, lead) : -1;
          if (lead) a.c[C_SENDJOBS]++;
          if (!stores) {
            push_job_r(d, a, o, hs, make_job(0, GX_LIST_NONE, meta_of(GX_JOB_SEND, 0, npass)), lead);
          } else if (lslot < 0) {
            if (lead) a.c[C_LDROP]++;
            push_job_r(d, a, o, hs, make_job(0, 0, meta_of(GX_JOB_LOST, 0, 1)), lead);
          } else {
            const uint32_t li_ = (uint32_t)lslot;
#pragma unroll
            for (int i = 0; i < SPL; i++) {
              const uint32_t sv = tl + T * i;
              const uint32_t rank = (uint32_t)__popcll(incm & ((1ull << sv) - 1ull));
              if (inc[i] && rank < d.L) {
                grec g;
                g.w = sw[i];
                g.r = o * d.S + sv;
                g.pad = 0;
                list_ptr(d, o, li_)[rank] = g;
              }
            }
            if (lead) d.arena_len[(size_t)idx * d.A + li_] = mlen;
            push_job_r(d, a, o, hs, make_job(0, li_ | (mlen << 16), meta_of(GX_JOB_SEND, 0, npass)), lead);
          }
          hs.bs_next = d.round + d.p.alive_interval_rounds;
          // TrackNewServices: AddServiceEntry of every included record into the own view
          bool acc[SPL], chg[SPL];
          uint64_t nw[SPL];
#pragma unroll
          for (int i = 0; i < SPL; i++) {
            bool stale = false;
            acc[i] = chg[i] = false;
            nw[i] = cur[i];
            if (inc[i]) {
              a.c[C_LOCAL_MERGES]++;
              nw[i] = merge_word(d, cur[i], sw[i], acc[i], stale);
              if (stale) a.c[C_STALE]++;
              if (acc[i]) {
                a.c[C_LOCAL_ACC]++;
                if (nw[i] != cur[i]) {
                  vrow(d, o)[o * d.S + tl + T * i] = nw[i];
                  a.changed = true;
                  atomicMin(&d.minexp[idx], exp_time(d.p, nw[i]));
                }
                chg[i] = st_of(cur[i]) == GX_ABSENT || st_of(cur[i]) != st_of(nw[i]);
              }
            }
            if (chg[i]) a.c[C_CHG]++;
          }
          const uint64_t accm = team_mask(acc), chgm = team_mask(chg);
          if (lead && accm) {
            gx_server_times *t = srv_times(d, o, o);
            t->last_updated_ns = d.now;  // server.LastUpdated (:323)
            if (chgm) {
              t->last_changed_ns = d.now;  // ServiceChanged (:195-215)
              d.vlc[idx] = d.now;
            }
          }
          const int32_t k = d.ev_slot[idx];
          if (k >= 0 && chgm) {  // ChangeEvents in list order
            const uint32_t ev0 = d.ev_cnt[k];
#pragma unroll
            for (int i = 0; i < SPL; i++) {
              const uint32_t sv = tl + T * i;
              if (chg[i])
                ev_put(d, k, ev0 + (uint32_t)__popcll(chgm & ((1ull << sv) - 1ull)), o * d.S + sv, nw[i],
                       st_of(cur[i]) == GX_ABSENT ? GX_UNKNOWN : st_of(cur[i]));
            }
            if (lead) d.ev_cnt[k] = ev0 + (uint32_t)__popcll(chgm);
          }
        } else {  // Broadcasts <- nil (:569): the looper blocks until the nil is consumed
          push_job_r(d, a, o, hs, make_job(0, 0, meta_of(GX_JOB_NIL_BS, 0, 1)), lead);
          hs.flags |= 1u;
        }
      }
      const bool tick = !(hs.flags & 2u) && !(lm && (hs.flags & 1u)) && hs.bt_next <= d.round;
      if (lead) {
        d.tick[idx] = tick ? 1 : 0;
        if (tick) {
          // (the tick's own merges only lower the bound to values >= now: same decision)
          if (mexp0 >= (unsigned long long)d.now) {  // nothing can expire in this view
            d.scan_cnt[idx] = 0;
            a.c[C_SCANSLOTS] += d.R;
          } else {
            d.work[atomicAdd(d.wl_cnt, 1u)] = idx;
            d.tick[idx] = 2;  // the tick streams the view first (k_scan, or k_send's prologue)
            queued = true;
          }
        }
        d.hs[idx] = hs;
      }
      if (FWD) {
        fwd.hs = hs;
        fwd.tick = tick ? 1u : 0u;  // the sends reload what the tick's finish changes
      }
    }
  }
  return queued;
}

template <int T, int B = 256>
__global__ __launch_bounds__(B) void k_owner(Dev d) {
  __shared__ gx_sleeper s_sl[B];  // the head of each host's sleep ring, one sleeper per team lane
  Acc a;
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // the next round's lists start empty
    *d.ovf_cnt_nx = 0;
    *d.wl_cnt_nx = 0;
  }
  TickFwd none;
  owner_tick<T>(d, a, blockIdx.x * (B / T) + threadIdx.x / T, &s_sl[threadIdx.x & ~(uint32_t)(T - 1)], none);
  acc_flush(d, a);
}

// ============================================== phase 1: TombstoneOthersServices full scan ==
// One 256-thread block per scanned view. k_owner left only the ticking views whose expiry bound
// is in the past on the worklist (a view with bound >= now cannot change: no slot has
// ts + lifespan < now), so a round with nothing to expire launches a small grid that exits at
// once. A listed row is streamed with 16-B loads (4 slots per thread per 1024-slot tile), the
// lifespans applied, and the first list_cap tombstones compacted in key order (packed block scan).
typedef unsigned long long v2u64 __attribute__((ext_vector_type(2)));
struct ScanLds {
  unsigned long long wave[4];
  unsigned long long red[4];
  uint32_t any[8];  // block_any256
  uint32_t lu[TILE_OWNERS];
  uint32_t last;
};
#ifndef SCAN_PF
#define SCAN_PF 1  // 4 tiles in flight (139 VGPRs, 3 waves/SIMD) measured slower on cfg 3: 1.59 vs 1.29 ms per round
#endif
// A chunk's result of a row split over blocks (k_scan_split, joined per view by k_scan_join).
struct ScanChunk {
  uint32_t cnt;              // expirations in the chunk (its first list_cap are listed)
  uint32_t last;             // 1 + the chunk's last expired key, 0 = none
  unsigned long long mexp;   // the chunk's exact expiry bound
};
// [r0, r1): the slots this block streams (tile-aligned; the whole row by default). co: chunk mode,
// the view's bookkeeping (list count, expiry bound, state.LastChanged, scan count) goes to *co for
// k_scan_join instead of the view. WT: S | 128 known at compile time (the LDS server-time path is
// not compiled: fewer registers, k_scan_split).
template <bool VEC, bool EV, bool WT = false>
GXD void scan_view(const Dev &d, uint32_t oi, grec *list, uint32_t list_cap, uint32_t *cnt_out, ScanLds &sm,
                   uint32_t r0 = 0, uint32_t r1 = 0xffffffffu, ScanChunk *co = nullptr) {
  if (r1 > d.R) r1 = d.R;
  unsigned long long *s_wave = sm.wave, *s_red = sm.red;
  uint32_t *s_lu = sm.lu;
  uint32_t &s_last = sm.last;
  uint64_t *row = &d.view[(size_t)oi * d.R];
  const int32_t evk = d.ev_slot[oi];
  const uint32_t ev0 = evk >= 0 ? d.ev_cnt[evk] : 0;
  uint32_t last_key = 0;  // 1 + the last expired key (state.LastChanged)
  uint32_t n_exp = 0;
  unsigned long long c_exp = 0, c_gc = 0, c_wr = 0, mexp = ~0ull, c_dep = 0;
  uint32_t t = threadIdx.x;
  // VEC: the next tile's two 16-B words per thread are in flight while this tile is processed
  // (nontemporal: a scanned row is not re-read soon)
  // (SCAN_PF tiles in flight per block: one 2 MB row per block is latency-bound otherwise)
  ulonglong2 nx[SCAN_PF][2];
  auto ld_into = [&](uint32_t base, ulonglong2 *dst) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint32_t q0 = base + 512 * h + 2 * t;
      if (q0 < r1) {
        v2u64 x = __builtin_nontemporal_load(reinterpret_cast<const v2u64 *>(&row[q0]));
        dst[h] = make_ulonglong2(x.x, x.y);
      } else {
        dst[h] = make_ulonglong2(GX_SLOT_ABSENT, GX_SLOT_ABSENT);
      }
    }
  };
  if (VEC) {
#pragma unroll
    for (int q = 0; q < SCAN_PF; q++) ld_into(r0 + 1024u * q, nx[q]);
  }
  // S | 128: an owner's slots sit in S/2 adjacent lanes of one wave, so the server times of a
  // tile's owners (the last expired record of each, key order) come from a ballot, with no LDS
  const bool wave_times = WT || (VEC && d.S >= 2 && (128 % d.S) == 0);
  const bool ev_on = EV && evk >= 0;
  bool listing = true;     // block-uniform: list positions (or event positions) still needed
  uint32_t my_last = 0;    // 1 + this thread's last expired key (state.LastChanged)
  unsigned long long cnt_tail = 0;  // expirations counted per thread once the list is full
  uint32_t any_par = 0;
  auto tile = [&](uint32_t base, const ulonglong2 *cur) {
    uint64_t w[4], nw[4];
    bool ex[4];
    bool valid[4];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      uint32_t r0 = VEC ? base + 512 * h + 2 * t : base + 2 * blockDim.x * h + 2 * t;
      valid[2 * h] = r0 < d.R;
      valid[2 * h + 1] = r0 + 1 < d.R;
      if (VEC) {
        w[2 * h] = cur[h].x;
        w[2 * h + 1] = cur[h].y;
      } else {
        w[2 * h] = valid[2 * h] ? row[r0] : GX_SLOT_ABSENT;
        w[2 * h + 1] = valid[2 * h + 1] ? row[r0 + 1] : GX_SLOT_ABSENT;
      }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
      bool gc;
      nw[k] = expiry_word(d, w[k], ex[k], gc);
      c_exp += ex[k];
      c_gc += gc;
      unsigned long long x = exp_time(d.p, nw[k]);
      mexp = x < mexp ? x : mexp;
    }
    if (d.departures) {  // gx.h false_expiries: the expiries of departed owners' records are not
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t r = (VEC ? base + 512 * (k >> 1) + 2 * t : base + 2 * blockDim.x * (k >> 1) + 2 * t) + (k & 1);
        if (ex[k]) c_dep += departed(d, owner_of(d, r));
      }
    }
#pragma unroll
    for (int h = 0; h < 2; h++) {
      uint32_t r0 = VEC ? base + 512 * h + 2 * t : base + 2 * blockDim.x * h + 2 * t;
      bool ch0 = nw[2 * h] != w[2 * h], ch1 = nw[2 * h + 1] != w[2 * h + 1];
      c_wr += ch0 + ch1;
      if (VEC && (ch0 || ch1)) {
        *reinterpret_cast<ulonglong2 *>(&row[r0]) = make_ulonglong2(nw[2 * h], nw[2 * h + 1]);
      } else if (!VEC) {
        if (ch0) row[r0] = nw[2 * h];
        if (ch1) row[r0 + 1] = nw[2 * h + 1];
      }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t r = (VEC ? base + 512 * (k >> 1) + 2 * t : base + 2 * blockDim.x * (k >> 1) + 2 * t) + (k & 1);
      if (ex[k]) my_last = r + 1;  // keys rise with k within a thread and across tiles
    }
    if (wave_times) {
      const uint32_t lane = t & 63, lpo = d.S / 2, gb = lane & ~(lpo - 1);
      const uint64_t gm = (lpo == 64 ? ~0ull : ((1ull << lpo) - 1ull)) << gb;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const bool e0 = ex[2 * h], e1 = ex[2 * h + 1];
        const uint64_t gbits = __ballot(e0 || e1) & gm;
        if (gbits && lane == 63u - (uint32_t)__clzll(gbits)) {  // the owner's last lane with an expiry
          const uint32_t r = base + 512 * h + 2 * t + (e1 ? 1u : 0u);
          gx_server_times *st = srv_times(d, oi + d.lo, r / d.S);
          const int64_t ts = ts_of(e1 ? nw[2 * h + 1] : nw[2 * h]);
          st->last_updated_ns = ts;
          st->last_changed_ns = ts;
        }
      }
    }
    if (!listing) {  // the list is full and nothing needs positions: count only
      cnt_tail += ex[0] + ex[1] + ex[2] + ex[3];
      return;
    }
    // a tile without expirations (GC writes only) needs no compaction: one barrier
    if (!block_any256(ex[0] || ex[1] || ex[2] || ex[3], sm.any, any_par)) return;
    unsigned long long cnt = (unsigned long long)(ex[0] + ex[1]) | ((unsigned long long)(ex[2] + ex[3]) << 16);
    unsigned long long tot;
    unsigned long long pre = block_excl_scan64(cnt, s_wave, tot);
    uint32_t pos[4];
    pos[0] = n_exp + fld(pre, 0);
    pos[1] = pos[0] + ex[0];
    pos[2] = n_exp + fld(tot, 0) + fld(pre, 1);
    pos[3] = pos[2] + ex[2];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (ex[k] && pos[k] < list_cap) {
        uint32_t r0 = (VEC ? base + 512 * (k >> 1) + 2 * t : base + 2 * blockDim.x * (k >> 1) + 2 * t) + (k & 1);
        grec g;
        g.w = nw[k];
        g.r = r0;
        g.pad = 0;
        list[pos[k]] = g;
      }
    }
    uint32_t tn = (uint32_t)(fld(tot, 0) + fld(tot, 1));
    if (tn && wave_times) {  // server times done above; events in list order
      if (ev_on) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
          if (!ex[k]) continue;
          uint32_t r = base + 512 * (k >> 1) + 2 * t + (k & 1);
          ev_put(d, evk, ev0 + pos[k], r, nw[k], st_of(w[k]));
        }
      }
    } else if (tn) {  // ServiceChanged per expiry (:673-676): server times, state.LastChanged, events
      uint32_t o0 = base / d.S, oe = ((base + 4 * blockDim.x < d.R ? base + 4 * blockDim.x : d.R) - 1) / d.S;
      for (uint32_t i = t; i <= oe - o0; i += blockDim.x) s_lu[i] = 0;
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 4; k++) {
        if (!ex[k]) continue;
        uint32_t r = (VEC ? base + 512 * (k >> 1) + 2 * t : base + 2 * blockDim.x * (k >> 1) + 2 * t) + (k & 1);
        atomicMax(&s_lu[r / d.S - o0], r + 1);
        if (pos[k] == n_exp + tn - 1) s_last = r + 1;
        if (EV && evk >= 0) ev_put(d, evk, ev0 + pos[k], r, nw[k], st_of(w[k]));
      }
      __syncthreads();
      tile_owner_times(d, oi + d.lo, row, o0, oe - o0 + 1, s_lu, s_lu);
      last_key = s_last;
      __syncthreads();
    }
    n_exp += tn;
    listing = ev_on || !wave_times || n_exp < list_cap;  // without wave_times the LDS path keeps the server times
  };
  for (uint32_t base = r0; base < r1; base += SCAN_PF * 1024u) {
#pragma unroll
    for (int q = 0; q < SCAN_PF; q++) {
      const uint32_t b = base + 1024u * q;
      if (b >= r1) break;
      ulonglong2 cur[2] = {nx[q][0], nx[q][1]};
      if (VEC && b + SCAN_PF * 1024u < r1) ld_into(b + SCAN_PF * 1024u, nx[q]);
      tile(b, cur);
    }
  }
  {
    unsigned long long tail;
    (void)block_excl_scan64(cnt_tail, s_wave, tail);
    n_exp += (uint32_t)tail;
    const unsigned long long lk = ~block_min(~(unsigned long long)my_last, s_red);
    last_key = (uint32_t)lk;
  }
  mexp = block_min(mexp, s_red);
  if (threadIdx.x == 0 && co) {  // chunk mode: k_scan_join finishes the view
    co->cnt = n_exp;
    co->last = last_key;
    co->mexp = mexp;
  } else if (threadIdx.x == 0) {
    atomicAdd(&d.work_cnt[GX_WC_SCANS], 1u);
    *cnt_out = n_exp;
    d.minexp[oi] = mexp;  // exact bound after the scan
    if (last_key) d.vlc[oi] = ts_of(row[last_key - 1]);
    if (evk >= 0) d.ev_cnt[evk] = ev0 + n_exp;
  }
  block_ctr(d, C_CHG, c_exp, s_red);
  bool changed = c_wr != 0;
  if (__ballot(changed) != 0 && (threadIdx.x & 63) == 0) mark_change(d);
  c_wr = wave_sum(c_wr);
  if ((threadIdx.x & 63) == 0) kbytes(d, GX_K_SCAN, c_wr * 8, 0);
  if (threadIdx.x == 0)
    kbytes(d, GX_K_SCAN, (unsigned long long)(r1 - r0) * 8 + 16ull * (n_exp < list_cap ? n_exp : list_cap), r1 - r0);
  block_ctr(d, C_EXPIRED, c_exp, s_red);
  block_ctr(d, C_FEXP, c_exp - c_dep, s_red);
  block_ctr(d, C_GC, c_gc, s_red);
  block_ctr(d, C_SCANSLOTS, threadIdx.x == 0 ? r1 - r0 : 0, s_red);
}

// only_host >= 0: that one view (the API's TombstoneOthersServices), list at list_base, count in
// cnt_out[0]. Otherwise the round's worklist, block-strided; view oi's list at oi * list_stride.
#ifdef GX_SCAN_WPE
#define GX_SCAN_ATTR __attribute__((amdgpu_waves_per_eu(GX_SCAN_WPE)))
#else
#define GX_SCAN_ATTR
#endif
template <bool VEC, bool EV>
__global__ __launch_bounds__(256) GX_SCAN_ATTR void k_scan(Dev d, grec *list_base, uint32_t list_stride, uint32_t list_cap,
                                               uint32_t *cnt_out, int only_host) {
  __shared__ ScanLds sm;
  if (only_host >= 0) {
    scan_view<VEC, EV>(d, li(d, (uint32_t)only_host), list_base, list_cap, cnt_out, sm);
    return;
  }
  const uint32_t n = *d.wl_cnt;
  unsigned long long *kp = kprof_scan(d);
  for (uint32_t w = blockIdx.x; w < n; w += gridDim.x) {
    const uint32_t oi = d.work[w];
    if (kp && threadIdx.x == 0 && w < d.H) kp[2 * w] = wall_clock64() | ((unsigned long long)__smid() << 48);
    scan_view<VEC, EV>(d, oi, &list_base[(size_t)oi * list_stride], list_cap, &cnt_out[oi], sm);
    if (kp && threadIdx.x == 0 && w < d.H) kp[2 * w + 1] = wall_clock64();
    __syncthreads();
  }
}


// The worklist's rows split into nch tile-aligned chunks of `clen` slots, one block per (view,
// chunk) (round 6): a row streamed by one block keeps too few bytes in flight, and a worklist of
// fewer rows than resident blocks leaves CUs idle (cfg 3: 1,600 rows of 2 MB). Each chunk lists its
// first list_cap expirations in key order at tmp[(oi * nch + c) * list_cap], writes its result to
// chunk[oi * nch + c], and k_scan_join concatenates them: the same list, count, expiry bound and
// state.LastChanged as scan_view over the whole row. Owners never straddle chunks (S | 128, the
// wave_times path; no listeners).
// Chunks per row this round (both kernels derive the same from the worklist count n): enough
// items for about SCAN_ITEMS blocks, at most nch (the allocation's stride); a long worklist keeps
// whole rows (each chunk restarts the tile pipeline: 1,600 rows of cfg 3 in 8 chunks measured 8%
// slower than whole rows, 400 rows 1.9x faster). clen: the chunk length, tile-aligned.
#ifndef SCAN_ITEMS
#define SCAN_ITEMS 2048u  // wave-level chunks, cfg 3 over 30 rounds: 1024 / 2048 / 4096 items 32.9 / 29.3 / 30.3 ms
#endif                    // lock off, 7.59 / 6.55 / 6.55 lock on (profiles/r06/ab/scan_wave_items_cfg3_*.jsonl)
GXD uint32_t scan_chunks(const Dev &d, uint32_t n, uint32_t nch, uint32_t &clen) {
  uint32_t c = n ? (SCAN_ITEMS + n - 1) / n : 1;
  c = c < nch ? c : nch;
  clen = (d.R / c + 1023u) / 1024u * 1024u;
  return (d.R + clen - 1) / clen;
}
// One chunk [r0, r1) of view oi by a block whose four waves each stream a contiguous quarter on
// their own (round 6): no block barrier per tile, SCAN_WPF 256-slot tiles in flight per wave, few
// registers (8 waves per SIMD). Each wave lists its first list_cap expirations in LDS (wave prefix
// from ballots); one barrier at the end concatenates the four lists in key order into `list` and
// writes the chunk's result, as scan_view's chunk mode does (S | 128: an owner's slots sit in S/2
// adjacent lanes of a 128-slot half-tile, so server times come from ballots). VEC, no listeners.
#ifndef SCAN_WPF
#define SCAN_WPF 2  // cfg 3 scan, 30 rounds: block scan 34.8 ms, WPF 2 / 3 / 4 29.3 / 29.5 / 34.5 (profiles/r06/ab/scan_wave_cfg3_lm0.jsonl)
#endif
GXD void scan_chunk_waves(const Dev &d, uint32_t oi, grec *list, uint32_t list_cap, uint32_t r0, uint32_t r1,
                          ScanChunk *co, grec *s_sub, uint32_t *s_wcnt, uint32_t *s_wlast,
                          unsigned long long *s_wmexp, unsigned long long *s_red) {
  if (r1 > d.R) r1 = d.R;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t q = ((r1 - r0) / 4 + 255u) / 256u * 256u;  // a wave's range, tile-aligned
  const uint32_t w0 = r0 + wv * q < r1 ? r0 + wv * q : r1, w1 = w0 + q < r1 ? w0 + q : r1;
  uint64_t *row = &d.view[(size_t)oi * d.R];
  grec *sub = &s_sub[(size_t)wv * list_cap];
  const uint32_t lpo = d.S / 2, gb = lane & ~(lpo - 1);
  const uint64_t gm = (lpo == 64 ? ~0ull : ((1ull << lpo) - 1ull)) << gb, lt = (1ull << lane) - 1ull;
  uint32_t n_exp = 0, my_last = 0;
  unsigned long long c_exp = 0, c_gc = 0, c_wr = 0, c_dep = 0, mexp = ~0ull;
  ulonglong2 nx[SCAN_WPF][2];
  auto ld = [&](uint32_t base, ulonglong2 *dst) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint32_t r = base + 128 * h + 2 * lane;
      if (r < w1) {
        v2u64 x = __builtin_nontemporal_load(reinterpret_cast<const v2u64 *>(&row[r]));
        dst[h] = make_ulonglong2(x.x, x.y);
      } else {
        dst[h] = make_ulonglong2(GX_SLOT_ABSENT, GX_SLOT_ABSENT);
      }
    }
  };
#pragma unroll
  for (int k = 0; k < SCAN_WPF; k++) ld(w0 + 256u * k, nx[k]);
  for (uint32_t base = w0; base < w1; base += SCAN_WPF * 256u) {
#pragma unroll
    for (int k = 0; k < SCAN_WPF; k++) {
      const uint32_t b = base + 256u * k;
      if (b >= w1) break;  // wave-uniform
      const ulonglong2 cur[2] = {nx[k][0], nx[k][1]};
      if (b + SCAN_WPF * 256u < w1) ld(b + SCAN_WPF * 256u, nx[k]);
      uint64_t wd[4] = {cur[0].x, cur[0].y, cur[1].x, cur[1].y}, nw[4];
      bool ex[4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        bool gc;
        nw[j] = expiry_word(d, wd[j], ex[j], gc);
        c_exp += ex[j];
        c_gc += gc;
        const unsigned long long x = exp_time(d.p, nw[j]);
        mexp = x < mexp ? x : mexp;
      }
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const uint32_t r = b + 128 * h + 2 * lane;
        const bool ch0 = nw[2 * h] != wd[2 * h], ch1 = nw[2 * h + 1] != wd[2 * h + 1];
        c_wr += ch0 + ch1;
        if (ch0 || ch1) *reinterpret_cast<ulonglong2 *>(&row[r]) = make_ulonglong2(nw[2 * h], nw[2 * h + 1]);
        if (d.departures) {  // gx.h false_expiries
          if (ex[2 * h]) c_dep += departed(d, owner_of(d, r));
          if (ex[2 * h + 1]) c_dep += departed(d, owner_of(d, r + 1));
        }
        if (ex[2 * h]) my_last = r + 1;
        if (ex[2 * h + 1]) my_last = r + 2;
        const uint64_t gbits = __ballot(ex[2 * h] || ex[2 * h + 1]) & gm;  // server times: owner's last expiry
        if (gbits && lane == 63u - (uint32_t)__clzll(gbits)) {
          const bool e1 = ex[2 * h + 1];
          gx_server_times *st = srv_times(d, oi + d.lo, (r + (e1 ? 1u : 0u)) / d.S);
          const int64_t ts = ts_of(e1 ? nw[2 * h + 1] : nw[2 * h]);
          st->last_updated_ns = ts;
          st->last_changed_ns = ts;
        }
      }
      const uint64_t b0 = __ballot(ex[0]), b1 = __ballot(ex[1]), b2 = __ballot(ex[2]), b3 = __ballot(ex[3]);
      const uint32_t tn = (uint32_t)(__popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3));
      if (tn && n_exp < list_cap) {  // key order: half 0 (lanes, 2 slots each), then half 1
        const uint32_t h1 = (uint32_t)(__popcll(b0) + __popcll(b1));
        uint32_t pos[4];
        pos[0] = n_exp + (uint32_t)(__popcll(b0 & lt) + __popcll(b1 & lt));
        pos[1] = pos[0] + ex[0];
        pos[2] = n_exp + h1 + (uint32_t)(__popcll(b2 & lt) + __popcll(b3 & lt));
        pos[3] = pos[2] + ex[2];
#pragma unroll
        for (int j = 0; j < 4; j++) {
          if (ex[j] && pos[j] < list_cap) {
            grec g;
            g.w = nw[j];
            g.r = b + 128 * (j >> 1) + 2 * lane + (j & 1);
            g.pad = 0;
            sub[pos[j]] = g;
          }
        }
      }
      n_exp += tn;
    }
  }
  // the wave's results, then the block's: the four lists in key order
  my_last = (uint32_t)~wave_min(~(unsigned long long)my_last);
  const unsigned long long wm = wave_min(mexp);
  if (lane == 0) {
    s_wcnt[wv] = n_exp;
    s_wlast[wv] = my_last;
    s_wmexp[wv] = wm;
  }
  __syncthreads();
  uint32_t tot = 0, last = 0, off[4];
  unsigned long long m = ~0ull;
#pragma unroll
  for (int w = 0; w < 4; w++) {
    off[w] = tot;
    tot += s_wcnt[w];
    if (s_wlast[w]) last = s_wlast[w];
    m = s_wmexp[w] < m ? s_wmexp[w] : m;
  }
  for (uint32_t i = threadIdx.x; i < 4 * list_cap; i += blockDim.x) {
    const uint32_t w = i / list_cap, j = i - w * list_cap;
    const uint32_t nw_ = s_wcnt[w] < list_cap ? s_wcnt[w] : list_cap;
    if (j < nw_ && off[w] + j < list_cap) list[off[w] + j] = s_sub[i];
  }
  if (threadIdx.x == 0) {
    co->cnt = tot;
    co->last = last;
    co->mexp = m;
  }
  block_ctr(d, C_CHG, c_exp, s_red);
  if (__ballot(c_wr != 0) != 0 && lane == 0) mark_change(d);
  c_wr = wave_sum(c_wr);
  if (lane == 0) kbytes(d, GX_K_SCAN, c_wr * 8, 0);
  if (threadIdx.x == 0)
    kbytes(d, GX_K_SCAN, (unsigned long long)(r1 - r0) * 8 + 16ull * (tot < list_cap ? tot : list_cap), r1 - r0);
  block_ctr(d, C_EXPIRED, c_exp, s_red);
  block_ctr(d, C_FEXP, c_exp - c_dep, s_red);
  block_ctr(d, C_GC, c_gc, s_red);
  block_ctr(d, C_SCANSLOTS, threadIdx.x == 0 ? r1 - r0 : 0, s_red);
}
#ifndef GX_SCAN_WAVE
#define GX_SCAN_WAVE 1
#endif
template <bool VEC>
__global__ __launch_bounds__(256) GX_SCAN_ATTR void k_scan_split(Dev d, grec *tmp, ScanChunk *chunk, uint32_t nch) {
  __shared__ ScanLds sm;
  extern __shared__ grec s_sub[];  // GX_SCAN_WAVE: [4][d.L] (dynamic)
  __shared__ uint32_t s_wcnt[4], s_wlast[4];
  __shared__ unsigned long long s_wmexp[4];
  uint32_t clen;
  const uint32_t nc = scan_chunks(d, *d.wl_cnt, nch, clen), n = *d.wl_cnt * nc;
  for (uint32_t w = blockIdx.x; w < n; w += gridDim.x) {
    const uint32_t oi = d.work[w / nc], c = w % nc;
    const size_t k = (size_t)oi * nch + c;
    if (GX_SCAN_WAVE && VEC)
      scan_chunk_waves(d, oi, &tmp[k * d.L], d.L, c * clen, (c + 1) * clen, &chunk[k], s_sub, s_wcnt, s_wlast, s_wmexp,
                       sm.red);
    else
      scan_view<VEC, false, VEC>(d, oi, &tmp[k * d.L], d.L, nullptr, sm, c * clen, (c + 1) * clen, &chunk[k]);
    __syncthreads();
  }
}
__global__ __launch_bounds__(256) void k_scan_join(Dev d, const grec *tmp, const ScanChunk *chunk, uint32_t nch_max) {
  __shared__ uint32_t s_pre[65];
  const uint32_t n = *d.wl_cnt, L = d.L;
  uint32_t clen;
  const uint32_t nch = scan_chunks(d, n, nch_max, clen);
  for (uint32_t w = blockIdx.x; w < n; w += gridDim.x) {
    const uint32_t oi = d.work[w];
    const ScanChunk *ch = &chunk[(size_t)oi * nch_max];
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t tot = 0, last = 0;
      unsigned long long mexp = ~0ull;
      for (uint32_t c = 0; c < nch; c++) {
        s_pre[c] = tot;
        tot += ch[c].cnt;
        mexp = ch[c].mexp < mexp ? ch[c].mexp : mexp;
        if (ch[c].last) last = ch[c].last;
      }
      s_pre[nch] = tot;
      d.scan_cnt[oi] = tot;
      d.minexp[oi] = mexp;  // exact bound after the scan
      if (last) d.vlc[oi] = ts_of(d.view[(size_t)oi * d.R + last - 1]);
      atomicAdd(&d.work_cnt[GX_WC_SCANS], 1u);
    }
    __syncthreads();
    grec *out = &d.scan_list[(size_t)oi * L];
    for (uint32_t c = 0; c < nch && s_pre[c] < L; c++) {
      const uint32_t nc = s_pre[c + 1] - s_pre[c], take = nc < L - s_pre[c] ? nc : L - s_pre[c];
      for (uint32_t i = threadIdx.x; i < take; i += blockDim.x) out[s_pre[c] + i] = tmp[((size_t)oi * nch_max + c) * L + i];
    }
  }
}

// The rest of a BroadcastTombstones tick on its own, for rounds where other phases push to the
// FIFO between the scan and the send (failure detector, storm); otherwise k_send runs it.
// Then the ExpireServer calls that waited for the host's lock (run_pending_expires), ending the
// owner phase.
__global__ __launch_bounds__(256) void k_bt_finish(Dev d) {
  Acc a;
  uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < d.Hl && d.tick[idx]) {
    uint32_t n = d.scan_cnt[idx];
    bt_finish(d, a, d.lo + idx, d.hs[idx].running, &d.scan_list[(size_t)idx * d.L], n < d.L ? n : d.L);
  }
  if (idx < d.Hl && d.pexp) {
    const uint32_t lw = d.hs[idx].lock;
    if ((lw & GX_LOCK_PENDING_EXPIRE) && !locked_in(d, lw) && !departed(d, d.lo + idx)) run_pending_expires(d, a, d.lo + idx);
  }
  acc_flush(d, a);
}

// ===================================================================== phase 2: departure storm ==
// One block per viewer. The other half's owners are walked in tiles of 1024/S owners whose S
// slots are contiguous; threads read the tile's words lane-contiguously (coalesced), fold each
// owner's presence mask and liveness in LDS, tombstone the live owners' present slots, and
// compact the EXPIRE jobs in owner order.
#define STORM_TILE 1024
// A locked viewer (gx.h lock_model): its ExpireServer calls for owners [lo, hi) wait for the lock
// (pexp bits; run_pending_expires at its first unlocked round). Block-wide, one word per thread.
GXD void storm_defer(const Dev &d, uint32_t vi, uint32_t lo, uint32_t hi) {
  uint32_t *w = &d.pexp[(size_t)vi * d.PW];
  for (uint32_t k = (lo >> 5) + threadIdx.x; hi > lo && k <= (hi - 1) >> 5; k += blockDim.x) {
    const uint32_t a = k * 32 > lo ? k * 32 : lo, b = k * 32 + 32 < hi ? k * 32 + 32 : hi;
    const uint32_t m = (b - a == 32 ? ~0u : ((1u << (b - a)) - 1u)) << (a & 31);
    w[k] |= m;
  }
  if (threadIdx.x == 0) {
    d.hs[vi].lock |= GX_LOCK_PENDING_EXPIRE;
    ctr_atomic(d, C_EXP_DEFER, hi - lo);
  }
}
template <bool EV>
__global__ __launch_bounds__(256) void k_storm(Dev d) {
  __shared__ unsigned long long s_mask[STORM_TILE];
  __shared__ uint32_t s_live[STORM_TILE];
  __shared__ uint32_t s_ebase[STORM_TILE];
  __shared__ unsigned long long s_wave[4];
  uint32_t vi = blockIdx.x, v = d.lo + vi;
  if (departed(d, v)) return;  // uniform per block
  uint32_t half = d.H / 2;
  uint32_t lo = v < half ? half : 0, hi = v < half ? d.H : half;
  gx_host_state *h = &d.hs[vi];
  if (d.p.lock_model && locked_in(d, h->lock)) {  // block-uniform
    storm_defer(d, vi, lo, hi);
    return;
  }
  const uint32_t tail0 = h->fifo_tail, st0 = h->fifo_stored, room = fifo_room(d, h->fifo_head, tail0, st0);
  uint32_t jobs = 0, n_ev = 0;
  unsigned long long c_wr = 0, c_chg = 0;
  uint64_t tomb = pack(d.now, GX_TOMBSTONE);
  const int32_t evk = d.ev_slot[vi];
  const uint32_t ev0 = evk >= 0 ? d.ev_cnt[evk] : 0;
  uint32_t OT = STORM_TILE / d.S;
  uint32_t t = threadIdx.x;
  for (uint32_t ob = lo; ob < hi; ob += OT) {
    uint32_t on = hi - ob < OT ? hi - ob : OT, ns = on * d.S;
    for (uint32_t i = t; i < on; i += blockDim.x) {
      s_mask[i] = 0;
      s_live[i] = 0;
    }
    __syncthreads();
    uint64_t *base = &d.view[(size_t)vi * d.R + (size_t)ob * d.S];
    uint64_t w[STORM_TILE / 256];
#pragma unroll
    for (int q = 0; q < STORM_TILE / 256; q++) {
      uint32_t k = t + 256 * q;
      w[q] = k < ns ? base[k] : GX_SLOT_ABSENT;
      if (st_of(w[q]) != GX_ABSENT) {
        uint32_t oi = k / d.S, s = k - oi * d.S;
        atomicOr(&s_mask[oi], 1ull << s);
        if (st_of(w[q]) != GX_TOMBSTONE) s_live[oi] = 1;
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < STORM_TILE / 256; q++) {
      uint32_t k = t + 256 * q;
      if (k < ns && st_of(w[q]) != GX_ABSENT && s_live[k / d.S] && w[q] != tomb) {
        base[k] = tomb;
        c_wr++;
      }
    }
    for (uint32_t i0 = 0; i0 < on; i0 += blockDim.x) {  // EXPIRE jobs in owner order
      uint32_t i = i0 + t;
      bool live = i < on && s_live[i];
      uint32_t ec = live ? (uint32_t)__popcll(s_mask[i]) : 0u;  // ServiceChanged per record
      unsigned long long tot;
      unsigned long long pre = block_excl_scan64((live ? 1ull : 0ull) | ((unsigned long long)ec << 16), s_wave, tot);
      uint32_t pos = (uint32_t)fld(pre, 0);
      if (live && jobs + pos < room)
        d.fifo[(size_t)vi * d.Q + ((tail0 + jobs + pos) % d.Q)] =
            make_job(s_mask[i], (uint32_t)d.round, GX_JOB_META(GX_JOB_EXPIRE, 0, d.p.tombstone_count, ob + i));
      if (live) {
        gx_server_times *st = srv_times(d, v, ob + i);
        st->last_updated_ns = d.now;
        st->last_changed_ns = d.now;
        s_ebase[i] = ev0 + n_ev + (uint32_t)fld(pre, 1);
      }
      c_chg += ec;
      jobs += (uint32_t)fld(tot, 0);
      n_ev += (uint32_t)fld(tot, 1);
    }
    __syncthreads();
    if (EV && evk >= 0) {  // events: owner order, then service order
#pragma unroll
      for (int q = 0; q < STORM_TILE / 256; q++) {
        uint32_t k = t + 256 * q;
        if (k >= ns || st_of(w[q]) == GX_ABSENT) continue;
        uint32_t oi = k / d.S, sv = k - oi * d.S;
        if (!s_live[oi]) continue;
        uint32_t pos = s_ebase[oi] + (uint32_t)__popcll(s_mask[oi] & ((1ull << sv) - 1));
        ev_put(d, evk, pos, ob * d.S + k, tomb, st_of(w[q]));
      }
      __syncthreads();
    }
  }
  bool changed = c_wr != 0;
  if (__ballot(changed) != 0 && (t & 63) == 0) {
    mark_change(d);
    atomicMin(&d.minexp[vi], exp_time(d.p, tomb));
  }
  c_wr = wave_sum(c_wr);
  c_chg = wave_sum(c_chg);
  if ((t & 63) == 0) {
    kbytes(d, GX_K_STORM, 8ull * c_wr, 0);
    ctr_atomic(d, C_CHG, c_chg);
  }
  if (t == 0) {
    const uint32_t ok = jobs < room ? jobs : room;  // stored; the rest deferred (gx.h gx_job)
    h->fifo_tail = tail0 + jobs;
    h->fifo_stored = st0 + ok;
    if (jobs) d.vlc[vi] = d.now;
    if (evk >= 0) d.ev_cnt[evk] = ev0 + n_ev;
    // + 16 B of server times (LastUpdated, LastChanged) per live owner
    kbytes(d, GX_K_STORM, 8ull * (hi - lo) * d.S + 16ull * ok + 16ull * jobs, (unsigned long long)(hi - lo) * d.S);
    ctr_atomic(d, C_EXPSRV, jobs);
    ctr_atomic(d, C_QDEFER, jobs - ok);
  }
}

// Storm for S | 64 (S >= 2): a wave's 128-word chunk holds 128/S whole owners, so the presence
// masks and liveness come from ballots (no LDS atomics); each owner's first lane emits its
// EXPIRE job. Rows stream with 16-B loads, the next 1024 words in flight while this tile is
// folded; one barrier per tile orders the jobs (per-chunk counts, double-buffered).
GXD uint64_t spread32(uint64_t x) {  // bit i -> bit 2i
  x &= 0xffffffffull;
  x = (x | (x << 16)) & 0x0000ffff0000ffffull;
  x = (x | (x << 8)) & 0x00ff00ff00ff00ffull;
  x = (x | (x << 4)) & 0x0f0f0f0f0f0f0f0full;
  x = (x | (x << 2)) & 0x3333333333333333ull;
  x = (x | (x << 1)) & 0x5555555555555555ull;
  return x;
}
#ifndef GX_STORM_TM
#define GX_STORM_TM 2  // 1024-word units per tile (one barrier per tile): 26.88 -> 26.41 ms at cfg 5
#endif                 // over TM 1 (profiles/r05/ab/storm.jsonl; TM 1 PF 4 26.54, TM 2 PF 3 26.97)
#ifndef GX_STORM_PF
#define GX_STORM_PF 2  // tiles whose loads are in flight while one is folded
#endif
template <bool EV, bool NT, int TM = GX_STORM_TM, int PF = GX_STORM_PF>
__global__ __launch_bounds__(256) void k_storm_p2(Dev d) {
  constexpr int NC = 2 * TM;     // 512-word chunks per tile (a thread takes 2 words of each)
  constexpr uint32_t TW = 1024u * TM;
  __shared__ uint32_t s_cnt[2][4 * NC];
  __shared__ uint32_t s_ecnt[2][4 * NC];
  uint32_t vi = blockIdx.x, v = d.lo + vi;
  if (departed(d, v)) return;  // uniform per block
  uint32_t half = d.H / 2;
  uint32_t lo = v < half ? half : 0, hi = v < half ? d.H : half;
  gx_host_state *h = &d.hs[vi];
  if (d.p.lock_model && locked_in(d, h->lock)) {  // block-uniform
    storm_defer(d, vi, lo, hi);
    return;
  }
  const uint32_t tail0 = h->fifo_tail, st0 = h->fifo_stored, room = fifo_room(d, h->fifo_head, tail0, st0);
  const uint32_t tail0q = tail0 % d.Q;  // the tail's ring position (jobs land at tail0q + pos < 2Q)
  uint32_t jobs = 0, n_ev = 0;
  unsigned long long c_wr = 0, c_chg = 0;
  const uint64_t tomb = pack(d.now, GX_TOMBSTONE);
  const int32_t evk = d.ev_slot[vi];
  const uint32_t ev0 = evk >= 0 ? d.ev_cnt[evk] : 0;
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint32_t LPO = d.S / 2;                      // lanes per owner
  const uint64_t omask = LPO == 32 ? 0xffffffffull : ((1ull << LPO) - 1);
  const bool leader = (lane & (LPO - 1)) == 0;
  uint64_t *row = &d.view[(size_t)vi * d.R + (size_t)lo * d.S];
  const uint32_t nw = (hi - lo) * d.S;
  // PF tiles of TW words in flight while one is folded (tile i in q[i % PF])
  ulonglong2 q[PF][NC];
  auto load = [&](uint32_t base, ulonglong2 *x) {
#pragma unroll
    for (int c = 0; c < NC; c++) {
      uint32_t r0 = base + 512 * c + 2 * t;
      if (r0 < nw) {
        if (NT) {
          v2u64 y = __builtin_nontemporal_load(reinterpret_cast<const v2u64 *>(&row[r0]));
          x[c] = make_ulonglong2(y.x, y.y);
        } else {
          x[c] = *reinterpret_cast<const ulonglong2 *>(&row[r0]);
        }
      } else {
        x[c] = make_ulonglong2(GX_SLOT_ABSENT, GX_SLOT_ABSENT);
      }
    }
  };
#pragma unroll
  for (int s = 0; s < PF; s++)
    if (s * TW < nw) load(s * TW, q[s]);
  auto tile = [&](uint32_t base, uint32_t it, const ulonglong2 *w) {
    bool lead_live[NC], live_c[NC];
    uint64_t pmask[NC];
    uint32_t rank[NC], erank[NC], sh_c[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) {
      bool p0 = st_of(w[c].x) != GX_ABSENT, p1 = st_of(w[c].y) != GX_ABSENT;
      bool l0 = p0 && st_of(w[c].x) != GX_TOMBSTONE, l1 = p1 && st_of(w[c].y) != GX_TOMBSTONE;
      uint64_t b0 = __ballot(p0), b1 = __ballot(p1), bl = __ballot(l0 || l1);
      uint32_t sh = lane & ~(LPO - 1);  // first lane of this lane's owner (S | 64: LPO a power of 2)
      bool live = ((bl >> sh) & omask) != 0;
      pmask[c] = spread32((b0 >> sh) & omask) | (spread32((b1 >> sh) & omask) << 1);
      uint64_t n0 = (p0 && live) ? tomb : w[c].x, n1 = (p1 && live) ? tomb : w[c].y;
      bool ch0 = n0 != w[c].x, ch1 = n1 != w[c].y;
      live_c[c] = live;
      sh_c[c] = sh;
      c_chg += live ? (unsigned)(p0 + p1) : 0u;  // ServiceChanged per record of a live owner
      if (ch0 || ch1) {
        if (NT) {
          v2u64 x = {n0, n1};
          __builtin_nontemporal_store(x, reinterpret_cast<v2u64 *>(&row[base + 512 * c + 2 * t]));
        } else {
          *reinterpret_cast<ulonglong2 *>(&row[base + 512 * c + 2 * t]) = make_ulonglong2(n0, n1);
        }
      }
      c_wr += ch0 + ch1;
      lead_live[c] = leader && live;
      uint64_t bj = __ballot(lead_live[c]);
      rank[c] = (uint32_t)__popcll(bj & ((1ull << lane) - 1));
      if (lane == 0) s_cnt[it][4 * c + wv] = (uint32_t)__popcll(bj);
      if (lead_live[c]) {  // serverChanged (:204-215) for a live owner: both fields in one 16-B store
        gx_server_times *st = srv_times(d, v, lo + ((base + 512 * c + 2 * t) >> d.logS));
        *reinterpret_cast<ulonglong2 *>(st) = make_ulonglong2((unsigned long long)d.now, (unsigned long long)d.now);
      }
      if (EV && evk >= 0) {  // events: owner order, then service order
        uint32_t ec = lead_live[c] ? (uint32_t)__popcll(pmask[c]) : 0u;
        uint32_t inc = ec;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          uint32_t y = __shfl_up(inc, o, 64);
          if ((int)lane >= o) inc += y;
        }
        erank[c] = inc - ec;
        if (lane == 63) s_ecnt[it][4 * c + wv] = inc;
      }
    }
    __syncthreads();
    // job positions in key order: chunk-major, then wave (chunk c of wave w is slots
    // base + 512c + 128w ..)
    uint32_t pre[NC], tot = 0;
#pragma unroll
    for (int c = 0; c < NC; c++) pre[c] = 0;
#pragma unroll
    for (int k = 0; k < 4 * NC; k++) {
      uint32_t x = s_cnt[it][k];
#pragma unroll
      for (int c = 0; c < NC; c++)
        if (k < 4 * c + (int)wv) pre[c] += x;
      tot += x;
    }
#pragma unroll
    for (int c = 0; c < NC; c++) {
      uint32_t pos = jobs + pre[c] + rank[c];
      if (lead_live[c] && pos < room) {
        uint32_t o = lo + ((base + 512 * c + 2 * t) >> d.logS);
        d.fifo[(size_t)vi * d.Q + ring_add(tail0q, pos, d.Q)] =
            make_job(pmask[c], (uint32_t)d.round, GX_JOB_META(GX_JOB_EXPIRE, 0, d.p.tombstone_count, o));
      }
    }
    jobs += tot;
    if (EV && evk >= 0) {
      uint32_t epre[NC], etot = 0;
#pragma unroll
      for (int c = 0; c < NC; c++) epre[c] = 0;
#pragma unroll
      for (int k = 0; k < 4 * NC; k++) {
        uint32_t x = s_ecnt[it][k];
#pragma unroll
        for (int c = 0; c < NC; c++)
          if (k < 4 * c + (int)wv) epre[c] += x;
        etot += x;
      }
#pragma unroll
      for (int c = 0; c < NC; c++) {
        uint32_t ob = __shfl(erank[c], (int)sh_c[c], 64);  // the owner's first event
        uint32_t r0 = base + 512 * c + 2 * t, key0 = lo * d.S + r0;
        uint32_t s0 = r0 & (d.S - 1);
        uint64_t below = pmask[c] & ((1ull << s0) - 1);
        uint32_t e0 = ev0 + n_ev + epre[c] + ob + (uint32_t)__popcll(below);
        bool p0 = st_of(w[c].x) != GX_ABSENT, p1 = st_of(w[c].y) != GX_ABSENT;
        if (live_c[c] && p0) ev_put(d, evk, e0, key0, tomb, st_of(w[c].x));
        if (live_c[c] && p1) ev_put(d, evk, e0 + p0, key0 + 1, tomb, st_of(w[c].y));
      }
      n_ev += etot;
    }
  };
  uint32_t it = 0;  // s_cnt buffer of the tile (alternates: the next tile's counts are written while
                    // slower waves may still read this one's)
  for (uint32_t base = 0; base < nw; base += PF * TW) {
#pragma unroll
    for (int s = 0; s < PF; s++) {
      const uint32_t bs = base + s * TW;
      if (bs < nw) {
        ulonglong2 w[NC];
#pragma unroll
        for (int c = 0; c < NC; c++) w[c] = q[s][c];
        if (bs + PF * TW < nw) load(bs + PF * TW, q[s]);
        tile(bs, it, w);
        it ^= 1u;
      }
    }
  }
  bool changed = c_wr != 0;
  if (__ballot(changed) != 0 && lane == 0) {
    mark_change(d);
    atomicMin(&d.minexp[vi], exp_time(d.p, tomb));
  }
  c_wr = wave_sum(c_wr);
  c_chg = wave_sum(c_chg);
  if (lane == 0) {
    kbytes(d, GX_K_STORM, 8ull * c_wr, 0);
    ctr_atomic(d, C_CHG, c_chg);
  }
  if (t == 0) {
    const uint32_t ok = jobs < room ? jobs : room;  // stored; the rest deferred (gx.h gx_job)
    h->fifo_tail = tail0 + jobs;
    h->fifo_stored = st0 + ok;
    if (jobs) d.vlc[vi] = d.now;
    if (evk >= 0) d.ev_cnt[evk] = ev0 + n_ev;
    // + 16 B of server times (LastUpdated, LastChanged) per live owner
    kbytes(d, GX_K_STORM, 8ull * (hi - lo) * d.S + 16ull * ok + 16ull * jobs, (unsigned long long)(hi - lo) * d.S);
    ctr_atomic(d, C_EXPSRV, jobs);
    ctr_atomic(d, C_QDEFER, jobs - ok);
  }
}

// ========================================================================= phase 3: gossip send ==
// The part of rng4(seed, ST_PEER, round, u, a) shared by every host of a round (sample_peers_h).
GXD uint64_t peer_seed(const Dev &d) {
  return mix64(mix64(d.p.seed ^ ((uint64_t)ST_PEER * 0xD1B54A32D192ED03ull)) ^ (uint64_t)d.round);
}
// sample_peers with the round's shared hash levels hoisted: rng4(...) = mix64(mix64(h2 ^ u) ^ a).
GXD uint32_t sample_peers_h(const Dev &d, uint64_t h2, uint32_t u, uint32_t *peers) {
  uint32_t base = 0, m = d.H;
  if (d.partitioned) {
    uint32_t half = d.H / 2;
    if (u < half) {
      base = 0;
      m = half;
    } else {
      base = half;
      m = d.H - half;
    }
  }
  if (m < 2) return 0;
  const uint64_t h3 = mix64(h2 ^ u);
  uint32_t want = d.K < m - 1 ? d.K : m - 1, cnt = 0;
  for (uint32_t a = 0; cnt < want && a < 64u * d.K; a++) {
    uint64_t x = mix64(h3 ^ a);
    uint32_t idx = unif(x, m - 1), self = u - base;
    uint32_t p = base + (idx >= self ? idx + 1 : idx);
    bool dup = false;
    for (uint32_t i = 0; i < cnt; i++) dup |= peers[i] == p;
    if (!dup) peers[cnt++] = p;
  }
  return cnt;
}
// memberlist kRandomNodes restated as a seeded sampler: k distinct peers != u on u's side.
GXD uint32_t sample_peers(const Dev &d, uint32_t u, uint32_t *peers) {
  uint32_t base = 0, m = d.H;
  if (d.partitioned) {
    uint32_t half = d.H / 2;
    if (u < half) {
      base = 0;
      m = half;
    } else {
      base = half;
      m = d.H - half;
    }
  }
  if (m < 2) return 0;
  uint32_t want = d.K < m - 1 ? d.K : m - 1, cnt = 0;
  for (uint32_t a = 0; cnt < want && a < 64u * d.K; a++) {
    uint64_t x = rng4(d.p.seed, ST_PEER, (uint64_t)d.round, u, a);
    uint32_t idx = unif(x, m - 1), self = u - base;
    uint32_t p = base + (idx >= self ? idx + 1 : idx);
    bool dup = false;
    for (uint32_t i = 0; i < cnt; i++) dup |= peers[i] == p;
    if (!dup) peers[cnt++] = p;
  }
  return cnt;
}

// Diagnostics: wall-clock mark k of this wave (k_send phases; Dev::kprof, env GX_KPROF).
#define GX_KP(k)                                                                                   \
  do {                                                                                             \
    if (d.kprof && (threadIdx.x & 63) == 0)                                                        \
      d.kprof[((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8 + (k)] = wall_clock64(); \
  } while (0)

// ---------------------------------------------------------------- planned GetBroadcasts --
// The same GetBroadcasts calls (record budget, no byte limit, no failure detector or departures,
// TOMBSTONE_RETRANSMIT > 0 so re-armed passes sleep and nothing is pushed to the FIFO during the
// sends) in two steps per chunk of up to PLAN_CH calls:
//  1. the control plan: each call's dequeued job (from the FIFO head jobs loaded up front), batch
//     length m, packet length l, and the pending ring's head before and after, with every FIFO,
//     sleep-ring and counter update of the call. This touches no record, so the calls of a chunk
//     plan back to back with no memory round trip.
//  2. the records of all the chunk's packets at once: record f of the chunk belongs to call k
//     (prefix sums of l) at index i; i < m is batch item i of k's job (list arena, job fields),
//     else pending ring position head_k + i - m, whose content is the batch of an earlier call of
//     the chunk that left records pending there (the latest such call), or the ring as loaded.
//     Every record load of the chunk is in flight together, then every receiver slot read of the
//     senders' filter, then the stores: a record that is stale or no newer than the receiver's
//     slot is a no-op at any position of the receiver's fold (see k_merge), so only live records
//     are written, compacted per packet, and a packet without one is not registered at all.
// Batch records that stay pending are written to the ring after the chunk's loads, position p by
// team lane p % T in call order (the sequential order of the ring writes).
#ifndef PLAN_CH
#define PLAN_CH 4  // calls planned per chunk
#endif
// Diagnostics (build with -DGX_SEND_SPLIT, engine created with GX_KPROF set): per wave, the time
// its lane-0 team spends in each part of the chunk loop, summed over chunks, in place of the
// k_send phase marks 1..6: plan, records, headers, ring writes + sync, chunks, refills.
#ifdef GX_SEND_SPLIT
#define GX_SPLIT_DECL unsigned long long sp_t = wall_clock64(), sp_acc[4] = {0, 0, 0, 0}, sp_n = 0, sp_rf = 0;
#define GX_SPLIT(k)                              \
  do {                                           \
    const unsigned long long t_ = wall_clock64(); \
    sp_acc[k] += t_ - sp_t;                      \
    sp_t = t_;                                   \
  } while (0)
#define GX_SPLIT_FLUSH()                                                                                 \
  do {                                                                                                   \
    if (d.kprof && (threadIdx.x & 63) == 0) {                                                           \
      unsigned long long *k_ = &d.kprof[((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8]; \
      k_[1] = sp_acc[0];                                                                                 \
      k_[2] = sp_acc[1];                                                                                 \
      k_[3] = sp_acc[2];                                                                                 \
      k_[4] = sp_acc[3];                                                                                 \
      k_[5] = sp_n;                                                                                      \
      k_[6] = sp_rf;                                                                                     \
    }                                                                                                    \
  } while (0)
#else
#define GX_SPLIT_DECL
#define GX_SPLIT(k) \
  do {              \
  } while (0)
#define GX_SPLIT_FLUSH() \
  do {                   \
  } while (0)
#endif
#ifndef GX_PLAN_RECS
#define GX_PLAN_RECS 32
#endif
#define PLAN_RECS GX_PLAN_RECS  // records of a chunk in flight per team (PLAN_RECS / T per lane)
struct PlanCall {
  // batch item i (i < m) as the record phase builds it: EXPIRE {bw, rb + (emask ? nth set bit : i)},
  // SEND {list[i].w + bw, list[i].r}, RETX {bw, rb}
  uint64_t bw;        // EXPIRE: the tombstone word; SEND: the pass increment; RETX: the record word
  uint64_t emask;     // EXPIRE: the service mask unless it is every service (0)
  const grec *list;   // SEND: the list records
  const uint64_t *row;  // the receiver's view row when it is on this shard (the filter), else null
  uint32_t kind, rb;  // job kind (0xff: none); EXPIRE: owner * S; RETX: the record key
  uint32_t m, l;      // batch length, packet length (> 0)
  uint32_t head, nh;  // pending ring head before and after the call
  uint32_t push;      // batch records left pending (written at nh .. nh + push - 1)
  uint32_t x, key;    // packet entry, global packet key
  uint32_t peer;      // receiver (global id)
  uint32_t lpre;      // records of the chunk's earlier calls
  uint32_t lk;        // the receiver (on this shard) holds the ServicesState lock this round
  uint32_t oslot;     // the packet's slot in the planned send buffer (Dev::ob_buf), or GX_NOSLOT
};
// The receiver's shard (hosts in contiguous blocks, floor(g * H / G) the first of shard g).
GXD uint32_t shard_of_d(const Dev &d, uint32_t v) {
  uint32_t g = (uint32_t)(((uint64_t)v * d.G) / d.H);
  while (g > 0 && (uint32_t)(((uint64_t)g * d.H) / d.G) > v) g--;
  while (g + 1 < d.G && (uint32_t)(((uint64_t)(g + 1) * d.H) / d.G) <= v) g++;
  return g;
}
// Slot header and records of the planned send buffer (k_outbox_pack_planned's layout).
GXD uint32_t *ob_slot_hdr(const Dev &d, uint32_t slot) {
  return reinterpret_cast<uint32_t *>(d.ob_buf + (size_t)slot * (16u + 16u * d.p.packet_cap));
}
static_assert(sizeof(PlanCall) >= 17 * sizeof(uint32_t), "a PlanCall slot holds a team's 16 peers and their count");
#define GX_NOSLOT 0xffffffffu  // inbox header slot: the records are in the message entry
// ... and each carries the receiver's slot word it was filtered against (msg_w0). Between that read
// and the receiver's merge only the receiver's own tick (its own records) and its expiry scan
// (a view whose tick is 2) write the view, so for every other record the merge takes that word
// instead of reading the slot again.
#define GX_NOSLOT_W0 0xfffffffeu
GXD bool w0_fwd(const Dev &d, uint32_t slot, uint32_t tick, uint32_t key, uint32_t v) {
  return slot == GX_NOSLOT_W0 && tick != 2 && !owned_by(d, key, v);
}

// Batch item i of a planned call's job (get_broadcasts_team's item() for i < m).
GXD grec plan_item(const Dev &d, const PlanCall &c, uint32_t i) {
  grec g;
  g.pad = 0;
  if (c.kind == GX_JOB_SEND) {  // Updated + pass * 50ns (services_state.go:588-599)
    const grec s = c.list[i];
    g.w = s.w + c.bw;
    g.r = s.r;
  } else if (c.kind == GX_JOB_EXPIRE) {  // the i-th tombstoned service of the owner
    g.w = c.bw;
    g.r = c.rb + (c.emask ? nth_set_bit(c.emask, i) : i);
  } else {  // RETX
    g.w = c.bw;
    g.r = c.rb;
  }
  return g;
}

// Every lane of host idx's team calls it (team-uniform hs, peers, np); lead lane stores.
// kb: algorithmic bytes (the caller flushes them to GX_K_SEND).
template <int T>
GXD void send_planned(const Dev &d, Acc &a, uint32_t idx, gx_host_state &hs, gx_job *pjs, PlanCall *pl,
                      const uint32_t *peers, uint32_t np, unsigned long long &kb, unsigned long long &kl,
                      uint32_t npf0 = 0) {
  constexpr int PLAN_Q = PLAN_RECS / T;
  const uint32_t lane = threadIdx.x & 63, tl = lane & (T - 1), tw = lane / T;
  const bool lead = tl == 0;
  const uint64_t tmask = T == 64 ? ~0ull : ((1ull << T) - 1ull);
  const uint32_t u = d.lo + idx, cap = d.p.packet_cap, mask = d.DQ - 1;
  grec *dq = &d.dq[(size_t)idx * d.DQ];
  grec *const arena_t = &d.arena[(size_t)idx * d.A * d.L];  // the host's SendServices lists
  // the team's message entries (its packets' records and filter words): entry x = idx * KE + k
  grec *const msg_t = &d.msg[(size_t)idx * d.KE * cap];
  uint64_t *const w0_t = &d.msg_w0[(size_t)idx * d.KE * cap];
  const int64_t t_stale = d.now - d.p.tombstone_lifespan_ns - d.p.stale_fudge_ns;
  const int64_t t_gc = d.now - d.p.tombstone_lifespan_ns;
  // FIFO head jobs, T at a time: position pf0 + q in pjs[q], q < npf (npf0 already loaded)
  uint32_t pf0 = hs.fifo_head, npf = npf0;
  uint32_t j = 0, n = 0;
  bool stop = np == 0;
  unsigned fm = 0, fs = 0, nlines = 0;
  GX_SPLIT_DECL
  const bool lmod = d.p.lock_model != 0;
  // The planned exchange packed here (Dev::ob_buf; GossipMessages 1, so entry j = peer j): every
  // peer on another shard gets a slot of its shard's region up front (lane tl claims for peers
  // tl + T * r), written with the packet's header and records, or as an empty slot at the end.
  constexpr int NR = (16 + T - 1) / T;
  const bool direct = d.ob_buf != nullptr;
  uint32_t osl[NR];
  uint32_t emit = 0;  // team-uniform: peers whose packet went into its slot
#pragma unroll
  for (int r = 0; r < NR; r++) osl[r] = GX_NOSLOT;
  // One atomic per destination shard per wave (thousands of single claims on G counters queue
  // at L2): the wave's claims for a shard take consecutive places in (r, lane) order, and the
  // first of them claims the run; every run's atomic is in flight at once, beside the lock loads.
  uint32_t og[NR], rk[NR], ksrc[NR], krun[NR], lc[NR], lb[NR], le[NR];
  if (direct) {
    unsigned long long pend[NR];
#pragma unroll
    for (int r = 0; r < NR; r++) {
      const uint32_t jj = (uint32_t)r * T + tl;
      og[r] = jj < np && peers[jj] - d.lo >= d.Hl ? shard_of_d(d, peers[jj]) : d.G;
      pend[r] = __ballot(og[r] < d.G);
      rk[r] = ksrc[r] = krun[r] = lc[r] = 0;
    }
    for (;;) {  // wave-uniform: one pass per destination shard the wave sends to
      int r0 = -1;
#pragma unroll
      for (int r = NR - 1; r >= 0; r--) r0 = pend[r] ? r : r0;
      if (r0 < 0) break;
      unsigned long long p0 = pend[0];
      uint32_t g0 = og[0];
#pragma unroll
      for (int r = 1; r < NR; r++) {
        p0 = r == r0 ? pend[r] : p0;
        g0 = r == r0 ? og[r] : g0;
      }
      const uint32_t src = (uint32_t)__builtin_ctzll(p0);  // the run's first claim: (src, r0)
      const uint32_t gs = (uint32_t)__shfl((int)g0, (int)src, 64);
      uint32_t acc = 0;
#pragma unroll
      for (int r = 0; r < NR; r++) {
        const unsigned long long m = __ballot(og[r] == gs);
        if (og[r] == gs) {
          rk[r] = acc + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
          ksrc[r] = src;
          krun[r] = (uint32_t)r0;
        }
        acc += (uint32_t)__popcll(m);
        pend[r] &= ~m;
      }
#pragma unroll
      for (int r = 0; r < NR; r++)
        if (r == r0 && lane == src) lc[r] = acc;
    }
#pragma unroll
    for (int r = 0; r < NR; r++) {  // a run's places: its first claim's registers (used after the lock loads)
      lb[r] = le[r] = 0;
      if (lc[r]) {
        lb[r] = atomicAdd(&d.ob_claim[og[r]], lc[r]);
        le[r] = d.ob_cnt[og[r]];
      }
    }
  }
  // the receivers' ServicesState lock this round (gx.h lock_model): bit j = peer j, on this shard,
  // holds it. A locked receiver's records all go to its pipeline (k_merge_seg), so they are stored
  // unfiltered and the receiver counts them; with lock_model = 0 they merge and are counted as locked.
  // A locked receiver whose pipeline was full when the round began (its count changes only in the
  // merge) drops every record of this round (memberlist's handoff queue): the call's packet is
  // counted as dropped here and neither stored nor registered (bit j of fullm).
  uint32_t lkm = 0, fullm = 0;
  for (uint32_t j0 = 0; j0 < np; j0 += T) {
    const uint32_t jj = j0 + tl;
    const uint32_t lw = jj < np && peers[jj] - d.lo < d.Hl ? gld(&hst(d, peers[jj])->lock) : 0u;
    const bool lk = locked_in(d, lw);
    lkm |= (uint32_t)((__ballot(lk) >> (tw * T)) & tmask) << j0;
    const bool full = lk && GX_LOCK_BUF(lw) >= pipe_cap(d, jj < np ? peers[jj] - d.lo : 0u, lw);
    fullm |= (uint32_t)((__ballot(full) >> (tw * T)) & tmask) << j0;
  }
  if (direct) {
#pragma unroll
    for (int r = 0; r < NR; r++) {  // [lb, le): the run's places in the buffer (region start + claim)
      if (lc[r]) {  // a run starts at this claim
        uint32_t st = 0;
        for (uint32_t x = 0; x < og[r]; x++) st += d.ob_cnt[x];
        if (lb[r] + lc[r] > le[r]) atomicOr(&d.work_cnt[GX_WC_ERR], GX_ERR_INBOX);  // past the plan's bound (cannot happen)
        lb[r] += st;
        le[r] += st;
      }
    }
#pragma unroll
    for (int r = 0; r < NR; r++) {
      uint32_t b = 0, e = 0;
#pragma unroll
      for (int r2 = 0; r2 < NR; r2++) {
        const uint32_t x = (uint32_t)__shfl((int)lb[r2], (int)ksrc[r], 64), y = (uint32_t)__shfl((int)le[r2], (int)ksrc[r], 64);
        if (krun[r] == (uint32_t)r2) {
          b = x;
          e = y;
        }
      }
      if (og[r] < d.G && b + rk[r] < e) osl[r] = b + rk[r];
    }
  }
  while (!stop) {
#ifdef GX_SEND_SPLIT
    sp_n++;
    sp_t = wall_clock64();
#endif
    // ---- 1. plan up to PLAN_CH calls (control state only)
    uint32_t nc = 0, tot = 0;
    bool any_push = false;
    while (nc < PLAN_CH && !stop) {
      PlanCall c;
      c.kind = 0xffu;
      c.bw = c.emask = 0;
      c.rb = 0;
      c.list = nullptr;
      c.m = 0;
      c.push = 0;
      c.peer = peers[j];
      c.row = c.peer - d.lo < d.Hl ? &d.view[(size_t)(c.peer - d.lo) * d.R] : nullptr;
      c.lk = ((lkm >> j) & 1u) | (lmod ? ((fullm >> j) & 1u) << 1 : 0u);
      c.x = idx * d.KE + j * d.NG + n;
      c.key = u * d.KE + j * d.NG + n;
      c.oslot = GX_NOSLOT;
      if (direct && !c.row) {  // peer j's claimed slot (lane j % T of the team, register j / T)
        uint32_t v = osl[0];
#pragma unroll
        for (int r = 1; r < NR; r++) v = j / T == (uint32_t)r ? osl[r] : v;
        c.oslot = (uint32_t)__shfl((int)v, (int)(j % T), T);
      }
      bool empty = false;
      if (hs.fifo_head != hs.fifo_tail) {  // case broadcast = <-d.state.Broadcasts (:94)
        gx_job jb = make_job(0, 0, 0);
        if (hs.fifo_head != hs.fifo_stored) {  // a stored job: from the LDS window
          uint32_t q = hs.fifo_head - pf0;
          if (q >= npf) {  // load the next stored head jobs (T, or GX_JPF * T under GossipMessages > 1)
            const uint32_t left = hs.fifo_stored - hs.fifo_head, win = pj_window<T>(d);
            const uint32_t nl = left < win ? left : win;
            wave_sync();
            for (uint32_t x = tl; x < nl; x += T) pjs[x] = d.fifo[(size_t)idx * d.Q + ((hs.fifo_head + x) % d.Q)];
            wave_sync();
#ifdef GX_SEND_SPLIT
            sp_rf++;
#endif
            pf0 = hs.fifo_head;
            npf = nl;
            q = 0;
            if (lead) kb += 16ull * npf;
          }
          jb = pjs[q];
          hs.fifo_head++;
        } else {
          jb = pop_job_r(d, idx, hs, nullptr);  // past the stored window: a looper's nil or LOST
        }
        if (lead) a.c[C_DEQ]++;
        const uint32_t kind = GX_JOB_KIND(jb.meta), pass = GX_JOB_PASS(jb.meta), npass = GX_JOB_NPASSES(jb.meta);
        if (kind == GX_JOB_LOST) {  // a deferred job reached the head: its batch is unknown
          count_lost(d, a, lead);
        } else if (kind == GX_JOB_NIL_BS) {  // the BroadcastServices looper unblocks (services_state.go:569)
          if (lead) a.c[C_NIL]++;
          hs.flags &= ~1u;
          hs.bs_next = d.round + d.p.alive_interval_rounds;
        } else if (kind == GX_JOB_NIL_BT) {  // ... BroadcastTombstones (:628)
          if (lead) a.c[C_NIL]++;
          hs.flags &= ~2u;
          hs.bt_next = d.round + d.p.tombstone_interval_rounds;
        } else if (kind == GX_JOB_SEND || kind == GX_JOB_EXPIRE) {
          if (pass + 1 < npass) {  // the looper re-arms after TOMBSTONE_RETRANSMIT (:585-601)
            gx_job nj = jb;
            nj.meta = GX_JOB_META(kind, pass + 1, npass, GX_JOB_OWNER(jb.meta));
            push_sleep_r(d, a, u, hs, nj, (uint32_t)(d.round + d.p.retransmit_rounds), lead);
          } else {
            free_list_r(d, idx, hs, jb, lead);  // read below; nothing reallocates it during the sends
          }
        }
        c.m = job_len(d, jb);
        c.kind = kind;
        const uint64_t dw = ((uint64_t)pass * (uint64_t)d.p.pass_increment_ns) << GX_TS_SHIFT;
        if (kind == GX_JOB_RETX) {
          c.bw = jb.a;
          c.rb = jb.c;
        } else if (kind == GX_JOB_SEND) {
          c.bw = dw;
          c.list = arena_t + (size_t)(jb.c & 0xffffu) * d.L;  // list_ptr(d, u, slot)
        } else if (kind == GX_JOB_EXPIRE) {  // Tombstone() at the call's now
          c.bw = pack(d.p.t0_ns + (int64_t)jb.c * d.p.round_ns, GX_TOMBSTONE) + dw;
          c.rb = GX_JOB_OWNER(jb.meta) * d.S;
          c.emask = (uint32_t)__popcll(jb.a) == d.S ? 0ull : jb.a;
        }
      } else if (hs.dq_len == 0) {  // default: nothing pending (:96-98)
        empty = true;
      }
      uint32_t l = 0;
      if (!empty) {  // packPacket's greedy prefix (:186-223) of batch ++ pendingBroadcasts
        const uint32_t nn = c.m + hs.dq_len;
        l = nn < cap ? nn : cap;
        c.head = hs.dq_head;
        if (l < c.m) {  // leftover = broadcast[l:]: batch records stay pending in front
          c.push = c.m - l;
          c.nh = (c.head - c.push) & mask;
          any_push = true;
        } else {
          c.nh = (c.head + (l - c.m)) & mask;
        }
        hs.dq_head = c.nh;
        hs.dq_len = nn - l;
        if (hs.dq_len > d.p.pending_cap) {  // pendingBroadcasts = leftover[:MAX_PENDING_LENGTH]
          if (lead) a.c[C_PDROP] += hs.dq_len - d.p.pending_cap;
          hs.dq_len = d.p.pending_cap;
        }
        if (l && lead) {
          a.c[C_PACKETS]++;
          a.c[C_RECSENT] += l;
          // records read from a list or the ring, and the receiver slots the filter reads
          const uint32_t lb = l < c.m ? l : c.m;
          const bool filt = c.row && !(lmod && c.lk);
          if (c.lk & 2u) {
            a.c[C_LOCK_DROP] += l;  // nothing of the packet is loaded or stored
          } else {
            kb += 16ull * ((c.kind == GX_JOB_SEND ? lb : 0u) + (l - lb)) + (filt ? 8ull * l : 0ull);
          }
          if (filt) fm += l;
          if (c.lk) {
            a.locked = true;
            if (!lmod) a.c[C_LOCKED_MERGES] += l;
          }
        }
      }
      c.l = l;
      c.lpre = tot;
      if (l) {  // (a dropped packet stays in the plan for its pending-ring writes; no record of it loads)
        if (c.oslot != GX_NOSLOT) emit |= 1u << j;
        if (lead) pl[nc] = c;
        nc++;
        if (!(c.lk & 2u)) tot += l;
      }
      // a call that leaves batch records pending ends the chunk: its ring writes follow the
      // chunk's loads, so no call of a chunk reads what another call of it wrote
      const bool pushed = c.push != 0;
      // GossipMessages: up to NG gathers per target; a target's gathering ends at an empty result,
      // an empty first gather ends the round (gossip_stop_on_empty)
      if (l == 0) {
        if (n == 0 && d.p.gossip_stop_on_empty) stop = true;
        j++;
        n = 0;
      } else if (++n == d.NG) {
        j++;
        n = 0;
      }
      if (j >= np) stop = true;
      if (pushed) break;
    }
    if (nc == 0) break;
    wave_sync();  // the plan in LDS
#ifndef GX_SEND_SPLIT
    if (j <= PLAN_CH) GX_KP(5);
#endif
    GX_SPLIT(0);
    // ---- 2. the chunk's records: loads, receiver slots, compacted stores. Record f of the chunk
    // belongs to call k (lpre), its live rank in the packet is run(f) - run(lpre_k), where run(x)
    // counts the live records before x (ballot prefix over the team, call starts in cb[]).
    uint32_t lp[PLAN_CH], cb[PLAN_CH];
#pragma unroll
    for (int k = 0; k < PLAN_CH; k++) {
      lp[k] = (uint32_t)k < nc ? pl[k].lpre : 0xffffffffu;
      cb[k] = 0;
    }
    uint32_t run = 0;
    uint32_t lcarry = 0xffffffffu;  // the view line of the team's last filtered record (diagnostic)
    for (uint32_t fb = 0; fb < tot; fb += T * PLAN_Q) {
      // Every load of the block is issued unconditionally (a record that needs none loads ring
      // slot 0, one past the end of the chunk loads it too) and used only after all are in flight:
      // a load guarded by a branch makes the compiler wait for it on the spot.
      uint64_t w[PLAN_Q];
      uint32_t r[PLAN_Q], ck[PLAN_Q];
      uint32_t sel[PLAN_Q];  // 0: computed from the job; 1: loaded list record (+ pass); 2: loaded ring record
      gx_u32x3 lx[PLAN_Q];   // the loads, kept apart from the computed words until all are issued
      uint64_t w0[PLAN_Q];   // the receivers' slots (senders' filter)
#pragma unroll
      for (int q = 0; q < PLAN_Q; q++) {
        const uint32_t f = fb + tl + T * q;
        uint32_t k = 0;
#pragma unroll
        for (int kk = 1; kk < PLAN_CH; kk++) k += f >= lp[kk] ? 1u : 0u;
        ck[q] = k;
        const PlanCall &c = pl[k];
        const uint32_t i = f - c.lpre;
        const bool valid = f < tot, batch = i < c.m;
        const grec *src = dq;
        sel[q] = 0;
        if (valid && batch && c.kind == GX_JOB_SEND) {
          src = &c.list[i];
          sel[q] = 1;
        } else if (valid && !batch) {
          src = &dq[(c.head + (i - c.m)) & mask];
          sel[q] = 2;
        }
        lx[q] = gld3(src);
        w[q] = c.bw;  // computed: the job's word
        r[q] = c.rb + (c.kind == GX_JOB_EXPIRE ? (c.emask ? nth_set_bit(c.emask, i) : i) : 0u);
        // the senders' filter reads the local receiver's slot; a computed record's key is known
        // now, so its slot load goes out with the record loads (one round trip for both). Records
        // nobody filters (a locked or remote receiver) load slot 0 of view 0 instead (one line).
        const bool filt = valid && c.row && !(lmod && c.lk);
        const uint64_t *row = filt ? c.row : reinterpret_cast<const uint64_t *>(dq);  // (a line of the team's ring)
        w0[q] = gld(&row[filt && sel[q] == 0 && r[q] < d.R ? r[q] : 0u]);
      }
      bool reload = false;  // a loaded record that is filtered: its slot load needs the record's key
#pragma unroll
      for (int q = 0; q < PLAN_Q; q++) {
        const PlanCall &c = pl[ck[q]];
        if (sel[q]) {  // loaded (+ pass * 50 ns for a list record, services_state.go:588-599)
          w[q] = ((uint64_t)lx[q].x | ((uint64_t)lx[q].y << 32)) + (sel[q] == 1 ? w[q] : 0ull);
          r[q] = lx[q].z;
          reload |= c.row && !(lmod && c.lk);
        }
      }
      if (__ballot(reload)) {  // wave-uniform: a second round trip only where a wave needs it
#pragma unroll
        for (int q = 0; q < PLAN_Q; q++) {
          const PlanCall &c = pl[ck[q]];
          const bool fl = sel[q] && c.row && !(lmod && c.lk);
          const uint64_t *row = fl ? c.row : reinterpret_cast<const uint64_t *>(dq);
          const uint64_t x = gld(&row[fl && r[q] < d.R ? r[q] : 0u]);
          w0[q] = fl ? x : w0[q];
        }
      }
#pragma unroll
      for (int q = 0; q < PLAN_Q; q++) {
        const uint32_t f = fb + tl + T * q, base = fb + T * q;
        const uint32_t k = ck[q];
        const PlanCall &c = pl[k];
        const bool valid = f < tot;
        const bool filt = c.row && !(lmod && c.lk);
        bool live = valid;
        if (valid && filt) {
          const int64_t ts = ts_of(w[q]);
          const bool stale = ts < t_stale;
          const bool gc = st_of(w0[q]) == GX_TOMBSTONE && ts_of(w0[q]) < t_gc;
          live = !stale && (st_of(w0[q]) == GX_ABSENT || ts > ts_of(w0[q]) || gc);
          fs += stale;
        }
        const uint64_t lm = (__ballot(live) >> (tw * T)) & tmask;
#pragma unroll
        for (int kk = 1; kk < PLAN_CH; kk++)  // run() at the calls starting in this block
          if (lp[kk] >= base && lp[kk] < base + T) cb[kk] = run + (uint32_t)__popcll(lm & ((1ull << (lp[kk] - base)) - 1ull));
        uint32_t cbk = 0;
#pragma unroll
        for (int kk = 1; kk < PLAN_CH; kk++) cbk = (uint32_t)kk == k ? cb[kk] : cbk;
        const uint32_t rank = filt ? run + (uint32_t)__popcll(lm & ((1ull << tl) - 1ull)) - cbk : f - c.lpre;
        {  // 128-B receiver view lines the filter read: a filtered record on a line other than the
           // previous record's (packet order) starts one (gx_timing.units of GX_K_SEND)
          const uint32_t line = valid && filt ? ((c.peer << 15) | (r[q] >> 4)) : 0xffffffffu;  // exact for R <= 2^19
          const uint32_t tb = lane & ~(uint32_t)(T - 1);
          const uint32_t up = (uint32_t)__shfl((int)line, (int)(tl ? lane - 1 : lane), 64);
          const uint32_t prev = tl ? up : lcarry;
          nlines += line != 0xffffffffu && line != prev;
          lcarry = (uint32_t)__shfl((int)line, (int)(tb + T - 1), 64);
        }
        if (live) {
          grec g;
          g.w = w[q];
          g.r = r[q];
          g.pad = 0;
          const uint32_t xo = (c.x - idx * d.KE) * cap + rank;  // within the team's entries
          grec *to = c.oslot != GX_NOSLOT ? reinterpret_cast<grec *>(ob_slot_hdr(d, c.oslot) + 4) + rank : &msg_t[xo];
          gst_rec(to, g);
          if (filt) gst(&w0_t[xo], w0[q]);
        }
        run += (uint32_t)__popcll(lm);
      }
    }
#pragma unroll
    for (int kk = 1; kk < PLAN_CH; kk++)  // dropped packets at the chunk's end start past its records
      if (lp[kk] == tot) cb[kk] = run;
    uint32_t stored_all = 0;  // records this team stores: the packets' headers below
    // ---- packet headers: lane k registers call k's packet when it holds a record
#ifndef GX_SEND_SPLIT
    if (j <= PLAN_CH) GX_KP(6);
#endif
    GX_SPLIT(1);
    if (tl < nc) {
      const PlanCall &c = pl[tl];
      uint32_t stored = 0;
#pragma unroll
      for (int kk = 0; kk < PLAN_CH; kk++) {
        const uint32_t end = kk + 1 < PLAN_CH && (uint32_t)(kk + 1) < nc ? cb[kk + 1] : run;
        stored = (uint32_t)kk == tl ? end - cb[kk] : stored;
      }
      const uint32_t rv = c.peer - d.lo;
      if (!c.row) stored = c.l;  // another shard's receiver filters on arrival (k_inbox_unpack)
      if (c.lk & 2u) stored = 0;
      d.msg_len[c.x] = stored;
      d.msg_dst[c.x] = c.peer;
      if (c.oslot != GX_NOSLOT)  // the slot header (k_outbox_pack_planned's pack_slot)
        *reinterpret_cast<uint4 *>(ob_slot_hdr(d, c.oslot)) = make_uint4(c.key, c.peer, stored, 0u);
      if (c.row && stored) {  // a locked receiver reads its slots itself (no forwarded words)
        inbox_header(d, rv, inbox_claim(d, rv), c.key, c.x, stored, lmod && c.lk ? GX_NOSLOT : GX_NOSLOT_W0);
        flag_live(d, rv, stored);
      }
      stored_all = stored + ((c.row && stored) ? 2u : 0u);  // a header and its count ~ 2 records
    }
    kb += 16ull * stored_all;
    GX_SPLIT(2);
    // ---- batch records left pending: position p by lane p % T, in call order
    if (any_push) {
      for (uint32_t k = 0; k < nc; k++) {
        const PlanCall &c = pl[k];
        for (uint32_t qq = (tl - c.nh) & (T - 1); qq < c.push; qq += T) {
          dq[(c.nh + qq) & mask] = plan_item(d, c, c.l + qq);
          kb += 16;
        }
      }
      __threadfence_block();  // the next chunk may read them on other lanes
    }
    wave_sync();  // the plan slots are rewritten by the next chunk
    GX_SPLIT(3);
  }
  GX_SPLIT_FLUSH();
#pragma unroll
  for (int r = 0; r < NR; r++)  // claimed slots no packet went into: empty (the receiver skips them)
    if (osl[r] != GX_NOSLOT && !((emit >> ((uint32_t)r * T + tl)) & 1u))
      *reinterpret_cast<uint4 *>(ob_slot_hdr(d, osl[r])) = make_uint4(GX_SLOT_EMPTY, 0u, 0u, 0u);
  a.c[C_GOSSIP_MERGES] += fm;
  kl += nlines;
  a.c[C_STALE] += fs;
}

// A team of T lanes per host: first the rest of a BroadcastTombstones tick (TombstoneServices +
// SendServices of own ++ others, services_state.go:606-633; lane 0, after the expiry scan), then
// GetBroadcasts once per sampled peer, in order (get_broadcasts_team). Each packet is registered
// in its receiver's inbox (inbox_claim / inbox_header).
// X (failure detector or departures): the targets are memberlist's (k_fd_send took their
// memberlist messages first and, in byte mode, the delegate gets the bytes left; the round stops
// at a packet that would be empty), and a packet to an unreachable peer is lost after
// GetBroadcasts took its records.
GXD bool filt_used(const Dev &d, uint32_t pos) { return d.sfilt && pos != 0xffffffffu; }
// PLAN: send_planned (the engine picks it when its conditions hold: record budget, !X, retransmit
// sleep > 0, senders' filter).
template <int T, bool X, bool PLAN = false, bool FWD = false>
GXD void send_host(const Dev &d, Acc &a, uint32_t idx, gx_job *pjs, int do_bt, unsigned &lost, PlanCall *pl,
                   unsigned long long &kb, unsigned long long &kl, const TickFwd &fwd) {
  const uint32_t lane = threadIdx.x & (T - 1);
  {
    uint32_t u = d.lo + idx;
    uint32_t cap = d.p.packet_cap;
    gx_host_state *h = &d.hs[idx];
    // the bookkeeping and tick flag: from the owner tick of this launch, or loaded (both before any store)
    gx_host_state hs = FWD ? fwd.hs : *h;
    const bool tick = do_bt && (FWD ? fwd.tick != 0 : d.tick[idx] != 0);
    bool pre = FWD;  // the FIFO head jobs the tick loaded are still at the head
    for (uint32_t j = lane; j < d.KG; j += T) {  // (the probe entries past KG were written by k_probe)
      d.msg_len[(size_t)idx * d.KE + j] = 0;
      d.msg_key[(size_t)idx * d.KE + j] = u * d.KE + j;
    }
    // the ExpireServer calls that waited for the host's lock end its owner phase (gx.h lock_model)
    const bool pend = do_bt && d.pexp && (hs.lock & GX_LOCK_PENDING_EXPIRE) && !locked_in(d, hs.lock) &&
                      (!X || !departed(d, u));
    if (tick || pend) {  // departed hosts never tick
      if (lane == 0) {
        const uint32_t n = d.scan_cnt[idx];
        if (tick) bt_finish(d, a, u, hs.running, &d.scan_list[(size_t)idx * d.L], n < d.L ? n : d.L);
        if (pend) {
          run_pending_expires(d, a, u);
          // other hosts' senders may have read this view's slots before the calls rewrote them: the
          // merge reads its slots itself (as for a view scanned this round), not the forwarded words
          d.tick[idx] = 2;
        }
      }
      __threadfence_block();  // the team reads the host's bookkeeping below
      hs = *h;
      pre = false;  // the finish pushed to the FIFO: its head jobs are loaded again
    }
    if (lane == 0) kb += 128;  // the host's bookkeeping read and written
    GX_KP(4);
    if (PLAN) {
      uint32_t *peers = reinterpret_cast<uint32_t *>(&pl[PLAN_CH]);  // the team's peers (k_send's prologue)
      const uint32_t np = peers[16];
      send_planned<T>(d, a, idx, hs, pjs, pl, peers, np, kb, kl, (pre && fwd.pf0 == hs.fifo_head) ? fwd.npf : 0u);
      hs.lock = lock_snap(hs.lock, hs.flags, d.round + 1, d.p.lock_readers != 0);  // the lock for the next round
      if (lane == 0) *h = hs;
    } else if (!X || !departed(d, u)) {
      const bool fd = X && d.p.fd_enable;
      uint32_t peers[16];
      uint32_t np;
      if (fd) {
        np = d.fd_np[idx];
        for (uint32_t j = 0; j < np; j++) peers[j] = d.fd_peers[(size_t)idx * d.K + j];
      } else {
        np = sample_peers(d, u, peers);
      }
      // The jobs at the FIFO head that this round's calls will dequeue are loaded up front, one
      // per team lane (call c takes job c while c < the jobs queued at the start: later pushes go
      // to the tail and cannot overwrite them), so a call waits on its list records only.
      const uint32_t head0 = hs.fifo_head, n0 = hs.fifo_stored - head0;  // stored jobs only
      if (lane < n0 && lane < np * d.NG) pjs[lane] = d.fifo[(size_t)idx * d.Q + ((head0 + lane) % d.Q)];
      // A packet to a reachable peer on this shard takes its receiver inbox slot before it is
      // packed, so its records go straight into the receiver's inbox when the slot is one of the
      // DR inline ones. With np <= T the claims are made up front, one lane per peer, their
      // atomics in flight together; otherwise lane 0 claims before each call.
      const bool early = np <= (uint32_t)T && d.NG == 1;
      uint32_t my_pos = 0xffffffffu;
      if (early && lane < np && (!X || reach(d, u, peers[lane])) && peers[lane] - d.lo < d.Hl)
        my_pos = inbox_claim(d, peers[lane] - d.lo);
      uint32_t called = 0;
      bool stop = false;
      for (uint32_t j = 0; j < np && !stop; j++) {
        const uint32_t pj = peers[j];
        const bool ok = !X || reach(d, u, pj), local = pj - d.lo < d.Hl;
        // GossipMessages: up to NG gathers per target, each its own packet (entry j * NG + n); a
        // target's gathering ends at an empty result, an empty first gather ends the round
        for (uint32_t n = 0; n < d.NG; n++) {
          const uint32_t c = j * d.NG + n;
          const size_t x = (size_t)idx * d.KE + c;
          uint32_t pos;
          if (early) {
            pos = __shfl(my_pos, (int)j, T);
          } else {
            pos = lane == 0 && ok && local ? inbox_claim(d, pj - d.lo) : 0xffffffffu;
            pos = __shfl(pos, 0, T);
          }
          uint32_t nf = fd ? d.fd_len[x] : 0, lim = d.p.limit_bytes, l = 0;
          bool call = true;
          if (fd && lim) {
            uint32_t used = nf * (d.p.fd_msg_bytes + 2);
            lim = lim > used ? lim - used : 0;
            call = lim > d.p.overhead_bytes;
          }
          grec *pk = pos < d.DR ? &d.in_rec[((size_t)(pj - d.lo) * d.DR + pos) * cap] : &d.msg[x * cap];
          // the receiver holds the ServicesState lock this round (gx.h lock_model): its records all go
          // to its pipeline unfiltered (k_merge_seg counts them); lock_model = 0 counts them as locked
          const bool rlk = pos != 0xffffffffu && host_locked(d, pj);
          if (call) {
            const uint32_t q = hs.fifo_head - head0;
            const bool pf = q < n0 && q < (uint32_t)T;
            // a packet registered in a local inbox
            const bool filt = d.sfilt && pos != 0xffffffffu && !(rlk && d.p.lock_model);
            l = get_broadcasts_team<T>(d, a, u, hs, cap, pk, lim, d.p.overhead_bytes, pf ? &pjs[q] : nullptr,
                                       filt ? &d.view[(size_t)(pj - d.lo) * d.R] : nullptr, pj - d.lo);
          }
          if (rlk && l && lane == 0) {
            a.locked = true;
            if (d.p.lock_model) flag_live(d, pj - d.lo, l);  // routes the receiver (k_merge_seg)
            else a.c[C_LOCKED_MERGES] += l;
          }
          called = j + 1;
          if (lane == 0) kb += 16 + 32ull * l + (filt_used(d, pos) && !(rlk && d.p.lock_model) ? 8ull * l : 0);  // job, records in/out, slots
          const bool live = l || nf;
          if (lane == 0) {
            d.msg_len[x] = ok ? l : 0;
            if (fd && !ok) d.fd_len[x] = 0;
            lost += live && !ok;
            d.msg_dst[x] = pj;
            if (pos != 0xffffffffu) inbox_header(d, pj - d.lo, pos, u * d.KE + c, (uint32_t)x, l);
          }
          if (l == 0 && nf == 0) {
            stop = n == 0 && d.p.gossip_stop_on_empty;
            break;
          }
        }
      }
      // slots claimed for peers the round stopped before (gossip() returned at an empty packet)
      if (early && lane >= called && my_pos != 0xffffffffu)
        inbox_header(d, peers[lane] - d.lo, my_pos, u * d.KE + lane, (uint32_t)((size_t)idx * d.KE + lane), 0);
      hs.lock = lock_snap(hs.lock, hs.flags, d.round + 1, d.p.lock_readers != 0);  // the lock for the next round
      if (lane == 0) *h = hs;
    }
  }
}

// SCAN: the round's expiry scans run here instead of in k_scan: the block first streams the views
// of its hosts whose tick needs one (tick == 2; scan_view, block-wide, one view at a time), then
// sends. A host's scan and send touch no other host's state, so no block waits for another.
// OWN > 0: the owner ticks run here too (phases 0-3 in one launch, plain rounds without
// listeners): the block's hosts tick with the same 4-lane teams, OWN services per lane, then the
// block scans its queued views and sends. Nothing of one host's tick or send reads another host's
// state except the receivers' inbox counts, zeroed a round ahead (Dev::in_cnt_nx).
template <int T, bool X, bool SCAN = false, bool VEC = false, bool EV = false, int OWN = 0, bool PLAN = false>
__global__ __launch_bounds__(256) void k_send(Dev d, int do_bt) {
  __shared__ gx_job s_pj[256 / T][T * GX_JPF];  // FIFO head jobs of the block's hosts, loaded ahead
  // send_planned's chunk plans, then the team's peers (16 u32 = one PlanCall's 64 B)
  __shared__ PlanCall s_pl[PLAN ? 256 / T : 1][PLAN_CH + 1];
  __shared__ ScanLds sm;
  __shared__ uint32_t s_scan[256 / T], s_nscan;
  __shared__ gx_sleeper s_sl[OWN ? 256 * GX_JPF : 1];  // sleep-ring heads of the owner ticks
  Acc a;
  const uint32_t idx = blockIdx.x * (256 / T) + threadIdx.x / T;
  unsigned lost = 0;
  GX_KP(0);
  TickFwd fwd;
  fwd.peers = reinterpret_cast<uint32_t *>(&s_pl[PLAN ? threadIdx.x / T : 0][PLAN_CH]);
  if (PLAN && OWN == 0 && (threadIdx.x & (T - 1)) == 0 && idx < d.Hl) {  // the sends' peers (count in [16])
    uint32_t pr[16];
    const uint32_t np = sample_peers_h(d, peer_seed(d), d.lo + idx, pr);
    for (uint32_t k = 0; k < np; k++) fwd.peers[k] = pr[k];
    fwd.peers[16] = np;
  }
  if (PLAN) wave_sync();
  fwd.pj = s_pj[threadIdx.x / T];
  fwd.npf = 0;
  fwd.pf0 = 0;
  fwd.tick = 0;
  if (d.snap && blockIdx.x == 0 && threadIdx.x == 0)  // scan_probe_begin: tagged with the round
    *d.snap = ((uint64_t)(uint32_t)d.round << 32) | d.work_cnt[GX_WC_SCANS];
  if constexpr (OWN > 0) {
    if (threadIdx.x == 0) {
      s_nscan = 0;
      if (blockIdx.x == 0) {  // the next round's lists start empty
        *d.ovf_cnt_nx = 0;
        *d.wl_cnt_nx = 0;
      }
    }
    __syncthreads();
    const bool q = owner_tick<T, OWN, PLAN, T * GX_JPF>(d, a, idx, &s_sl[(threadIdx.x / T) * (T * GX_JPF)], fwd);
    if (q) s_scan[atomicAdd(&s_nscan, 1u)] = idx;  // lead lanes only
    GX_KP(1);
    __syncthreads();  // the block's ticks before its scans and sends read them
    GX_KP(2);
    for (uint32_t k = 0; k < s_nscan; k++) {
      const uint32_t oi = s_scan[k];
      scan_view<VEC, EV>(d, oi, &d.scan_list[(size_t)oi * d.L], d.L, &d.scan_cnt[oi], sm);
      __syncthreads();
    }
  } else if (SCAN && *d.wl_cnt) {  // block-uniform: a round with no scan anywhere skips the barriers
    if (threadIdx.x == 0) s_nscan = 0;
    __syncthreads();
    if ((threadIdx.x & (T - 1)) == 0 && idx < d.Hl && d.tick[idx] == 2) s_scan[atomicAdd(&s_nscan, 1u)] = idx;
    __syncthreads();
    for (uint32_t k = 0; k < s_nscan; k++) {
      const uint32_t oi = s_scan[k];
      scan_view<VEC, EV>(d, oi, &d.scan_list[(size_t)oi * d.L], d.L, &d.scan_cnt[oi], sm);
      __syncthreads();  // the list and count before the tick's finish reads them
    }
  }
  unsigned long long kb = 0, kl = 0;
  GX_KP(3);
  if (idx < d.Hl)  // (PLAN runs without departures: every host ticked)
    send_host<T, X, PLAN, PLAN && (OWN > 0)>(d, a, idx, s_pj[threadIdx.x / T], do_bt, lost,
                                            s_pl[PLAN ? threadIdx.x / T : 0], kb, kl, fwd);
  GX_KP(7);
  acc_flush(d, a);
  if (X && lost) ctr_atomic(d, C_LOST, lost);
  // algorithmic bytes: bookkeeping, FIFO jobs, records read (lists, ring), receiver slots read,
  // records and headers written (send_planned; the record-budget path counts the same per record)
  // units: the receiver view lines the senders' filter read (128 B each; send_planned only)
  kb = wave_sum(kb);
  kl = wave_sum(kl);
  if ((threadIdx.x & 63) == 0) kbytes(d, GX_K_SEND, kb, kl);
  if (PLAN && d.ob_buf) {  // the last block to finish: every region filled exactly, claims reset
    __shared__ uint32_t s_last;
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence();
      s_last = atomicAdd(&d.ob_claim[XPLAN_GMAX], 1u) == gridDim.x - 1u;
    }
    __syncthreads();
    if (s_last) {
      __threadfence();
      if (threadIdx.x < d.G && atomicExch(&d.ob_claim[threadIdx.x], 0u) != d.ob_cnt[threadIdx.x])
        atomicOr(&d.work_cnt[GX_WC_ERR], GX_ERR_INBOX);  // a slot left unwritten (cannot happen)
      if (threadIdx.x == 0) atomicExch(&d.ob_claim[XPLAN_GMAX], 0u);
    }
  }
}


// ================================================ memberlist probe traffic (gx.h probe_piggyback) ==
// memberlist's sendMsg piggybacks getBroadcasts on every UDP message (the absent fork; parity
// unpinned). With probe_piggyback, each host's probe ping (every fd_probe_rounds at its seeded
// phase, to its image under the round's keyed Feistel permutation) and its ack to the one host
// that may have pinged it (the permutation's preimage) are one GetBroadcasts call each, before
// the round's owner phase: packet entries KG (ping) and KG + 1 (ack), registered in the
// receivers' inboxes like send_host's packets (unplanned path: the receiver's filter at the
// sender, a locked receiver's records unfiltered to its pipeline). A team of T lanes per host.
GXD bool probe_tick_of(const Dev &d, uint32_t u) {
  const uint32_t P = d.p.fd_probe_rounds;
  return (uint64_t)d.round % P == rng4(d.p.seed, ST_FD_PHASE, u, 0, 0) % P;
}
template <int T>
__global__ __launch_bounds__(256) void k_probe(Dev d) {
  Acc a;
  const uint32_t idx = blockIdx.x * (256 / T) + threadIdx.x / T, lane = threadIdx.x & (T - 1);
  unsigned lost = 0;
  unsigned long long kb = 0;
  if (idx < d.Hl) {
    const uint32_t u = d.lo + idx, cap = d.p.packet_cap;
    gx_host_state *h = &d.hs[idx];
    gx_host_state hs = *h;
    const uint64_t key = rng4(d.p.seed, ST_PROBE, (uint64_t)d.round, 0, 0);
    for (uint32_t c = 0; c < 2; c++) {
      const size_t x = (size_t)idx * d.KE + d.KG + c;
      if (lane == 0) {
        d.msg_len[x] = 0;
        d.msg_key[x] = u * d.KE + d.KG + c;
      }
      if (departed(d, u)) continue;
      uint32_t peer;
      if (c == 0) {  // the ping: u's image, when u probes this round
        if (!probe_tick_of(d, u)) continue;
        peer = feistel_perm(key, u, d.H);
        if (peer == u) continue;
      } else {  // the ack: to the preimage, when its ping reached u
        peer = feistel_inv(key, u, d.H);
        if (peer == u || departed(d, peer) || !probe_tick_of(d, peer) || !reach(d, peer, u)) continue;
      }
      const bool ok = reach(d, u, peer), local = peer - d.lo < d.Hl;
      uint32_t pos = lane == 0 && ok && local ? inbox_claim(d, peer - d.lo) : 0xffffffffu;
      pos = (uint32_t)__shfl((int)pos, 0, T);
      uint32_t lim = d.p.limit_bytes;
      bool call = true;
      if (lim) {  // the ping or ack message takes its bytes first
        const uint32_t used = d.p.fd_msg_bytes + 2;
        lim = lim > used ? lim - used : 0;
        call = lim > d.p.overhead_bytes;
      }
      grec *pk = pos < d.DR ? &d.in_rec[((size_t)(peer - d.lo) * d.DR + pos) * cap] : &d.msg[x * cap];
      const bool rlk = pos != 0xffffffffu && host_locked(d, peer);
      const bool filt = d.sfilt && pos != 0xffffffffu && !(rlk && d.p.lock_model);
      uint32_t l = 0;
      if (call)
        l = get_broadcasts_team<T>(d, a, u, hs, cap, pk, lim, d.p.overhead_bytes, nullptr,
                                   filt ? &d.view[(size_t)(peer - d.lo) * d.R] : nullptr, peer - d.lo);
      if (rlk && l && lane == 0) {
        a.locked = true;
        if (d.p.lock_model) flag_live(d, peer - d.lo, l);
        else a.c[C_LOCKED_MERGES] += l;
      }
      if (lane == 0) {
        kb += 16 + 32ull * l + (filt ? 8ull * l : 0);
        d.msg_len[x] = ok ? l : 0;
        lost += l && !ok;
        d.msg_dst[x] = peer;
        if (pos != 0xffffffffu) inbox_header(d, peer - d.lo, pos, u * d.KE + d.KG + c, (uint32_t)x, l);
      }
    }
    if (lane == 0) *h = hs;
  }
  acc_flush(d, a);
  if (lost) ctr_atomic(d, C_LOST, lost);
  kb = wave_sum(kb);
  if ((threadIdx.x & 63) == 0) kbytes(d, GX_K_SEND, kb, 0);
}

// ============================================================== phase 4: gather-then-merge ==
// One wave per receiver. Its inbox (the packet headers the senders registered, in arrival order)
// is loaded together with its count; the few headers are ranked by global sender key in
// registers and staged sorted in LDS, so the fold order is the reference receiver's (ascending
// sender, then packet order). Each 64-record tile takes one record per lane straight from the
// senders' packets (one predicated load per packet overlapping the tile, all independent) and
// prefetches the tile's view slots as soon as the keys are known: three dependent global loads
// per receiver (inbox, records, view slots), no routing pass. Duplicate keys are grouped by an
// in-register bitonic sort of (key, arrival lane), and each group folds its occurrences in
// arrival order with the AddServiceEntry rule (one wave-uniform step per occurrence of the
// longest group, usually 1). The group's first lane writes the slot once. Accepted foreign
// records are compacted with a wave ballot into the receiver's FIFO (retransmit), in arrival
// order. A receiver with more than DI packets (overflow list) is folded by one lane walking its
// inbox in key order through the scalar AddServiceEntry path (add_entry): same semantics, slow.
template <bool K32>
GXD uint64_t bitonic64(uint64_t x, uint32_t lane) {  // ascending across the 64 lanes
#pragma unroll
  for (uint32_t k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      uint64_t o;
      if (K32) o = (uint32_t)__shfl_xor((uint32_t)x, (int)j, 64);
      else o = __shfl_xor(x, (int)j, 64);
      bool keep_min = ((lane & j) == 0) == ((lane & k) == 0);
      x = keep_min ? (o < x ? o : x) : (o > x ? o : x);
    }
  }
  return x;
}

GXD uint32_t rdl(uint32_t x, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, (int)l); }

// Overflowed inbox: one lane folds every packet in key order through the scalar path and
// flushes its own counters. The ServicesState lock (gx.h lock_model): a locked receiver appends the
// records to its pipeline instead; an unlocked one with nbuf queued records merges those first.
GXD void merge_inbox_serial(const Dev &d, uint32_t vi, bool lockd = false, uint32_t nbuf = 0) {
  Acc a;
  const uint32_t v = d.lo + vi, cnt = d.in_cnt[vi];
  int64_t after = -1;
  unsigned long long recs = 0;
  grec *lkb = d.lkb ? &d.lkb[(size_t)vi * d.C] : nullptr;
  if (lockd) {
    uint32_t nb = GX_LOCK_BUF(d.hs[vi].lock);
    const uint32_t capv = pipe_cap(d, vi, d.hs[vi].lock);  // a waiting merge holds places (lock_readers)
    for (uint32_t n = 0; n < cnt; n++) {
      const uint4 h = inbox_next(d, vi, after);
      after = h.x;
      const grec *pk = packet_recs(d, vi, h.w, h.y);
      for (uint32_t x = 0; x < h.z; x++) {
        if (nb < capv) {
          lkb[nb++] = pk[x];
          a.c[C_LOCK_BUF]++;
        } else {
          a.c[C_LOCK_DROP]++;
        }
      }
      recs += h.z;
    }
    d.hs[vi].lock = (d.hs[vi].lock & ((1u << GX_LOCK_BUF_SHIFT) - 1u)) | nb << GX_LOCK_BUF_SHIFT;
    kbytes(d, GX_K_MERGE, 32ull * recs + 16ull * cnt + 4, 0);
    for (int i = 0; i < C_NCTR; i++) ctr_atomic(d, i, a.c[i]);
    return;
  }
  for (uint32_t k = 0; k < nbuf; k++) add_entry(d, a, v, lkb[k], SRC_GOSSIP);  // the pipeline drains
  const unsigned m0 = a.c[C_GOSSIP_MERGES], s0 = a.c[C_STALE];
  if (nbuf) {
    a.c[C_LOCK_DRAIN] += nbuf;
    d.hs[vi].lock &= (1u << GX_LOCK_BUF_SHIFT) - 1u;
  }
  for (uint32_t n = 0; n < cnt; n++) {
    const uint4 h = inbox_next(d, vi, after);
    after = h.x;
    const grec *pk = packet_recs(d, vi, h.w, h.y);
    for (uint32_t x = 0; x < h.z; x++) add_entry(d, a, v, pk[x], SRC_GOSSIP);
    recs += h.z;
  }
  recs += nbuf;
  a.c[C_GOSSIP_MERGES] = m0;  // the packets' merges and stale drops: counted by the senders
  a.c[C_STALE] = s0;
  kbytes(d, GX_K_MERGE, 28ull * recs + 16ull * cnt + 4, recs);
  for (int i = 0; i < C_NCTR; i++) ctr_atomic(d, i, a.c[i]);
  if (a.changed) mark_change(d);
}

#define INBOX_PREFETCH 8
#define MERGE_WAVES 4
#define MSET 512  // merge_receiver's written-key set (power of two)
#define MSET_EMPTY 0xffffffffu
GXD uint32_t mset_slot(uint32_t key) { return (key * 0x9E3779B1u) >> (32 - 9); }
GXD bool mset_has(const uint32_t *set, uint32_t key) {
  for (uint32_t h = mset_slot(key), n = 0; n < MSET; n++, h = (h + 1) & (MSET - 1)) {
    const uint32_t x = set[h];
    if (x == key) return true;
    if (x == MSET_EMPTY) return false;
  }
  return false;
}
GXD void mset_add(uint32_t *set, uint32_t key) {
  for (uint32_t h = mset_slot(key), n = 0; n < MSET; n++, h = (h + 1) & (MSET - 1)) {
    const uint32_t x = atomicCAS(&set[h], MSET_EMPTY, key);
    if (x == MSET_EMPTY || x == key) return;
  }
}
struct MergeLds {  // one wave's staging for one receiver at a time
  uint4 hdr[GX_DI_MAX];     // headers in sender order (inboxes of more than 64 packets use all of it)
  uint32_t pst[GX_DI_MAX];  // wide inboxes: keys while ranking, then each packet's first record index
  uint64_t accw[64];
  uint32_t wset[MSET];  // keys written by earlier tiles of the receiver (merge_receiver)
  uint8_t accf[64], chg[64], prev[64];
};
// The full gather-then-merge of receiver vi by one wave (every lane calls it, wave-uniform vi).
template <bool K32, bool EV>
GXD void merge_receiver(const Dev &d, const uint32_t vi, MergeLds &L) {
  uint4 *s_hdr = L.hdr;
  uint8_t *s_accf = L.accf, *s_chg = L.chg, *s_prev = L.prev;
  uint64_t *s_accw = L.accw;
  const uint32_t lane = threadIdx.x & 63, v = d.lo + vi;
  // hop 1: the inbox count and its first headers together (most inboxes hold a few packets)
  const uint32_t npre = d.DI < INBOX_PREFETCH ? d.DI : INBOX_PREFETCH;
  uint4 hd = lane < npre ? d.in_hdr[(size_t)vi * d.DI + lane] : make_uint4(0u, 0u, 0u, 0u);
  const uint32_t deg = d.in_cnt[vi];
  // the ServicesState lock (gx.h lock_model): a locked receiver appends its records to its pipeline
  // (lkb) instead of merging them; an unlocked one with nbuf records queued there merges those
  // first, as the first nbuf records of its fold
  uint32_t lw = 0, nbuf = 0;
  bool lockd = false;
  if (d.p.lock_model) {
    lw = __builtin_amdgcn_readfirstlane(d.hs[vi].lock);
    lockd = locked_in(d, lw);
    nbuf = lockd || departed(d, v) ? 0u : GX_LOCK_BUF(lw);
  }
  if (deg == 0 && nbuf == 0) return;
  if (deg > d.DI) {
    if (lane == 0) merge_inbox_serial(d, vi, lockd, nbuf);
    return;
  }
  // wide inbox (more than 64 packets, GossipMessages > 1): the headers are ranked and staged in
  // LDS, with each packet's first record index beside them; the fold below reads both from there
  const bool wide = deg > 64;
  uint4 sh = make_uint4(0u, 0u, 0u, 0u);  // {key, entry, len, slot} of packet `lane` (deg <= 64)
  uint32_t pstart = 0, total = 0;
  if (!wide) {
    if (deg > npre && lane >= npre && lane < deg) hd = d.in_hdr[(size_t)vi * d.DI + lane];
    // sender order: rank of each header's key among the deg distinct keys
    const uint32_t hkey = lane < deg ? hd.x : 0xffffffffu;
    uint32_t hrank = 0;  // ties (refused by k_inbox_unpack) broken by lane: every rank is written once
    for (uint32_t j = 0; j < deg; j++) hrank += rdl(hkey, j) < hkey || (rdl(hkey, j) == hkey && j < lane);
    if (lane < deg) s_hdr[hrank] = hd;
    wave_sync();
    sh = lane < deg ? s_hdr[lane] : make_uint4(0u, 0u, 0u, 0u);
    uint32_t incl = sh.z;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      uint32_t y = __shfl_up(incl, o, 64);
      if ((int)lane >= o) incl += y;
    }
    pstart = incl - sh.z;
    total = __shfl(incl, 63, 64);
  } else {
    constexpr int HPL = GX_DI_MAX / 64;  // headers per lane
    uint4 hw[HPL];
#pragma unroll
    for (int c = 0; c < HPL; c++) {  // every header in one round trip
      const uint32_t j = lane + 64u * c;
      hw[c] = j < deg ? (j < npre ? hd : d.in_hdr[(size_t)vi * d.DI + j]) : make_uint4(0u, 0u, 0u, 0u);
      if (j < deg) L.pst[j] = hw[c].x;
    }
    wave_sync();
    uint32_t rk[HPL];
#pragma unroll
    for (int c = 0; c < HPL; c++) rk[c] = 0;
    for (uint32_t j = 0; j < deg; j++) {  // rank by key, ties by arrival index (broadcast LDS reads)
      const uint32_t kj = L.pst[j];
#pragma unroll
      for (int c = 0; c < HPL; c++) {
        const uint32_t me = lane + 64u * c;
        rk[c] += kj < hw[c].x || (kj == hw[c].x && j < me);
      }
    }
#pragma unroll
    for (int c = 0; c < HPL; c++)
      if (lane + 64u * c < deg) s_hdr[rk[c]] = hw[c];
    wave_sync();
    for (uint32_t c0 = 0; c0 < deg; c0 += 64) {  // first record index of every packet, in sender order
      const uint32_t j = c0 + lane;
      const uint32_t ln = j < deg ? s_hdr[j].z : 0u;
      uint32_t incl = ln;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(incl, o, 64);
        if ((int)lane >= o) incl += y;
      }
      if (j < deg) L.pst[j] = total + incl - ln;
      total += __shfl(incl, 63, 64);
    }
    wave_sync();
  }
  const uint32_t vtick = d.tick[vi];
  gx_host_state *h = &d.hs[vi];
  const uint32_t tail0 = h->fifo_tail, st0 = h->fifo_stored, room = fifo_room(d, h->fifo_head, tail0, st0);
  uint32_t n_retx = 0, n_ev = 0;
  uint32_t c_merge = 0, c_acc = 0, c_stale = 0, c_rd = 0, c_wr = 0, c_chg = 0;  // per lane: < 2^32
  unsigned long long mexp = ~0ull;
  uint64_t *row = &d.view[(size_t)vi * d.R];
  const uint32_t INV = K32 ? 0x3ffffffu : 0xffffffffu;  // sorts after every real key
  const int32_t evk = d.ev_slot[vi];
  const uint32_t ev0 = evk >= 0 ? d.ev_cnt[evk] : 0;
  int64_t vlc_ts = 0;
  bool vlc_set = false;
  // Records are prefetched a tile ahead (tile t + 1's while tile t is folded). Each record's slot
  // word at the start of the merge came with it (msg_w0, read by its sender) wherever nothing can
  // have changed the slot since (w0_fwd: not an own record, the view not scanned this round), so
  // the receiver reads the slot itself only for the other records and for keys an earlier tile of
  // this receiver wrote: an LDS set of the written keys (open addressing; once it holds more than
  // MSET / 2 keys, every later record reads its slot).
  // Record i's packet: the last with start <= i (a binary search of the sender-ordered starts in
  // LDS), so a tile's records are one load per lane (and one of its msg_w0 word), whatever the
  // packets' lengths: a fixed count of loads in flight, which the waits below can count past.
  if (!wide) {
    if (lane < deg) L.pst[lane] = pstart;
    wave_sync();
  }
  const grec *lkb = nbuf ? &d.lkb[(size_t)vi * d.C] : nullptr;
  const uint32_t ntot = nbuf + total;  // the fold: the drained pipeline, then the packets
  auto load_recs = [&](uint32_t tb, grec &g, uint32_t &fslot, uint64_t &fw0) {
    uint32_t i = tb + lane;
    g.w = 0;
    g.r = INV;
    g.pad = 0;
    fw0 = 0;
    fslot = 0;
    if (i < nbuf) {  // a queued record reads its slot (fslot 0: no forwarded word)
      g = gld_rec(&lkb[i]);
      return;
    }
    i -= nbuf;
    if (i < total) {  // hop 2
      uint32_t lo = 0, hi = deg;
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (L.pst[mid] <= i) lo = mid;
        else hi = mid;
      }
      const uint4 hk = s_hdr[lo];  // {key, entry, len, slot}
      const uint32_t off = i - L.pst[lo];
      fslot = hk.w;
      g = packet_recs(d, vi, hk.w, hk.y)[off];
      if (hk.w == GX_NOSLOT_W0) fw0 = d.msg_w0[(size_t)hk.y * d.p.packet_cap + off];
    }
  };
  if (lockd) {  // the pipeline takes the records in arrival order while it has room (gx.h lock_model)
    const uint32_t capv = pipe_cap(d, vi, lw), nb0 = GX_LOCK_BUF(lw), room_l = capv > nb0 ? capv - nb0 : 0u;
    const uint32_t keep = total < room_l ? total : room_l;
    grec *dst = &d.lkb[(size_t)vi * d.C + nb0];
    for (uint32_t t0 = 0; t0 < keep; t0 += 64) {
      grec g;
      uint32_t fs;
      uint64_t fw;
      load_recs(t0, g, fs, fw);
      if (t0 + lane < keep) gst_rec(&dst[t0 + lane], g);
    }
    if (lane == 0) {
      d.hs[vi].lock = (lw & ((1u << GX_LOCK_BUF_SHIFT) - 1u)) | (nb0 + keep) << GX_LOCK_BUF_SHIFT;
      ctr_atomic(d, C_LOCK_BUF, keep);
      ctr_atomic(d, C_LOCK_DROP, total - keep);
      kbytes(d, GX_K_MERGE, 32ull * keep + 16ull * deg + 4, 0);  // records in and out, headers
    }
    wave_sync();
    return;
  }
  const bool track = ntot > 64;  // wave-uniform: later tiles consult the written-key set
  if (track)
    for (uint32_t q = lane; q < MSET; q += 64) L.wset[q] = MSET_EMPTY;
  uint32_t nset = 0;  // keys in the set (wave-uniform)
  grec gc, gn;
  uint32_t fsc, fsn = 0;
  uint64_t fwc, fwn = 0;
  load_recs(0, gc, fsc, fwc);
  gn.w = 0;
  gn.r = INV;
  gn.pad = 0;
  if (64 < ntot) load_recs(64, gn, fsn, fwn);
  wave_sync();
  unsigned long long *kpm = kprof_merge(d);  // diagnostics: phase cycles of the whole-wave tiles
  unsigned long long ph[5] = {0, 0, 0, 0, 0}, tk = 0;
  uint32_t c_dstale = 0;  // stale drops among the drained records (the packets' counted by the senders)
  for (uint32_t t0 = 0; t0 < ntot; t0 += 64) {
    if (kpm) tk = __builtin_amdgcn_s_memtime();
    const uint32_t i = t0 + lane;
    const bool valid = i < ntot;
    uint32_t key = INV;
    uint64_t val = 0, w0 = 0;
    bool rd = false;  // this record reads its slot (hop 3)
    if (valid) {
      key = gc.r;
      val = gc.w;
      bool fwd = w0_fwd(d, fsc, vtick, key, v);
      if (fwd && t0 > 0) fwd = nset <= MSET / 2 && !mset_has(L.wset, key);
      rd = !fwd;
      w0 = fwd ? fwc : row[key];
    }
    // the tile after next's records, issued after this tile's slot reads so that waiting for
    // those leaves them in flight
    grec gnn;
    uint32_t fsnn = 0;
    uint64_t fwnn = 0;
    gnn.w = 0;
    gnn.r = INV;
    gnn.pad = 0;
    if (t0 + 128 < ntot) load_recs(t0 + 128, gnn, fsnn, fwnn);
    c_merge += valid;
    c_rd += rd;  // view slots read by the receiver
    // A record that is stale, or no newer than the slot's word at the start of the tile, is a
    // no-op whatever its position in the fold: the slot's timestamp only grows (an accept needs a
    // strictly newer one, services_state.go:321), and IsStale does not depend on the slot. Only the
    // other records ("live") enter the fold; a tile without any (every copy of an epidemic
    // broadcast after the first) is done here.
    const bool stale0 = valid && ts_of(val) < d.now - d.p.tombstone_lifespan_ns - d.p.stale_fudge_ns;
    const bool live = valid && !stale0 && (st_of(w0) == GX_ABSENT || ts_of(val) > ts_of(w0));
    c_stale += stale0;
    c_dstale += stale0 && i < nbuf;
    const bool any_live = __ballot(live) != 0;
    if (kpm) {  // [8] records and slots in (waits), [9] sort, [10] fold + writes, [11] the rest, [12] tiles
      const unsigned long long x = __builtin_amdgcn_s_memtime();
      ph[0] += x - tk;
      tk = x;
      ph[4]++;
    }
    if (any_live) {  // wave-uniform
    if (!live) key = INV;
    uint64_t sk = K32 ? (uint64_t)((key << 6) | lane) : (((uint64_t)key << 6) | lane);
    sk = bitonic64<K32>(sk, lane);
    if (kpm) {
      const unsigned long long x = __builtin_amdgcn_s_memtime() + (sk & 0);
      ph[1] += x - tk;
      tk = x;
    }
    const uint32_t src = (uint32_t)(sk & 63), skey = (uint32_t)(sk >> 6);
    const bool vs = skey != INV;
    const uint64_t sval = __shfl(val, (int)src, 64), sw0 = __shfl(w0, (int)src, 64);
    uint32_t pkey = __shfl_up(skey, 1, 64);
    const bool head = vs && (lane == 0 || pkey != skey);
    const uint64_t heads = __ballot(head);
    const uint64_t le = lane == 63 ? ~0ull : ((2ull << lane) - 1);
    const uint32_t gs = 63 - (uint32_t)__clzll((heads & le) | 1ull);  // first lane of this group
    const uint32_t kpos = lane - gs;
    const uint64_t after = heads & ~le;
    const uint32_t nvs = (uint32_t)__popcll(__ballot(vs));
    const uint32_t glen = (after ? (uint32_t)__ffsll((long long)after) - 1 : nvs) - lane;  // heads only
    uint32_t kmax = vs ? kpos : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      uint32_t y = __shfl_xor(kmax, o, 64);
      kmax = y > kmax ? y : kmax;
    }
    uint64_t wg = sw0, wme = 0, wprev = GX_SLOT_ABSENT;
    bool acc = false, stl = false;
    for (uint32_t kk = 0; kk <= kmax; kk++) {  // occurrence kk of every group, arrival order
      uint64_t wcur = __shfl(wg, (int)gs, 64);
      if (vs && kpos == kk) {
        wprev = wcur;
        wme = merge_word(d, wcur, sval, acc, stl);
      }
      uint64_t wn = __shfl(wme, (int)((gs + kk) & 63), 64);
      if (head && kk < glen) wg = wn;
    }
    c_stale += stl;
    c_acc += acc;
    const bool wrote = head && wg != sw0;
    if (wrote) {
      row[skey] = wg;
      c_wr++;
      unsigned long long x = exp_time(d.p, wg);
      mexp = x < mexp ? x : mexp;
    }
    if (track && nset <= MSET / 2) {  // later tiles read these keys' slots (at most MSET / 2 + 64 held)
      if (wrote) mset_add(L.wset, skey);
      nset += (uint32_t)__popcll(__ballot(wrote));
    }
    if (kpm) {
      const unsigned long long x = __builtin_amdgcn_s_memtime() + (wg & 0);
      ph[2] += x - tk;
      tk = x;
    }
    // ServiceChanged: an insert, or a stored status that differs (:317-340)
    const bool chg = acc && (st_of(wprev) == GX_ABSENT || st_of(wprev) != st_of(wme));
    c_chg += chg;
    s_accf[src] = vs && acc && !owned_by(d, skey, v);
    if (EV) {
      s_chg[src] = chg;
      s_prev[src] = (uint8_t)(st_of(wprev) == GX_ABSENT ? GX_UNKNOWN : st_of(wprev));
    }
    s_accw[src] = wme;
    // per owner (contiguous in key order): its last accepted and last status-changing
    // occurrence in arrival order (segmented max of arrival lane + 1)
    const uint32_t own = vs ? owner_of(d, skey) : 0xffffffffu;
    uint32_t mu = acc ? src + 1 : 0, mc = chg ? src + 1 : 0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      uint32_t yu = __shfl_down(mu, o, 64), yc = __shfl_down(mc, o, 64), yo = __shfl_down(own, o, 64);
      if (lane + o < 64 && yo == own) {
        mu = yu > mu ? yu : mu;
        mc = yc > mc ? yc : mc;
      }
    }
    uint32_t pown = __shfl_up(own, 1, 64);
    const bool ohead = vs && (lane == 0 || pown != own);
    uint32_t mcmax = mc;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      uint32_t y = __shfl_xor(mcmax, o, 64);
      mcmax = y > mcmax ? y : mcmax;
    }
    __threadfence_block();  // slot stores land before a later tile reads the same keys
    wave_sync();
    if (ohead && (mu || mc)) {
      gx_server_times *st = srv_times(d, v, own);
      if (mu) st->last_updated_ns = ts_of(s_accw[mu - 1]);  // server.LastUpdated (:323)
      if (mc) st->last_changed_ns = ts_of(s_accw[mc - 1]);  // serverChanged (:204-215)
      c_wr += (mu != 0) + (mc != 0);                        // counted as written words
    }
    if (mcmax) {
      vlc_ts = ts_of(s_accw[mcmax - 1]);  // state.LastChanged
      vlc_set = true;
    }
    if (EV && evk >= 0) {  // ChangeEvents in arrival order
      bool fe = s_chg[lane] != 0;
      unsigned long long me = __ballot(fe);
      if (fe)
        ev_put(d, evk, ev0 + n_ev + (uint32_t)__popcll(me & ((1ull << lane) - 1ull)), key, s_accw[lane],
               s_prev[lane]);
      n_ev += (uint32_t)__popcll(me);
    }
    bool f = s_accf[lane];  // ordered ballot compaction -> retransmit jobs (arrival order)
    unsigned long long m = __ballot(f);
    uint32_t pos = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    if (f && n_retx + pos < room)
      d.fifo[(size_t)vi * d.Q + ((tail0 + n_retx + pos) % d.Q)] = make_job(s_accw[lane], key, meta_of(GX_JOB_RETX, 0, 1));
    n_retx += (uint32_t)__popcll(m);
    wave_sync();
    }  // live records in the tile
    if (kpm) ph[3] += __builtin_amdgcn_s_memtime() - tk;
    gc = gn;
    fsc = fsn;
    fwc = fwn;
    gn = gnn;
    fsn = fsnn;
    fwn = fwnn;
  }
  if (kpm && lane == 0)
    for (int q = 0; q < 5; q++) atomicAdd(&kpm[8 + q], ph[q]);
  const unsigned long long m_merge = wave_sum(c_merge), m_acc = wave_sum(c_acc), m_rd = wave_sum(c_rd),
                           m_wr = wave_sum(c_wr), m_chg = wave_sum(c_chg);
  if (nbuf) {
    const unsigned long long m_ds = wave_sum(c_dstale);
    if (lane == 0) ctr_atomic(d, C_STALE, m_ds);
  }
  (void)c_stale;  // stale drops: counted by the senders
  mexp = wave_min(mexp);
  if (lane == 0) {
    const uint32_t ok = n_retx < room ? n_retx : room;  // stored; the rest deferred (gx.h gx_job)
    if (n_retx) {
      h->fifo_tail = tail0 + n_retx;
      h->fifo_stored = st0 + ok;
    }
    if (vlc_set) d.vlc[vi] = vlc_ts;
    if (evk >= 0) d.ev_cnt[evk] = ev0 + n_ev;
    ctr_atomic(d, C_CHG, m_chg);
    if (nbuf) {  // the drained pipeline: AddServiceEntry calls of this round
      d.hs[vi].lock = lw & ((1u << GX_LOCK_BUF_SHIFT) - 1u);
      ctr_atomic(d, C_GOSSIP_MERGES, nbuf);
      ctr_atomic(d, C_LOCK_DRAIN, nbuf);
    }
    // 12 B per record (word + key) + 8 B per slot read / written + 16 B per stored retransmit job
    // + 16 B per inbox header + the count (merges and stale drops: counted by the senders)
    kbytes(d, GX_K_MERGE, 12ull * m_merge + 8ull * (m_rd + m_wr) + 16ull * ok + 16ull * deg + 4, m_merge);
    ctr_atomic(d, C_GOSSIP_ACC, m_acc);
    ctr_atomic(d, C_RETX, n_retx);
    ctr_atomic(d, C_QDEFER, n_retx - ok);
    if (m_wr) {
      mark_change(d);
      atomicMin(&d.minexp[vi], mexp);
    }
  }
  wave_sync();
}

// The same merge for receivers whose live records fit one segment of SEG lanes (64 / SEG
// receivers per wave): their inbox (deg <= SEG headers, within DI) holds at most SEG records, which
// is one tile. Every step of merge_receiver runs within the segment: header ranking and the
// packet scan by segment shuffles, one record per lane, the bitonic sort of (key, arrival lane)
// over SEG lanes, the per-group fold in arrival order, the per-owner server times, the ordered
// ballot compaction of retransmits and ChangeEvents on the segment's ballot bits. Returns false
// (nothing done) for a receiver that does not fit: the caller merges it with the whole wave.
template <int SEG>
GXD uint32_t seg_sum(uint32_t x) {
#pragma unroll
  for (int o = SEG / 2; o > 0; o >>= 1) x += __shfl_xor(x, o, SEG);
  return x;
}
template <int SEG>
GXD uint32_t seg_max(uint32_t x) {
#pragma unroll
  for (int o = SEG / 2; o > 0; o >>= 1) {
    const uint32_t y = __shfl_xor(x, o, SEG);
    x = y > x ? y : x;
  }
  return x;
}
template <bool K32, bool EV, int SEG>
GXD bool merge_seg(const Dev &d, const uint32_t vi, const bool act, MergeLds &L) {
  const uint32_t lane = threadIdx.x & 63, sl = lane & (SEG - 1), sb = lane - sl;
  const uint64_t smask = SEG == 64 ? ~0ull : ((1ull << SEG) - 1ull);
  auto sballot = [&](bool p) -> uint64_t { return (__ballot(p) >> sb) & smask; };
  const uint32_t v = d.lo + vi;
  // hop 1: count, headers, FIFO counters and the event log slot together
  uint4 hd = make_uint4(0u, 0u, 0u, 0u);
  uint32_t deg = 0, tail0 = 0, head0 = 0, st0 = 0;
  int32_t evk = -1;
  uint32_t vtick = 2;
  if (act) {
    if (sl < d.DI) hd = d.in_hdr[(size_t)vi * d.DI + sl];
    deg = d.in_cnt[vi];
    tail0 = d.hs[vi].fifo_tail;
    head0 = d.hs[vi].fifo_head;
    st0 = d.hs[vi].fifo_stored;
    vtick = d.tick[vi];
    if (EV) evk = d.ev_slot[vi];
  }
  const uint32_t len = sl < deg ? hd.z : 0u;
  const uint32_t total = seg_sum<SEG>(len);
  const bool fits = !act || (deg <= d.DI && deg <= (uint32_t)SEG && total <= (uint32_t)SEG);
  if (sballot(!fits)) return false;  // the segment's receiver takes the full path
  if (!act || deg == 0) return true;
  // sender order: rank of each header's key among the segment's deg keys (ties by lane)
  const uint32_t hkey = sl < deg ? hd.x : 0xffffffffu;
  uint32_t hrank = 0;
  for (uint32_t j = 0; j < deg; j++) {
    const uint32_t kj = (uint32_t)__shfl((int)hkey, (int)j, SEG);
    hrank += kj < hkey || (kj == hkey && j < sl);
  }
  uint4 *s_hdr = &L.hdr[sb];
  if (sl < deg) s_hdr[hrank] = hd;
  wave_sync();
  const uint4 sh = sl < deg ? s_hdr[sl] : make_uint4(0u, 0u, 0u, 0u);  // packet sl in sender order
  uint32_t incl = sh.z;
#pragma unroll
  for (int o = 1; o < SEG; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o, SEG);
    if ((int)sl >= o) incl += y;
  }
  const uint32_t pstart = incl - sh.z;
  // record sl: packet k with pstart_k <= sl < pstart_k + len_k
  const bool valid = sl < total;
  uint32_t kp = 0;
  for (uint32_t j = 1; j < deg; j++) kp += sl >= (uint32_t)__shfl((int)pstart, (int)j, SEG) ? 1u : 0u;
  const uint32_t ps = (uint32_t)__shfl((int)pstart, (int)kp, SEG);
  const uint32_t pe = (uint32_t)__shfl((int)sh.y, (int)kp, SEG), pw = (uint32_t)__shfl((int)sh.w, (int)kp, SEG);
  const uint32_t INV = K32 ? 0x3ffffffu : 0xffffffffu;  // sorts after every real key
  uint32_t key = INV;
  uint64_t val = 0, w0 = 0;
  uint64_t *row = &d.view[(size_t)vi * d.R];
  if (valid) {  // hop 2 (the record and the slot word its sender read), hop 3 only where that can be stale
    const grec g = gld_rec(&packet_recs(d, vi, pw, pe)[sl - ps]);
    const uint64_t fw0 = pw == GX_NOSLOT_W0 ? gld(&d.msg_w0[(size_t)pe * d.p.packet_cap + (sl - ps)]) : 0ull;
    key = g.r;
    val = g.w;
    w0 = w0_fwd(d, pw, vtick, key, v) ? fw0 : row[key];
  }
  const uint32_t room = fifo_room(d, head0, tail0, st0);
  const uint32_t ev0 = (EV && evk >= 0) ? d.ev_cnt[evk] : 0;
  const bool stale0 = valid && ts_of(val) < d.now - d.p.tombstone_lifespan_ns - d.p.stale_fudge_ns;
  const bool live = valid && !stale0 && (st_of(w0) == GX_ABSENT || ts_of(val) > ts_of(w0));
  unsigned long long c_wr = 0, mexp = ~0ull;
  uint32_t c_acc = 0, c_chg = 0, n_retx = 0;
  if (!live) key = INV;
  uint64_t sk = K32 ? (uint64_t)((key << 6) | sl) : (((uint64_t)key << 6) | sl);
#pragma unroll
  for (uint32_t k = 2; k <= (uint32_t)SEG; k <<= 1) {  // bitonic sort over the segment
#pragma unroll
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      uint64_t o;
      if (K32) o = (uint32_t)__shfl_xor((uint32_t)sk, (int)j, SEG);
      else o = __shfl_xor(sk, (int)j, SEG);
      const bool keep_min = ((sl & j) == 0) == ((sl & k) == 0);
      sk = keep_min ? (o < sk ? o : sk) : (o > sk ? o : sk);
    }
  }
  const uint32_t src = (uint32_t)(sk & 63), skey = (uint32_t)(sk >> 6);
  const bool vs = skey != INV;
  const uint64_t sval = __shfl(val, (int)src, SEG), sw0 = __shfl(w0, (int)src, SEG);
  const uint32_t pkey = __shfl_up(skey, 1, SEG);
  const bool head = vs && (sl == 0 || pkey != skey);
  const uint64_t heads = sballot(head);
  const uint64_t le = sl == 63 ? ~0ull : ((2ull << sl) - 1);
  const uint32_t gs = 63 - (uint32_t)__clzll((heads & le) | 1ull);  // first lane of this group
  const uint32_t kpos = sl - gs;
  const uint64_t after = heads & ~le;
  const uint32_t nvs = (uint32_t)__popcll(sballot(vs));
  const uint32_t glen = (after ? (uint32_t)__ffsll((long long)after) - 1 : nvs) - sl;  // heads only
  const uint32_t kmax = seg_max<SEG>(vs ? kpos : 0);
  uint64_t wg = sw0, wme = 0, wprev = GX_SLOT_ABSENT;
  bool acc = false, stl = false;
  for (uint32_t kk = 0; kk <= kmax; kk++) {  // occurrence kk of every group, arrival order
    const uint64_t wcur = __shfl(wg, (int)gs, SEG);
    if (vs && kpos == kk) {
      wprev = wcur;
      wme = merge_word(d, wcur, sval, acc, stl);
    }
    const uint64_t wn = __shfl(wme, (int)((gs + kk) & (SEG - 1)), SEG);
    if (head && kk < glen) wg = wn;
  }
  c_acc += acc;
  if (head && wg != sw0) {
    row[skey] = wg;
    c_wr++;
    const unsigned long long x = exp_time(d.p, wg);
    mexp = x < mexp ? x : mexp;
  }
  // ServiceChanged: an insert, or a stored status that differs (:317-340)
  const bool chg = acc && (st_of(wprev) == GX_ABSENT || st_of(wprev) != st_of(wme));
  c_chg += chg;
  uint8_t *s_accf = &L.accf[sb], *s_chg = &L.chg[sb], *s_prev = &L.prev[sb];
  uint64_t *s_accw = &L.accw[sb];
  s_accf[src] = vs && acc && !owned_by(d, skey, v);
  if (EV) {
    s_chg[src] = chg;
    s_prev[src] = (uint8_t)(st_of(wprev) == GX_ABSENT ? GX_UNKNOWN : st_of(wprev));
  }
  s_accw[src] = wme;
  // per owner (contiguous in key order): its last accepted and last status-changing occurrence
  const uint32_t own = vs ? owner_of(d, skey) : 0xffffffffu;
  uint32_t mu = acc ? src + 1 : 0, mc = chg ? src + 1 : 0;
#pragma unroll
  for (int o = 1; o < SEG; o <<= 1) {
    const uint32_t yu = __shfl_down(mu, o, SEG), yc = __shfl_down(mc, o, SEG), yo = __shfl_down(own, o, SEG);
    if (sl + o < (uint32_t)SEG && yo == own) {
      mu = yu > mu ? yu : mu;
      mc = yc > mc ? yc : mc;
    }
  }
  const uint32_t pown = __shfl_up(own, 1, SEG);
  const bool ohead = vs && (sl == 0 || pown != own);
  const uint32_t mcmax = seg_max<SEG>(mc);
  __threadfence_block();
  wave_sync();
  if (ohead && (mu || mc)) {
    gx_server_times *st = srv_times(d, v, own);
    if (mu) st->last_updated_ns = ts_of(s_accw[mu - 1]);  // server.LastUpdated (:323)
    if (mc) st->last_changed_ns = ts_of(s_accw[mc - 1]);  // serverChanged (:204-215)
    c_wr += (mu != 0) + (mc != 0);
  }
  uint32_t n_ev = 0;
  if (EV && evk >= 0) {  // ChangeEvents in arrival order
    const bool fe = s_chg[sl] != 0;
    const uint64_t me = sballot(fe);
    if (fe) ev_put(d, evk, ev0 + (uint32_t)__popcll(me & ((1ull << sl) - 1ull)), key, s_accw[sl], s_prev[sl]);
    n_ev = (uint32_t)__popcll(me);
  }
  const bool f = s_accf[sl];  // ordered ballot compaction -> retransmit jobs (arrival order)
  const uint64_t m = sballot(f);
  const uint32_t pos = (uint32_t)__popcll(m & ((1ull << sl) - 1ull));
  if (f && pos < room) d.fifo[(size_t)vi * d.Q + ((tail0 + pos) % d.Q)] = make_job(s_accw[sl], key, meta_of(GX_JOB_RETX, 0, 1));
  n_retx = (uint32_t)__popcll(m);
  c_wr = seg_sum<SEG>((uint32_t)c_wr);
  c_acc = seg_sum<SEG>(c_acc);
  c_chg = seg_sum<SEG>(c_chg);
#pragma unroll
  for (int o = SEG / 2; o > 0; o >>= 1) {
    const unsigned long long y = __shfl_xor(mexp, o, SEG);
    mexp = y < mexp ? y : mexp;
  }
  if (sl == 0) {
    const uint32_t ok = n_retx < room ? n_retx : room;  // stored; the rest deferred (gx.h gx_job)
    if (n_retx) {
      d.hs[vi].fifo_tail = tail0 + n_retx;
      d.hs[vi].fifo_stored = st0 + ok;
    }
    if (mcmax) d.vlc[vi] = ts_of(s_accw[mcmax - 1]);  // state.LastChanged
    if (EV && evk >= 0) d.ev_cnt[evk] = ev0 + n_ev;
    ctr_atomic(d, C_CHG, c_chg);
    // 12 B per record + 8 B per slot read / written + 16 B per stored retransmit + 16 B per header
    // + count (merges and stale drops: counted by the senders)
    kbytes(d, GX_K_MERGE, 12ull * total + 8ull * (total + c_wr) + 16ull * ok + 16ull * deg + 4, total);
    ctr_atomic(d, C_GOSSIP_ACC, c_acc);
    ctr_atomic(d, C_RETX, n_retx);
    ctr_atomic(d, C_QDEFER, n_retx - ok);
    if (c_wr) {
      mark_change(d);
      atomicMin(&d.minexp[vi], mexp);
    }
  }
  wave_sync();
  return true;
}

// Phase 4 for the receivers with live records (mrec: the live records the senders registered for
// each, a routing hint). A block takes MERGE_NR consecutive receivers and routes the ones with a
// count to work items by it: one receiver with more than 32 live records per item (a whole wave,
// merge_receiver), two of 17..32 (32-lane segments) or four of up to 16 (16-lane segments,
// merge_seg). The items go to the block's waves in turn, so the large inboxes of a block are folded
// side by side, not one after another by one wave. A receiver whose inbox does not fit its segment
// after all (more packets than lanes, or a count that overstates nothing) is merged by a whole wave
// at the end.
#ifndef MERGE_WPE_GM
#define MERGE_WPE_GM 4  // waves per SIMD of the merge at GossipMessages > 1 (wide inboxes)
#endif
// A locked receiver's round (gx.h lock_model): its packets' records join its pipeline in arrival
// order (ascending sender key) while it has room, the rest are dropped; nothing merges. SEG lanes
// per receiver (four receivers per wave at SEG 16): the segment ranks the headers by key in
// registers, finds each output record's packet by the ranked starts, and issues every record
// load of a pass (RPL per lane) before its stores. Returns false (the caller takes the
// whole-wave path) for an inbox of more than SEG packets; the result is the whole-wave path's.
#ifndef LOCK_RPL
#define LOCK_RPL 4  // 8 measured 13% slower in the buffering rounds (profiles/r05/ab/lock_rpl8_cfg5.jsonl)
#endif
template <int SEG>
GXD bool lock_append_seg(const Dev &d, uint32_t vi, bool act) {
  const uint32_t lane = threadIdx.x & 63, sl = lane & (SEG - 1), sb = lane & ~(uint32_t)(SEG - 1);
  // the count, the lock word and the first SEG header slots in one round trip (slots past the
  // count hold stale headers and are masked below)
  const uint32_t deg = act ? d.in_cnt[vi] : 0u;
  const uint32_t lw = act ? d.hs[vi].lock : 0u;
  uint4 hd = d.in_hdr[(size_t)vi * d.DI + (sl < d.DI ? sl : 0u)];
  if (deg > (uint32_t)SEG || deg > d.DI) return false;  // segment-uniform
  if (sl >= deg) hd = make_uint4(0xffffffffu, 0u, 0u, 0u);
  uint32_t start = 0, total = 0;
  for (uint32_t j = 0; j < (uint32_t)SEG; j++) {  // first record of this lane's packet in sender order
    const uint32_t kj = (uint32_t)__shfl((int)hd.x, (int)(sb + j), 64);
    const uint32_t lj = (uint32_t)__shfl((int)hd.z, (int)(sb + j), 64);
    const bool before = j < deg && (kj < hd.x || (kj == hd.x && j < sl));
    start += before ? lj : 0u;
    total += j < deg ? lj : 0u;
  }
  const uint32_t capv = pipe_cap(d, vi, lw), nb0 = GX_LOCK_BUF(lw), room = capv > nb0 ? capv - nb0 : 0u;
  const uint32_t keep = total < room ? total : room;
  grec *dst = act ? &d.lkb[(size_t)vi * d.C + nb0] : d.lkb;
  for (uint32_t o0 = 0; o0 < keep; o0 += SEG * LOCK_RPL) {
    grec g[LOCK_RPL];
#pragma unroll
    for (int q = 0; q < LOCK_RPL; q++) {  // output record o: the packet whose [start, start + len) holds it
      const uint32_t o = o0 + sl + SEG * q;
      uint32_t entry = 0, slot = 0, off = 0;
      for (uint32_t j = 0; j < deg; j++) {
        const uint32_t sj = (uint32_t)__shfl((int)start, (int)(sb + j), 64);
        const uint32_t lj = (uint32_t)__shfl((int)hd.z, (int)(sb + j), 64);
        const uint32_t ej = (uint32_t)__shfl((int)hd.y, (int)(sb + j), 64);
        const uint32_t wj = (uint32_t)__shfl((int)hd.w, (int)(sb + j), 64);
        if (o >= sj && o < sj + lj) {
          entry = ej;
          slot = wj;
          off = o - sj;
        }
      }
      g[q] = gld_rec(&packet_recs(d, vi, slot, entry)[off]);  // past keep: a harmless inbox slot-0 read
    }
#pragma unroll
    for (int q = 0; q < LOCK_RPL; q++) {
      const uint32_t o = o0 + sl + SEG * q;
      if (o < keep) gst_rec(&dst[o], g[q]);
    }
  }
  if (act && sl == 0 && deg) {
    d.hs[vi].lock = (lw & ((1u << GX_LOCK_BUF_SHIFT) - 1u)) | (nb0 + keep) << GX_LOCK_BUF_SHIFT;
    ctr_atomic(d, C_LOCK_BUF, keep);
    ctr_atomic(d, C_LOCK_DROP, total - keep);
    kbytes(d, GX_K_MERGE, 32ull * keep + 16ull * deg + 4, 0);  // records in and out, headers
  }
  return true;
}

// The ServicesState lock (gx.h lock_model), ahead of k_merge_seg: the pipeline appends of locked
// receivers, 16 lanes per receiver (lock_append_seg) at 8 waves per SIMD, so a round whose receivers
// are all locked keeps more of these short dependent chains in flight than k_merge_seg's item
// waves (3 per SIMD, sized for the merge path). A receiver done here has its routing count cleared
// (k_merge_seg skips it); one with more packets than a segment takes stays for k_merge_seg.
#ifndef GX_LOCK_APPEND_WPE
#define GX_LOCK_APPEND_WPE 8
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GX_LOCK_APPEND_WPE))) void k_lock_append(Dev d) {
  const uint32_t vi = (blockIdx.x * 256u + threadIdx.x) >> 4;
  bool act = false;
  if (vi < d.Hl) act = d.mrec[vi] != 0 && locked_in(d, d.hs[vi].lock);  // segment-uniform
  if (__ballot(act) == 0) return;  // wave-uniform: nothing to append (a round whose pipelines are full)
  const bool ok = lock_append_seg<16>(d, act ? vi : 0u, act);
  if (act && ok && (threadIdx.x & 15) == 0) d.mrec[vi] = 0;
}

#define MERGE_NR 64  // receivers per block (16 measured 3% slower in the accepting stretch, profiles/r03/ab)
#define MERGE_NONE 0xffffffffu
template <bool K32, bool EV, int NR = MERGE_NR, int WPE = 3>
__global__ __launch_bounds__(64 * MERGE_WAVES) __attribute__((amdgpu_waves_per_eu(WPE))) void k_merge_seg(Dev d) {
  static_assert(NR <= 64, "one routing lane per receiver");
  __shared__ MergeLds s_l[MERGE_WAVES];
  __shared__ uint32_t s_it[NR][4];  // work items: up to 4 receivers (MERGE_NONE: empty)
  __shared__ uint32_t s_ty[NR];     // 0: four 16-lane segments, 1: two 32-lane, 2: one wave, 3: four locked
  __shared__ uint32_t s_fb[NR], s_n[2];
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t r0 = blockIdx.x * NR;
  if (wv == 0) {  // routing: lane k reads receiver r0 + k's count
    const uint32_t vi = r0 + lane;
    uint32_t t = 0;
    if (lane < (uint32_t)NR && vi < d.Hl) t = d.mrec[vi];
    if (t) d.mrec[vi] = 0;  // the senders count next round's
    if (lane < (uint32_t)NR)
      for (int q = 0; q < 4; q++) s_it[lane][q] = MERGE_NONE;
    // the ServicesState lock (gx.h lock_model): a locked receiver with records, and an unlocked one
    // whose pipeline holds records to drain, take the whole-wave path (merge_receiver)
    // (round 5) a locked receiver takes a 16-lane pipeline append (lock_append_seg), four per wave
    bool lkw = false, lka = false;
    if (d.p.lock_model && lane < (uint32_t)NR && vi < d.Hl) {
      const uint32_t lw = d.hs[vi].lock;
      if (locked_in(d, lw) && d.p.fd_handoff_shared) t = 0;  // k_fd_recv takes its items (fd_handoff_locked)
      else if (locked_in(d, lw)) lka = t != 0;
      else lkw = GX_LOCK_BUF(lw) != 0 && !departed(d, d.lo + vi);
    }
    const bool sm = !lkw && !lka && t && t <= 16, md = !lkw && !lka && t > 16 && t <= 32;
    const bool lg = lkw || (!lka && t > 32);
    const uint64_t bs = __ballot(sm), bm = __ballot(md), bl = __ballot(lg), ba = __ballot(lka), below = (1ull << lane) - 1ull;
    const uint32_t nl = (uint32_t)__popcll(bl), nm = (uint32_t)__popcll(bm), ns = (uint32_t)__popcll(bs);
    const uint32_t na = (uint32_t)__popcll(ba);
    const uint32_t nim = (nm + 1) / 2, nis = (ns + 3) / 4, nia = (na + 3) / 4;
    wave_sync();
    if (lka) {
      const uint32_t q = (uint32_t)__popcll(ba & below), it = nl + nim + nis + q / 4;
      s_it[it][q & 3] = vi;
      s_ty[it] = 3;
    } else if (lg) {
      const uint32_t it = (uint32_t)__popcll(bl & below);
      s_it[it][0] = vi;
      s_ty[it] = 2;
    } else if (md) {
      const uint32_t q = (uint32_t)__popcll(bm & below), it = nl + q / 2;
      s_it[it][q & 1] = vi;
      s_ty[it] = 1;
    } else if (sm) {
      const uint32_t q = (uint32_t)__popcll(bs & below), it = nl + nim + q / 4;
      s_it[it][q & 3] = vi;
      s_ty[it] = 0;
    }
    if (lane == 0) {
      s_n[0] = nl + nim + nis + nia;
      s_n[1] = 0;
    }
    if (unsigned long long *kp = kprof_merge(d); kp && lane == 0 && (nl | nm | ns)) {  // diagnostics
      atomicAdd(&kp[0], (unsigned long long)(nl + nm + ns));
      atomicAdd(&kp[1], (unsigned long long)ns);
      atomicAdd(&kp[2], (unsigned long long)nm);
      atomicAdd(&kp[3], (unsigned long long)nl);
    }
    if (unsigned long long *kp = kprof_merge(d); kp && t) atomicAdd(&kp[5], (unsigned long long)t);
  }
  __syncthreads();
  const uint32_t ni = s_n[0];
  if (ni == 0) return;  // block-uniform
  for (uint32_t it = wv; it < ni; it += MERGE_WAVES) {  // wave-uniform item type
    const uint32_t ty = s_ty[it];
    if (ty == 2) {
      merge_receiver<K32, EV>(d, s_it[it][0], s_l[wv]);
    } else if (ty == 3) {
      const uint32_t v = s_it[it][lane >> 4];
      const bool act = v != MERGE_NONE;
      const bool ok = lock_append_seg<16>(d, act ? v : 0u, act);
      if (!ok && (lane & 15) == 0) s_fb[atomicAdd(&s_n[1], 1u)] = v;
    } else if (ty == 1) {
      const uint32_t v = s_it[it][lane >> 5];
      const bool act = v != MERGE_NONE;
      const bool ok = merge_seg<K32, EV, 32>(d, act ? v : 0u, act, s_l[wv]);
      if (!ok && (lane & 31) == 0) s_fb[atomicAdd(&s_n[1], 1u)] = v;
    } else {
      const uint32_t v = s_it[it][lane >> 4];
      const bool act = v != MERGE_NONE;
      const bool ok = merge_seg<K32, EV, 16>(d, act ? v : 0u, act, s_l[wv]);
      if (!ok && (lane & 15) == 0) s_fb[atomicAdd(&s_n[1], 1u)] = v;
    }
  }
  __syncthreads();
  const uint32_t nf = s_n[1];
  if (unsigned long long *kp = kprof_merge(d); kp && threadIdx.x == 0 && nf) atomicAdd(&kp[4], (unsigned long long)nf);
  for (uint32_t k = wv; k < nf; k += MERGE_WAVES) merge_receiver<K32, EV>(d, s_fb[k], s_l[wv]);
}

// ============================================================= phase 5: anti-entropy push-pull ==
// Dense view-pair merge: a <- b and, when `both`, b <- a's pre-exchange words. VEC streams both
// rows with 16-B loads, 4 slots per thread per 1024-slot tile, and compacts each side's
// retransmits in key order with one packed block scan per tile.
template <bool NT>
GXD ulonglong2 ld16(const uint64_t *p) {
  if (NT) {
    typedef unsigned long long v2u64 __attribute__((ext_vector_type(2)));
    v2u64 x = __builtin_nontemporal_load(reinterpret_cast<const v2u64 *>(p));
    return make_ulonglong2(x.x, x.y);
  }
  return *reinterpret_cast<const ulonglong2 *>(p);
}

// Server times of one push-pull side for S dividing 128 (S >= 2, 16-B mapping): a wave's
// 128-slot chunk holds whole owners, S/2 lanes each, so the last accepted / status-changing
// key of every owner comes from a max over its lane group (no LDS, no barrier). f = accepted
// bits 0-3 | changed bits 4-7 of this thread's slots; lk = this thread's running last changed
// key + 1 (state.LastChanged, reduced at the end of the pass).
GXD void side_times_shfl(const Dev &d, uint32_t x, uint32_t base, uint32_t f, const uint64_t *nw, uint32_t &lk,
                         uint32_t &words_written) {
  const uint32_t t = threadIdx.x, lane = t & 63, lpo = d.S / 2;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const uint32_t r0 = base + 512 * h + 2 * t;
    const uint32_t fa0 = (f >> (2 * h)) & 1u, fa1 = (f >> (2 * h + 1)) & 1u;
    const uint32_t fc0 = (f >> (4 + 2 * h)) & 1u, fc1 = (f >> (4 + 2 * h + 1)) & 1u;
    const uint64_t bu_all = __ballot(fa0 | fa1);
    if (!bu_all) continue;  // changes only come with accepts
    // An owner's slots sit in its lane group in key order, so its last accepted (changed) slot is
    // in the group's highest lane with that flag: two ballots and one shuffle per field.
    // The group's highest flagged lane holds the word, so it stores the field itself (no shuffle).
    const uint32_t g0 = lane & ~(lpo - 1);
    const uint64_t gmask = (lpo == 32 ? 0xffffffffull : ((1ull << lpo) - 1ull)) << g0;
    const uint64_t bu = bu_all & gmask, bc = __ballot(fc0 | fc1) & gmask;
    const bool wu = bu && lane == 63u - (uint32_t)__clzll((long long)bu);
    const bool wc = bc && lane == 63u - (uint32_t)__clzll((long long)bc);
    if (wu || wc) {
      gx_server_times *st = srv_times(d, x, owner_of(d, r0));
      if (wu) st->last_updated_ns = ts_of(fa1 ? nw[2 * h + 1] : nw[2 * h]);
      if (wc) st->last_changed_ns = ts_of(fc1 ? nw[2 * h + 1] : nw[2 * h]);
      words_written += (uint32_t)wu + (uint32_t)wc;
    }
    const uint32_t kc = fc1 ? r0 + 2 : (fc0 ? r0 + 1 : 0u);  // state.LastChanged: max over all lanes later
    lk = kc > lk ? kc : lk;
  }
}

// Server times and ChangeEvents of one push-pull tile, key order: fl bit
// 8*side + k = slot k accepted, bit 8*side + 4 + k = its status changed; os = old statuses
// (3 bits per slot). The stored words are read back from the rows. s_last[side] keeps 1 + the
// last changed key of the pass (tiles come in key order, so a running max). EV: also the
// ChangeEvents of listening views; returns the tile's changed counts (side a | side b << 16).
template <bool VEC, bool EV>
GXD uint32_t ae_book(const Dev &d, uint32_t a, uint32_t b, bool both, uint32_t base, uint32_t fl, uint32_t os,
                     const uint64_t *A, const uint64_t *B, uint32_t *s_lu, uint32_t *s_lc, uint32_t *s_last,
                     unsigned long long *s_wave, int32_t evka, int32_t evkb, uint32_t evba, uint32_t evbb) {
  const uint32_t t = threadIdx.x, TILE = 4 * blockDim.x;
  const uint32_t o0 = base / d.S, no = ((base + TILE < d.R ? base + TILE : d.R) - 1) / d.S - o0 + 1;
  unsigned long long epre = 0, etot = 0;
  if (EV) {
    const unsigned long long ec = (unsigned long long)__popc(fl & 0x30u) |
                                  ((unsigned long long)__popc(fl & 0xC0u) << 16) |
                                  ((unsigned long long)__popc(fl & 0x3000u) << 32) |
                                  ((unsigned long long)__popc(fl & 0xC000u) << 48);
    epre = block_excl_scan64(ec, s_wave, etot);
  }
  for (int side = 0; side < (both ? 2 : 1); side++) {
    const uint64_t *X = side ? B : A;
    for (uint32_t i = t; i < no; i += blockDim.x) s_lu[i] = s_lc[i] = 0;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t r = (VEC ? base + 512 * (k >> 1) + 2 * t : base + 2 * blockDim.x * (k >> 1) + 2 * t) + (k & 1);
      if ((fl >> (8 * side + k)) & 1u) atomicMax(&s_lu[owner_of(d, r) - o0], r + 1);
      if ((fl >> (8 * side + 4 + k)) & 1u) {
        atomicMax(&s_lc[owner_of(d, r) - o0], r + 1);
        atomicMax(&s_last[side], r + 1);
        if (EV) {
          const int32_t evk = side ? evkb : evka;
          if (evk >= 0) {
            const int h = k >> 1;
            const uint32_t pos = fld(epre, 2 * side + h) + (h ? fld(etot, 2 * side) : 0u) +
                                 ((k & 1) ? ((fl >> (8 * side + 4 + k - 1)) & 1u) : 0u);
            const int prev = (int)((os >> (3 * (4 * side + k))) & 7u);
            ev_put(d, evk, (side ? evbb : evba) + pos, r, X[r], prev == GX_ABSENT ? GX_UNKNOWN : prev);
          }
        }
      }
    }
    __syncthreads();
    tile_owner_times(d, side ? b : a, X, o0, no, s_lu, s_lc);
    __syncthreads();
  }
  return EV ? (fld(etot, 0) + fld(etot, 1)) | ((fld(etot, 2) + fld(etot, 3)) << 16) : 0u;
}

// `ext` (when both = false): B is host b's row from another shard (read-only); the pair's
// exchange is counted where a is the pair's first member (count_ex). With `xs` (cross-shard pair,
// gx.h "lead"/"return"), B is rebuilt block by block: a block the partner leads is decoded from
// its lead block, a block this side leads from the partner's return block (own slots = A's
// word), and every other block is A's own block (the digests matched), which merges with the
// counts of the identical remote block and no change.
// PF = tiles whose loads are in flight while one is merged; NT = non-temporal loads.
#define XS_MAXB 2048  // digest blocks per row whose offsets ae_pair stages in LDS (R <= 2^20)
struct XSrc {
  const uint8_t *lead;   // the partner's lead blocks (message + 16)
  const uint8_t *ret;    // the partner's return blocks (after the count table)
  const uint32_t *rcnt;  // literal counts of the return blocks
  const uint32_t *lmask, *fmask;  // blocks this side leads / follows
  const uint16_t *lt;    // literal counts of the partner's blocks (its digests)
  const uint32_t *bcnt;  // own blocks: present | stale << 16 (digest pass)
};
// Slots s, s + 1 (s even) of an encoded block (gx.h): own slots keep w[], the others take their
// literal (popcount rank in the neu mask). The prefix popcount of the neu words below slot s's
// word is eight independent loads of the block header (one 128-B line the whole wave reads).
GXD void dec_pair_u(const uint64_t *enc, uint32_t s, bool v0, bool v1, uint64_t *w) {
  const uint32_t wi = s >> 6;
  int32_t pre = -1;
  uint64_t om = 0, nm = 0;
#pragma unroll
  for (uint32_t i = 0; i < 8; i++) {
    const uint64_t x = enc[8 + i];
    pre += i < wi ? __popcll(x) : 0;
    nm = i == wi ? x : nm;
  }
  om = enc[wi];
#pragma unroll
  for (int e = 0; e < 2; e++) {
    const uint32_t b = (s + e) & 63;
    if ((e ? v1 : v0) && !((om >> b) & 1ull)) w[e] = enc[16 + pre + __popcll(nm & ((2ull << b) - 1ull))];
  }
}
// locked: a side holds the ServicesState lock and the pair runs anyway (lock_model = 0): its merges
// are counted as locked (gx.h gx_stats.locked_merges).
template <bool VEC, int PF = 1, bool NT = false, bool EV = false, bool NTS = false>
GXD void ae_pair(const Dev &d, uint32_t a, uint32_t b, bool both, unsigned long long *s_wave,
                 unsigned long long *s_red, const uint64_t *ext = nullptr, bool count_ex = false,
                 const XSrc *xs = nullptr, bool locked = false) {
  uint64_t *A = vrow(d, a);
  uint64_t *B = xs ? A : ext ? const_cast<uint64_t *>(ext) : vrow(d, b);
  gx_host_state *ha = hst(d, a), *hb = both ? hst(d, b) : ha;
  // retransmits: the first `room` of each side are stored, the rest deferred (gx.h gx_job)
  const uint32_t ta0 = ha->fifo_tail, sa0 = ha->fifo_stored, rooma = fifo_room(d, ha->fifo_head, ta0, sa0);
  const uint32_t tb0 = hb->fifo_tail, sb0 = hb->fifo_stored, roomb = fifo_room(d, hb->fifo_head, tb0, sb0);
  const uint32_t ta0q = ta0 % d.Q, tb0q = tb0 % d.Q;  // ring positions of the tails (one division each)
  uint32_t na = 0, nb = 0;
  uint32_t c_merge = 0, c_acc = 0, c_stale = 0, c_wr = 0, c_chg = 0;  // per thread: < 2^32
  uint32_t c_qa = 0, c_qb = 0;  // retransmits counted once both stored windows are full (all deferred)
  const int64_t stale_cut = d.now - d.p.tombstone_lifespan_ns - d.p.stale_fudge_ns;  // merge_word's stale gate
  unsigned long long ma = ~0ull, mb = ~0ull;
  uint32_t t = threadIdx.x;
  const uint32_t TILE = 4 * blockDim.x;
  // change bookkeeping: per-owner last accept / status change of each tile, the
  // last status change of the pass (state.LastChanged), events for listening views; key order
  __shared__ uint32_t s_lu[TILE_OWNERS], s_lc[TILE_OWNERS];
  __shared__ uint32_t s_last[2];
  __shared__ uint32_t s_any[8];  // block_any256
  uint32_t any_par = 0;
  if (t < 2) s_last[t] = 0;  // read after the pass's barriers
  const int32_t evka = __builtin_amdgcn_readfirstlane(d.ev_slot[li(d, a)]);
  const int32_t evkb = __builtin_amdgcn_readfirstlane(both ? d.ev_slot[li(d, b)] : -1);
  const uint32_t ev0a = __builtin_amdgcn_readfirstlane(evka >= 0 ? d.ev_cnt[evka] : 0);
  const uint32_t ev0b = __builtin_amdgcn_readfirstlane(evkb >= 0 ? d.ev_cnt[evkb] : 0);
  uint32_t nev_a = 0, nev_b = 0;
  // S | 128 without events: server times by lane-group shuffles (side_times_shfl)
  const bool shfl_times = !EV && VEC && d.S >= 2 && (128u % d.S) == 0;
  uint32_t lk_a = 0, lk_b = 0;
  // Software pipeline: the next PF 1024-slot tiles' loads are in flight while this tile is
  // merged, written back and (only if something was accepted) compacted.
  uint64_t qa[PF][4], qb[PF][4];
  uint64_t xo_f = 0, xo_r = 0;  // byte offsets of the next lead / return block (block-uniform)
  uint32_t xj = 0, xskip = 0;   // return blocks used; slots of matching blocks not loaded
  // Cross pairs: every block's class and message offset up front in LDS (two block scans), so a
  // tile's blocks wait on their encoded words only, not on the previous block's length.
  __shared__ uint32_t s_xo[XS_MAXB];  // offset | class << 30 (0 digests matched, 1 lead msg, 2 return msg)
  const bool xs_lds = xs && d.nblk_ae <= XS_MAXB;
  if (xs_lds) {
    const uint32_t nb = d.nblk_ae, c = (nb + blockDim.x - 1) / blockDim.x, b0 = t * c;
    const uint32_t b1 = b0 + c < nb ? b0 + c : nb;
    uint32_t fsz = 0, nl = 0;
    for (uint32_t b = b0; b < b1; b++) {
      if ((xs->fmask[b >> 5] >> (b & 31)) & 1u) fsz += 128 + 8u * xs->lt[b];
      else if ((xs->lmask[b >> 5] >> (b & 31)) & 1u) nl++;
    }
    unsigned long long tot;
    const unsigned long long pre = block_excl_scan64((unsigned long long)fsz | ((unsigned long long)nl << 32), s_wave, tot);
    uint32_t fo = (uint32_t)pre, li_ = (uint32_t)(pre >> 32), rsz = 0;
    for (uint32_t b = b0; b < b1; b++)
      if (!((xs->fmask[b >> 5] >> (b & 31)) & 1u) && ((xs->lmask[b >> 5] >> (b & 31)) & 1u))
        rsz += 128 + 8u * xs->rcnt[li_++];
    const unsigned long long rpre = block_excl_scan64(rsz, s_wave, tot);
    uint32_t ro = (uint32_t)rpre;
    li_ = (uint32_t)(pre >> 32);
    for (uint32_t b = b0; b < b1; b++) {
      if ((xs->fmask[b >> 5] >> (b & 31)) & 1u) {
        s_xo[b] = fo | (1u << 30);
        fo += 128 + 8u * xs->lt[b];
      } else if ((xs->lmask[b >> 5] >> (b & 31)) & 1u) {
        s_xo[b] = ro | (2u << 30);
        ro += 128 + 8u * xs->rcnt[li_++];
      } else {
        s_xo[b] = 0;
      }
    }
    __syncthreads();
  }
  // returns the number of the tile's two blocks that were skipped (cross pairs, digests matched)
  auto load_tile = [&](uint32_t base, uint64_t *xa, uint64_t *xb) -> uint32_t {
    uint32_t skipped = 0;
#pragma unroll
    for (int h = 0; h < 2; h++) {
      uint32_t r0 = VEC ? base + 512 * h + 2 * t : base + 2 * blockDim.x * h + 2 * t;
      bool v0 = r0 < d.R, v1 = r0 + 1 < d.R;
      const uint64_t *Bp = B + r0;  // B[r0], B[r0 + 1]
      const uint64_t *enc = nullptr;
      uint32_t blk = (base >> 9) + h;
      if (xs_lds && base + GX_DIGEST_SLOTS * h < d.R) {
        const uint32_t x = s_xo[blk];
        if (x >> 30) {
          enc = reinterpret_cast<const uint64_t *>((x >> 30) == 1 ? xs->lead : xs->ret) + ((x & 0x3fffffffu) >> 3);
        } else {
          if (t == 0) {
            const uint32_t c = xs->bcnt[blk];
            c_merge += c & 0xffffu;
            c_stale += c >> 16;
          }
          xskip += GX_DIGEST_SLOTS;
          skipped++;
          xa[2 * h] = xa[2 * h + 1] = xb[2 * h] = xb[2 * h + 1] = GX_SLOT_ABSENT;
          continue;
        }
      } else if (xs && base + GX_DIGEST_SLOTS * h < d.R) {
        if ((xs->fmask[blk >> 5] >> (blk & 31)) & 1u) {
          enc = reinterpret_cast<const uint64_t *>(xs->lead + xo_f);
          xo_f += 128 + 8ull * xs->lt[blk];
        } else if ((xs->lmask[blk >> 5] >> (blk & 31)) & 1u) {
          enc = reinterpret_cast<const uint64_t *>(xs->ret + xo_r);
          xo_r += 128 + 8ull * xs->rcnt[xj++];
        } else {
          // digests matched: merging the partner's block = merging A's own, which changes
          // nothing; count its present and stale records from the digest pass, load nothing
          if (t == 0) {
            const uint32_t c = xs->bcnt[blk];
            c_merge += c & 0xffffu;
            c_stale += c >> 16;
          }
          xskip += GX_DIGEST_SLOTS;
          skipped++;
          xa[2 * h] = xa[2 * h + 1] = xb[2 * h] = xb[2 * h + 1] = GX_SLOT_ABSENT;
          continue;
        }
      }
      if (enc) {  // a decoded block starts from A's own words (B == A): one load
        if (VEC && v0) {
          ulonglong2 pa = ld16<NT>(&A[r0]);
          xa[2 * h] = xb[2 * h] = pa.x;
          xa[2 * h + 1] = xb[2 * h + 1] = pa.y;
        } else {
          xa[2 * h] = xb[2 * h] = v0 ? A[r0] : GX_SLOT_ABSENT;
          xa[2 * h + 1] = xb[2 * h + 1] = v1 ? A[r0 + 1] : GX_SLOT_ABSENT;
        }
        dec_pair_u(enc, r0 - blk * GX_DIGEST_SLOTS, v0, v1, &xb[2 * h]);
        continue;
      }
      if (VEC) {
        // unconditional loads (a tail tile's slots past R read slot 0 and are masked where the
        // tile is merged): a guarded load here makes the compiler wait on the tile in flight
        // inside the merge of the current one (profiles/r04/kprof_ae.jsonl)
        const uint32_t rc = v0 ? r0 : 0;
        ulonglong2 pa = ld16<NT>(&A[rc]);
        ulonglong2 pb = ld16<NT>(&B[rc]);
        xa[2 * h] = pa.x;
        xa[2 * h + 1] = pa.y;
        xb[2 * h] = pb.x;
        xb[2 * h + 1] = pb.y;
      } else {
        xa[2 * h] = v0 ? A[r0] : GX_SLOT_ABSENT;
        xa[2 * h + 1] = v1 ? A[r0 + 1] : GX_SLOT_ABSENT;
        xb[2 * h] = v0 ? Bp[0] : GX_SLOT_ABSENT;
        xb[2 * h + 1] = v1 ? Bp[1] : GX_SLOT_ABSENT;
      }
    }
    return skipped;
  };
  auto merge_tile = [&](uint32_t base, const uint64_t *wa, const uint64_t *wb) {
    uint64_t nwa[4], nwb[4];
    bool fa[4], fb[4];
    uint32_t accb = 0;  // bit k: side a accepted slot k, bit 8 + k: side b
    // every element defined before the first merge: a partly defined array is copied as a vector
    // whose undefined elements are whatever registers the next tile is loading into, and the copy
    // then waits for those loads (the pipeline stalls inside the merge)
#pragma unroll
    for (int k = 0; k < 4; k++) {
      nwa[k] = wa[k];
      nwb[k] = wb[k];
      fa[k] = fb[k] = false;
    }
    bool same = true;
#pragma unroll
    for (int k = 0; k < 4; k++) same &= wa[k] == wb[k];
    if (__ballot(!same) == 0) {
      // The wave's slots hold the same word on both sides (most of a pass outside an accepting
      // stretch): each present record is merged both ways and is stale or not newer, so merging
      // only counts (merge_word's rules with old == u); nothing is accepted or written
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t pres = st_of(wb[k]) != GX_ABSENT, stl = pres && ts_of(wb[k]) < stale_cut;
        c_merge += both ? 2u * pres : pres;
        c_stale += both ? 2u * stl : stl;
      }
    } else {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      uint32_t r = (VEC ? base + 512 * (k >> 1) + 2 * t : base + 2 * blockDim.x * (k >> 1) + 2 * t) + (k & 1);
      if (st_of(wb[k]) != GX_ABSENT) {  // a.Merge(b): every present record of b
        bool ac, st;
        c_merge++;
        nwa[k] = merge_word(d, wa[k], wb[k], ac, st);
        c_stale += st;
        if (ac) {  // an accepted word is a changed word (insert, or strictly newer)
          fa[k] = !owned_by(d, r, a);
          accb |= 1u << k;
          const unsigned long long x = exp_time(d.p, nwa[k]);
          ma = x < ma ? x : ma;
        }
      }
      if (both && st_of(wa[k]) != GX_ABSENT) {  // b.Merge(a's snapshot)
        bool ac, st;
        c_merge++;
        nwb[k] = merge_word(d, wb[k], wa[k], ac, st);
        c_stale += st;
        if (ac) {
          fb[k] = !owned_by(d, r, b);
          accb |= 1u << (8 + k);
          const unsigned long long x = exp_time(d.p, nwb[k]);
          mb = x < mb ? x : mb;
        }
      }
    }
    const uint32_t nacc = (uint32_t)__popc(accb);
    c_acc += nacc;
    c_wr += nacc;
#pragma unroll
    for (int h = 0; h < 2; h++) {
      uint32_t r0 = VEC ? base + 512 * h + 2 * t : base + 2 * blockDim.x * h + 2 * t;
      const bool cha = (accb >> (2 * h)) & 3u, chb = (accb >> (8 + 2 * h)) & 3u;
      if (VEC) {
        if (NTS) {  // nontemporal stores (A/B)
          typedef unsigned long long v2u64s __attribute__((ext_vector_type(2)));
          if (cha) __builtin_nontemporal_store((v2u64s){nwa[2 * h], nwa[2 * h + 1]}, reinterpret_cast<v2u64s *>(&A[r0]));
          if (chb) __builtin_nontemporal_store((v2u64s){nwb[2 * h], nwb[2 * h + 1]}, reinterpret_cast<v2u64s *>(&B[r0]));
        } else {
          if (cha) *reinterpret_cast<ulonglong2 *>(&A[r0]) = make_ulonglong2(nwa[2 * h], nwa[2 * h + 1]);
          if (chb) *reinterpret_cast<ulonglong2 *>(&B[r0]) = make_ulonglong2(nwb[2 * h], nwb[2 * h + 1]);
        }
      } else {
        if ((accb >> (2 * h)) & 1u) A[r0] = nwa[2 * h];
        if ((accb >> (2 * h + 1)) & 1u) A[r0 + 1] = nwa[2 * h + 1];
        if ((accb >> (8 + 2 * h)) & 1u) B[r0] = nwb[2 * h];
        if ((accb >> (8 + 2 * h + 1)) & 1u) B[r0 + 1] = nwb[2 * h + 1];
      }
    }
    }  // the wave's slots differ somewhere
    unsigned long long cnt = (unsigned long long)(fa[0] + fa[1]) | ((unsigned long long)(fa[2] + fa[3]) << 16) |
                             ((unsigned long long)(fb[0] + fb[1]) << 32) | ((unsigned long long)(fb[2] + fb[3]) << 48);
    // change flags and old statuses, packed so that they are all the bookkeeping below keeps
    // fl bit 8*side + k: accepted, bit 8*side + 4 + k: status changed (ServiceChanged: an insert,
    // or a stored status that differs, :317-340); os: old statuses (events only)
    uint32_t fl = 0, os = 0;
    const bool wave_acc = __ballot(accb != 0) != 0;
    if (wave_acc) {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        bool ca = ((accb >> k) & 1u) && (st_of(wa[k]) == GX_ABSENT || st_of(wa[k]) != st_of(nwa[k]));
        bool cb = ((accb >> (8 + k)) & 1u) && (st_of(wb[k]) == GX_ABSENT || st_of(wb[k]) != st_of(nwb[k]));
        fl |= (accb & (0x101u << k)) | ((uint32_t)ca << (4 + k)) | ((uint32_t)cb << (12 + k));
        c_chg += ca + cb;
        if (EV) os |= ((uint32_t)st_of(wa[k]) << (3 * k)) | ((uint32_t)st_of(wb[k]) << (3 * (4 + k)));
      }
    }
    if (shfl_times) {
      if (wave_acc) {  // this wave accepted something
        side_times_shfl(d, a, base, fl & 0xffu, nwa, lk_a, c_wr);  // server times count as written words
        if (both) side_times_shfl(d, b, base, (fl >> 8) & 0xffu, nwb, lk_b, c_wr);
      }
      // Both stored windows full (block-uniform): every further retransmit is deferred, a count
      // whose order does not matter; count it per thread and reduce once after the pass (no
      // scan, no barrier). Behind a deferred job this holds from the first tile.
      if (na >= rooma && (!both || nb >= roomb)) {
        c_qa += fld(cnt, 0) + fld(cnt, 1);
        c_qb += fld(cnt, 2) + fld(cnt, 3);
        return;
      }
    }
    // (a one-barrier scan with alternating buffers measured within noise at cfg 2, 4 and 5,
    // profiles/r03/ab/ae_scan_barriers.txt)
    if (!block_any256(shfl_times ? cnt != 0 : fl != 0, s_any, any_par)) return;
    unsigned long long tot;
    const unsigned long long pre = block_excl_scan64(cnt, s_wave, tot);
    uint32_t pa[4], pb[4];
    pa[0] = na + fld(pre, 0);
    pa[1] = pa[0] + fa[0];
    pa[2] = na + fld(tot, 0) + fld(pre, 1);
    pa[3] = pa[2] + fa[2];
    pb[0] = nb + fld(pre, 2);
    pb[1] = pb[0] + fb[0];
    pb[2] = nb + fld(tot, 2) + fld(pre, 3);
    pb[3] = pb[2] + fb[2];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      uint32_t r = (VEC ? base + 512 * (k >> 1) + 2 * t : base + 2 * blockDim.x * (k >> 1) + 2 * t) + (k & 1);
      if (fa[k] && pa[k] < rooma)
        d.fifo[(size_t)li(d, a) * d.Q + ring_add(ta0q, pa[k], d.Q)] = make_job(nwa[k], r, meta_of(GX_JOB_RETX, 0, 1));
      if (fb[k] && pb[k] < roomb)
        d.fifo[(size_t)li(d, b) * d.Q + ring_add(tb0q, pb[k], d.Q)] = make_job(nwb[k], r, meta_of(GX_JOB_RETX, 0, 1));
    }
    na += fld(tot, 0) + fld(tot, 1);
    nb += fld(tot, 2) + fld(tot, 3);
    // server times (both sides) and ChangeEvents, key order (out of line: rare, register-heavy)
    if (!shfl_times) {
      uint32_t done = ae_book<VEC, EV>(d, a, b, both, base, fl, os, A, B, s_lu, s_lc, s_last, s_wave, evka, evkb,
                                       ev0a + nev_a, ev0b + nev_b);
      nev_a += done & 0xffffu;
      nev_b += done >> 16;
    }
  };
  uint32_t qk[PF];  // blocks of the tile in flight that were skipped (2 = nothing to merge)
#pragma unroll
  for (int s = 0; s < PF; s++) {
    qk[s] = 0;
    if (s * TILE < d.R) qk[s] = load_tile(s * TILE, qa[s], qb[s]);
  }
  for (uint32_t base = 0; base < d.R; base += PF * TILE) {
#pragma unroll
    for (int s = 0; s < PF; s++) {
      uint32_t bs = base + s * TILE;
      if (bs < d.R) {
        uint64_t wa[4], wb[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          wa[k] = qa[s][k];
          wb[k] = qb[s][k];
        }
        if (VEC && bs + TILE > d.R) {  // the tail tile (block-uniform): slots past R are absent
#pragma unroll
          for (int k = 0; k < 4; k++)
            if (bs + 512 * (k >> 1) + 2 * t >= d.R) wa[k] = wb[k] = GX_SLOT_ABSENT;
        }
        const uint32_t sk = qk[s];
        if (bs + PF * TILE < d.R) qk[s] = load_tile(bs + PF * TILE, qa[s], qb[s]);
        if (sk < 2) merge_tile(bs, wa, wb);  // block-uniform
      }
    }
  }
  ma = block_min(ma, s_red);
  mb = block_min(mb, s_red);
  if (shfl_times) {
    unsigned long long q = block_sum((unsigned long long)c_qa | ((unsigned long long)c_qb << 32), s_red);
    na += (uint32_t)q;
    nb += (uint32_t)(q >> 32);
  }
  block_ctr(d, C_CHG, c_chg, s_red);
  if (shfl_times) {  // the pass's last changed key per side (it is in the row now)
    for (int o = 32; o > 0; o >>= 1) {
      uint32_t ya = __shfl_xor(lk_a, o, 64), yb = __shfl_xor(lk_b, o, 64);
      lk_a = ya > lk_a ? ya : lk_a;
      lk_b = yb > lk_b ? yb : lk_b;
    }
    if ((t & 63) == 0) {
      if (lk_a) atomicMax(&s_last[0], lk_a);
      if (lk_b) atomicMax(&s_last[1], lk_b);
    }
    __syncthreads();
  }
  if (t == 0) {
    if (s_last[0]) d.vlc[li(d, a)] = ts_of(A[s_last[0] - 1]);
    if (both && s_last[1]) d.vlc[li(d, b)] = ts_of(B[s_last[1] - 1]);
    if (evka >= 0) d.ev_cnt[evka] = ev0a + nev_a;
    if (evkb >= 0) d.ev_cnt[evkb] = ev0b + nev_b;
  }
  bool changed = c_wr != 0;
  if (__ballot(changed) != 0 && (t & 63) == 0) mark_change(d);
  unsigned long long cw = wave_sum((unsigned long long)c_wr);
  if ((t & 63) == 0) kbytes(d, GX_K_AE, 8ull * cw, 0);
  block_ctr(d, C_AE_MERGES, c_merge, s_red);
  if (locked) block_ctr(d, C_LOCKED_MERGES, c_merge, s_red);  // block-uniform
  block_ctr(d, C_AE_ACC, c_acc, s_red);
  block_ctr(d, C_STALE, c_stale, s_red);
  if (t == 0) {
    if (ma != ~0ull) atomicMin(&d.minexp[li(d, a)], ma);
    if (both && mb != ~0ull) atomicMin(&d.minexp[li(d, b)], mb);
    const uint32_t oka = na < rooma ? na : rooma, okb = nb < roomb ? nb : roomb;
    if (na) {
      ha->fifo_tail = ta0 + na;
      ha->fifo_stored = sa0 + oka;
    }
    if (both && nb) {
      hb->fifo_tail = tb0 + nb;
      hb->fifo_stored = sb0 + okb;
    }
    ctr_atomic(d, C_RETX, na + (both ? nb : 0));
    ctr_atomic(d, C_QDEFER, (na - oka) + (both ? nb - okb : 0));
    ctr_atomic(d, C_AESLOTS, (unsigned long long)d.R * (both ? 2 : 1));
    const uint64_t loaded = d.R > xskip ? d.R - xskip : 0;  // cross pairs: matching blocks are not read
    kbytes(d, GX_K_AE, 16ull * loaded + 16ull * (oka + (both ? okb : 0)), (unsigned long long)d.R * (both ? 2 : 1));
    if (both || count_ex) ctr_atomic(d, C_AEX, 1);
  }
}

// The ServicesState lock of a push-pull pair whose hosts are both here (gx.h lock_model): a locked
// side's LocalState blocks behind the pending writer, so the exchange does not run (returns true:
// skip it); with lock_model = 0 it runs and `locked` says its merges are counted. Block-uniform.
// gx.h lock_readers: a pair whose locked sides are all read-locked with no writer waiting is flagged
// (ro_flag[t], t its index in the launch) for k_ae_ro, which runs it after the launch.
GXD bool ae_lock_skip(const Dev &d, uint32_t a, uint32_t b, bool &locked, uint32_t t) {
  locked = host_locked(d, a) || host_locked(d, b);
  if (!locked) return false;
  const bool ro = d.p.lock_model && ro_pair(d, a, b);
  if (threadIdx.x == 0) {
    atomicMin(&d.ctr->first_drop[shard_id()][1], (unsigned long long)d.round);
    if (ro) d.ro_flag[t] = 1;
    else if (d.p.lock_model) ctr_atomic(d, C_AE_LOCKED, 1);
  }
  return d.p.lock_model != 0;
}
// Pair t of the round's perfect matching (halves while partitioned): hosts a, b.
GXD void ae_pair_hosts(const Dev &d, uint32_t t, uint64_t key0, uint64_t key1, uint32_t &a, uint32_t &b) {
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
  a = base + feistel_perm(key, 2 * q, m);
  b = base + feistel_perm(key, 2 * q + 1, m);
}
// A block takes a chunk of up to 256 pairs (np / gridDim.x rounded up): each thread checks one
// pair's members (a crashed member, the failure detector's view, the ServicesState lock) so the
// chunk's skipped pairs cost one round trip together, then the block merges the pairs that run,
// one after another. Pairs are disjoint, so their order does not matter.
#define AE_GRID 4096
template <bool VEC, bool EV, int PF, bool NT, bool NTS = false>
GXD void ae_round_pair(const Dev &d, uint64_t key0, uint64_t key1) {
  __shared__ unsigned long long s_wave[4];
  __shared__ unsigned long long s_red[4];
  uint32_t t = blockIdx.x, base = 0, m = d.H, q = t;
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
  unsigned long long *kp = kprof_ae(d);
  if (kp && threadIdx.x == 0) kp[2 * blockIdx.x] = wall_clock64() | ((unsigned long long)__smid() << 48);
  uint32_t a = base + feistel_perm(key, 2 * q, m);
  uint32_t b = base + feistel_perm(key, 2 * q + 1, m);
  // a crashed member skips the pair; with the failure detector the network path is needed and
  // the initiator (a) must see b ALIVE (memberlist pushPull picks among alive nodes)
  if (d.departures || d.p.fd_enable) {
    bool ok = !departed(d, a) && !departed(d, b);
    if (ok && d.p.fd_enable) ok = reach(d, a, b) && memp(d, a, b)->state == GX_M_ALIVE;
    if (!ok) return;
  }
  bool locked;
  if (ae_lock_skip(d, a, b, locked, t)) return;
  ae_pair<VEC, PF, NT, EV, NTS>(d, a, b, true, s_wave, s_red, nullptr, false, nullptr, locked);
  if (kp && threadIdx.x == 0) kp[2 * blockIdx.x + 1] = wall_clock64();
}

template <bool VEC, bool EV, int PF, bool NT, bool NTS = false>
GXD void ae_round_pairs(const Dev &d, uint64_t key0, uint64_t key1, uint32_t np) {
  __shared__ unsigned long long s_wave[4];
  __shared__ unsigned long long s_red[4];
  __shared__ uint32_t s_run[256];  // pair index | 1 << 31 when a side holds the lock (lock_model = 0)
  __shared__ uint32_t s_nrun, s_nlock;
  const uint32_t per = (np + gridDim.x - 1) / gridDim.x;  // <= 256 (the launch sizes the grid)
  const uint32_t c0 = blockIdx.x * per, c1 = c0 + per < np ? c0 + per : np;
  unsigned long long *kp = kprof_ae(d);
  if (kp && threadIdx.x == 0) kp[2 * blockIdx.x] = wall_clock64() | ((unsigned long long)__smid() << 48);
  if (threadIdx.x == 0) s_nrun = s_nlock = 0;
  __syncthreads();
  const uint32_t tq = c0 + threadIdx.x;
  if (tq < c1) {
    uint32_t a, b;
    ae_pair_hosts(d, tq, key0, key1, a, b);
    // a crashed member skips the pair; with the failure detector the network path is needed and
    // the initiator (a) must see b ALIVE (memberlist pushPull picks among alive nodes)
    bool ok = true;
    if (d.departures || d.p.fd_enable) {
      ok = !departed(d, a) && !departed(d, b);
      if (ok && d.p.fd_enable) ok = reach(d, a, b) && memp(d, a, b)->state == GX_M_ALIVE;
    }
    if (ok) {
      const bool locked = host_locked(d, a) || host_locked(d, b);
      const bool ro = locked && d.p.lock_model && ro_pair(d, a, b);  // k_ae_ro runs it (lock_readers)
      if (ro) {
        d.ro_flag[tq] = 1;
        atomicMin(&d.ctr->first_drop[shard_id()][1], (unsigned long long)d.round);
      } else if (locked) {
        atomicAdd(&s_nlock, 1u);
      }
      if (!(locked && d.p.lock_model)) s_run[atomicAdd(&s_nrun, 1u)] = tq | (locked ? 1u << 31 : 0u);
    }
  }
  __syncthreads();
  const uint32_t nrun = s_nrun;
  if (threadIdx.x == 0 && s_nlock) {
    atomicMin(&d.ctr->first_drop[shard_id()][1], (unsigned long long)d.round);
    if (d.p.lock_model) ctr_atomic(d, C_AE_LOCKED, s_nlock);
  }
  for (uint32_t k = 0; k < nrun; k++) {
    const uint32_t x = s_run[k];
    uint32_t a, b;
    ae_pair_hosts(d, x & 0x7fffffffu, key0, key1, a, b);
    ae_pair<VEC, PF, NT, EV, NTS>(d, a, b, true, s_wave, s_red, nullptr, false, nullptr, (x >> 31) != 0);
    __syncthreads();  // the next pair's shared state
  }
  if (kp && threadIdx.x == 0) kp[2 * blockIdx.x + 1] = wall_clock64();
}
// Blocks of a push-pull launch: one pair per block without the lock model (blocks are scheduled as
// CUs free up, which evens out pairs of different cost: static chunks of 4 pairs measured 4% slower
// over the bench window, profiles/r05/c5), chunks of at most 256 pairs with it (a locked round's
// pairs then cost 17 us instead of a contended counter atomic per pair).
GXHD uint32_t ae_grid(uint32_t np, uint32_t lock_model) {
  if (!lock_model) return np;
  const uint32_t g = np < AE_GRID ? np : AE_GRID;
  return g > (np + 255) / 256 ? g : (np + 255) / 256;
}

// The push-pull kernel, without ChangeEvents (no listener anywhere): kept within 128 VGPRs so
// that 4 waves per SIMD stay resident; with events (listeners present) a separate entry point.
#ifndef GX_AE_WPE
#define GX_AE_WPE 4  // 5 / 6 spill 47 / 87 VGPRs: 1.8x / 2.6x slower at cfg 2 (profiles/r05/ab/ae_wpe_cfg*.jsonl)
#endif
template <bool VEC, int PF = 1, bool NT = false, bool NTS = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GX_AE_WPE))) void k_ae(Dev d, uint64_t key0,
                                                                                   uint64_t key1) {
  ae_round_pair<VEC, false, PF, NT, NTS>(d, key0, key1);
}
template <bool VEC>
__global__ __launch_bounds__(256) void k_ae_ev(Dev d, uint64_t key0, uint64_t key1) {
  ae_round_pair<VEC, true, 1, false>(d, key0, key1);
}
// Under the lock model: chunks of pairs per block (ae_round_pairs), grid ae_grid(np, 1).
template <bool VEC, int PF = 1, bool NT = false, bool NTS = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_ae_chunk(Dev d, uint64_t key0,
                                                                                         uint64_t key1, uint32_t np) {
  ae_round_pairs<VEC, false, PF, NT, NTS>(d, key0, key1, np);
}

// gx.h lock_readers: the exchanges of the last push-pull launch whose locked sides are all
// read-locked with no writer waiting (ro_flag[t]; pair t of the matching round from key0/key1, or
// of the initiate batch pa/pb). One block, after the launch: (1) the read-locked sides claim their
// pool slots (slot v % P, free at the launch's start: the lowest host id gets it, whatever the
// order, as the oracle's ae_claims); (2) the flagged pairs in pair order: a read-locked side keeps
// the partner's pre-exchange row in its slot (services_delegate.go:153-167 -> services_state.go:
// 367-373 -> UpdateService :138-140, blocked behind the lock) or counts it lost, then the unlocked
// side merges the partner's row (ae_pair, one direction); (3) the claims are reset. The pairs are
// disjoint and no other pair of the launch touches their rows, so running them after the launch is
// the oracle's result (ae_exchange_read_locked). Clears ro_flag.
template <bool VEC, bool EV>
__global__ __launch_bounds__(256) void k_ae_ro(Dev d, const uint32_t *pa, const uint32_t *pb, uint64_t key0, uint64_t key1,
                                               uint32_t n) {
  __shared__ unsigned long long s_wave[4];
  __shared__ unsigned long long s_red[4];
  __shared__ uint32_t s_pre[256];
  __shared__ uint32_t s_n;
  const uint32_t tid = threadIdx.x, per = (n + 255) / 256, t0 = tid * per < n ? tid * per : n;
  const uint32_t t1 = t0 + per < n ? t0 + per : n;
  auto hosts = [&](uint32_t t, uint32_t &a, uint32_t &b) {
    if (pa) {
      a = pa[t];
      b = pb[t];
    } else {
      ae_pair_hosts(d, t, key0, key1, a, b);
    }
  };
  uint32_t c = 0;
  for (uint32_t t = t0; t < t1; t++) {  // (1) claims
    if (!d.ro_flag[t]) continue;
    c++;
    uint32_t a, b;
    hosts(t, a, b);
    for (int k = 0; k < 2; k++) {
      const uint32_t x = k ? b : a;
      if (!host_locked(d, x)) continue;
      const uint32_t slot = x % d.P;
      if (d.dpool_host[slot] == GX_NOHOST) atomicMin(&d.dclaim[slot], x);
    }
  }
  s_pre[tid] = c;
  __syncthreads();
  if (tid == 0) {  // the flagged pairs' places in pair order (threads hold consecutive ranges)
    uint32_t run = 0;
    for (uint32_t i = 0; i < 256; i++) {
      const uint32_t x = s_pre[i];
      s_pre[i] = run;
      run += x;
    }
    s_n = run;
  }
  __syncthreads();
  uint32_t pos = s_pre[tid];
  for (uint32_t t = t0; t < t1; t++)
    if (d.ro_flag[t]) {
      d.ro_list[pos++] = t;
      d.ro_flag[t] = 0;
    }
  __threadfence();
  __syncthreads();
  const uint32_t nro = s_n;
  for (uint32_t k = 0; k < nro; k++) {  // (2) the exchanges
    uint32_t a, b;
    hosts(d.ro_list[k], a, b);
    const bool la = host_locked(d, a), lb = host_locked(d, b);
    __syncthreads();  // every thread has read the lock words before a side's DEFER bit is set
    for (int q = 0; q < 2; q++) {  // a read-locked side keeps the partner's row (before any merge)
      const uint32_t x = q ? b : a, y = q ? a : b;
      if (!(q ? lb : la)) continue;
      const uint32_t slot = x % d.P;
      if (d.dclaim[slot] != x) {  // the slot went to another host: the merge is lost
        if (tid == 0) ctr_atomic(d, C_AE_DEFER_LOST, 1);
        continue;
      }
      const uint64_t *src = vrow(d, y);
      uint64_t *dst = &d.dpool[(size_t)slot * d.R];
      unsigned long long np = 0;
      for (uint32_t r = tid; r < d.R; r += blockDim.x) {
        const uint64_t w = src[r];
        dst[r] = w;
        np += st_of(w) != GX_ABSENT;
      }
      np = block_sum(np, s_red);
      if (tid == 0) {
        d.dpool_host[slot] = x;
        d.dpool_res[slot] = np < GX_LOCK_DEFER_RES ? (uint32_t)np : GX_LOCK_DEFER_RES;
        hst(d, x)->lock |= GX_LOCK_DEFER_MERGE;
        ctr_atomic(d, C_AE_DEFER, 1);
        kbytes(d, GX_K_AE, 16ull * d.R, 0);
      }
    }
    __threadfence();
    __syncthreads();
    if (!la) ae_pair<VEC, 1, false, EV>(d, a, b, false, s_wave, s_red);  // the unlocked side merges now
    else if (!lb) ae_pair<VEC, 1, false, EV>(d, b, a, false, s_wave, s_red);
    if (tid == 0) ctr_atomic(d, C_AEX, 1);
    __syncthreads();
  }
  for (uint32_t x = tid; x < d.P; x += blockDim.x) d.dclaim[x] = GX_NOHOST;  // (3)
}
// gx.h lock_readers: the waiting merge of pool slot s's host at the receive phase of the host's
// first unlocked round, before its pipeline and this round's packets (k_merge_seg runs after): the
// kept row through Merge in key order (ae_pair from the pool row, SRC_AE). Oracle: run_deferred_merge.
// The receiver's row changed after its senders read the slot words they forward, so its merge
// reads the slots again (tick 2: w0_fwd).
template <bool VEC, bool EV>
__global__ __launch_bounds__(256) void k_defer_drain(Dev d) {
  __shared__ unsigned long long s_wave[4];
  __shared__ unsigned long long s_red[4];
  const uint32_t s = blockIdx.x, x = d.dpool_host[s];
  if (x == GX_NOHOST || x - d.lo >= d.Hl) return;  // block-uniform
  const uint32_t vi = x - d.lo, lw = d.hs[vi].lock;
  if (locked_in(d, lw) || departed(d, x)) return;
  ae_pair<VEC, 1, false, EV>(d, x, x, false, s_wave, s_red, &d.dpool[(size_t)s * d.R]);
  if (threadIdx.x == 0) {
    d.dpool_host[s] = GX_NOHOST;
    d.dpool_res[s] = 0;
    d.hs[vi].lock = lw & ~GX_LOCK_DEFER_MERGE;
    d.tick[vi] = 2;
  }
}

template <bool VEC, bool EV>
__global__ __launch_bounds__(256) void k_merge_views(Dev d, uint32_t dst, uint32_t src) {
  __shared__ unsigned long long s_wave[4];
  __shared__ unsigned long long s_red[4];
  ae_pair<VEC, 1, false, EV>(d, dst, src, false, s_wave, s_red);
}

// Sharded push-pull: plan entry i = (a, b, k): k < 0 -> both members here (a <-> b); k >= 0 ->
// a is here and b is cross pair k, its row rebuilt from the lead and return inboxes: a <- b only.
struct AeIn {
  const uint8_t *lead, *ret;         // the two inboxes
  const uint64_t *ioff, *rioff;      // [k] message offsets in them
  const uint32_t *lmask, *fmask;     // [k][nmw]
  const uint16_t *lt;                // [k][nblk]
  const uint32_t *nlead;             // [k]
  const uint32_t *bcnt;              // [k][nblk] own blocks' present | stale << 16
  uint32_t nmw, nblk;
};
template <bool VEC, bool EV, int PF = 1>
GXD void ae_plan_pair(Dev d, const uint32_t *pa, const uint32_t *pb, const int32_t *prow,
                      const uint8_t *pcount, const AeIn &in, const uint8_t *skip) {
  __shared__ unsigned long long s_wave[4];
  __shared__ unsigned long long s_red[4];
  uint32_t i = blockIdx.x;
  int32_t k = prow[i];
  if (k < 0 && d.p.fd_enable && !(reach(d, pa[i], pb[i]) && memp(d, pa[i], pb[i])->state == GX_M_ALIVE))
    return;  // memberlist pushPull: the initiator (pa) needs the path and sees the partner alive
  if (k >= 0 && (skip[k] & 1u)) return;  // the same decision for a cross-shard pair (digest flag)
  if (k < 0) {
    bool locked;
    if (ae_lock_skip(d, pa[i], pb[i], locked, i)) return;
    ae_pair<VEC, PF, false, EV>(d, pa[i], pb[i], true, s_wave, s_red, nullptr, false, nullptr, locked);
  } else {
    const uint32_t nl = in.nlead[k];
    const uint8_t *rm = in.ret + in.rioff[k];
    XSrc xs;
    xs.lead = in.lead + in.ioff[k] + 16;
    xs.rcnt = reinterpret_cast<const uint32_t *>(rm + 16);
    xs.ret = rm + 16 + 4ull * (nl + (nl & 1u));
    xs.lmask = in.lmask + (size_t)k * in.nmw;
    xs.fmask = in.fmask + (size_t)k * in.nmw;
    xs.lt = in.lt + (size_t)k * in.nblk;
    xs.bcnt = in.bcnt + (size_t)k * in.nblk;
    ae_pair<VEC, PF, false, EV>(d, pa[i], pb[i], false, s_wave, s_red, nullptr, pcount[i] != 0, &xs, (skip[k] & 2u) != 0);
  }
}
template <bool VEC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_ae_plan(
    Dev d, const uint32_t *pa, const uint32_t *pb, const int32_t *prow, const uint8_t *pcount, AeIn in,
    const uint8_t *skip) {
  ae_plan_pair<VEC, false>(d, pa, pb, prow, pcount, in, skip);
}
// Launches too small to fill the chip (a few pairs per CU): two tiles in flight per block.
template <bool VEC>
__global__ __launch_bounds__(256) void k_ae_plan_pf2(Dev d, const uint32_t *pa, const uint32_t *pb,
                                                      const int32_t *prow, const uint8_t *pcount, AeIn in,
                                                      const uint8_t *skip) {
  ae_plan_pair<VEC, false, 2>(d, pa, pb, prow, pcount, in, skip);
}
template <bool VEC>
__global__ __launch_bounds__(256) void k_ae_plan_ev(Dev d, const uint32_t *pa, const uint32_t *pb, const int32_t *prow,
                                                     const uint8_t *pcount, AeIn in, const uint8_t *skip) {
  ae_plan_pair<VEC, true>(d, pa, pb, prow, pcount, in, skip);
}

// Push-pull pairs of this round in global order t (group 0's n0 pairs, then group 1's), drawn
// like k_ae draws them: (base + perm(2q), base + perm(2q + 1)).
__global__ void k_ae_pairs(uint32_t base0, uint32_t m0, uint64_t key0, uint32_t base1, uint32_t m1, uint64_t key1,
                           uint32_t n0, uint32_t np, uint32_t *pa, uint32_t *pb) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= np) return;
  const bool g1 = t >= n0;
  const uint32_t q = g1 ? t - n0 : t, base = g1 ? base1 : base0, m = g1 ? m1 : m0;
  const uint64_t key = g1 ? key1 : key0;
  pa[t] = base + feistel_perm(key, 2 * q, m);
  pb[t] = base + feistel_perm(key, 2 * q + 1, m);
}

// Push-pull digests of this shard's cross-pair rows (gx.h "digest"): one block per pair, one wave
// per 512-slot block at a time. Also kept in `own` for the comparison.
// Slot hash of the block digest (gx.h): 32-bit multiply-xorshift rounds (no 64-bit multiplies,
// which cost four 32-bit ones each and made the digest pass ALU-bound).
GXD uint64_t dig_hash(uint64_t w, uint32_t i) {
  const uint64_t x = w ^ ((uint64_t)i << 40) ^ i;
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  uint32_t a = (lo ^ ((hi << 16) | (hi >> 16))) * 0x85EBCA6Bu;
  uint32_t b = (hi ^ (a >> 15)) * 0xC2B2AE35u;
  a = (a ^ (b >> 13)) * 0x27D4EB2Fu;
  a ^= a >> 16;
  b = (b ^ (a >> 11)) * 0x165667B1u;
  b ^= b >> 15;
  return (uint64_t)a << 32 | b;
}
// With the failure detector the initiator's side decides whether the pair runs (it needs the
// path and sees the partner alive, memberlist pushPull) and says so in header word 3.
GXD bool ae_initiator_runs(const Dev &d, uint32_t mine, uint32_t other) {
  return reach(d, mine, other) && memp(d, mine, other)->state == GX_M_ALIVE;
}
// digest message size (gx.h): + the host's round-start member list with push-pull membership
GXHD size_t dig_stride(const Dev &d, uint32_t nblk) {
  return 16 + 16ull * nblk + (d.p.fd_enable && d.p.fd_push_pull_state ? 8ull * d.H : 0);
}
template <bool VEC>
__global__ __launch_bounds__(256) void k_ae_digest(Dev d, const uint32_t *host, const uint32_t *pair_t,
                                                    const uint32_t *other, const uint8_t *first, uint8_t *out,
                                                    ulonglong2 *own, uint32_t nblk, uint32_t *bcnt) {
  const uint32_t k = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint8_t *msg = out + (size_t)k * dig_stride(d, nblk);
  if (d.p.fd_enable && d.p.fd_push_pull_state) {  // the member list, snapshot of this AE round (k_fd_snap)
    const uint64_t *snap = &d.fd_snap[(size_t)li(d, host[k]) * d.H];
    uint64_t *dst = reinterpret_cast<uint64_t *>(msg + 16 + 16ull * nblk);
    for (uint32_t x = threadIdx.x; x < d.H; x += blockDim.x) dst[x] = snap[x];
  }
  if (threadIdx.x == 0) {
    uint32_t *hdr = reinterpret_cast<uint32_t *>(msg);
    hdr[0] = pair_t[k];
    hdr[1] = host[k];
    hdr[2] = nblk;
    // bit 0: with the failure detector, the initiator's decision that the pair runs; bit 1: this
    // side's host holds the ServicesState lock this round (gx.h lock_model)
    hdr[3] = (d.p.fd_enable && first[k] && ae_initiator_runs(d, host[k], other[k]) ? 1u : 0u) |
             (host_locked(d, host[k]) ? 2u : 0u);
  }
  if (d.p.lock_model && host_locked(d, host[k])) {  // the pair fails (gx.h digest): zero digests, no row read
    for (uint32_t b = threadIdx.x; b < nblk; b += blockDim.x)
      *reinterpret_cast<ulonglong2 *>(msg + 16 + 16ull * b) = make_ulonglong2(0ull, 0ull);
    return;
  }
  const uint64_t *row = vrow(d, host[k]);
  // software pipeline: the wave's next block is in flight while this one is hashed and reduced
  ulonglong2 cur[4], nxt[4];
  auto load_blk = [&](uint32_t b, ulonglong2 *x) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint32_t i = b * GX_DIGEST_SLOTS + 2 * (64 * q + lane);
      const bool v0 = i < d.R, v1 = i + 1 < d.R;
      if (VEC && v0) {
        x[q] = *reinterpret_cast<const ulonglong2 *>(&row[i]);
      } else {
        x[q].x = v0 ? row[i] : 0;
        x[q].y = v1 ? row[i + 1] : 0;
      }
    }
  };
  const int64_t thr = d.now - d.p.tombstone_lifespan_ns - d.p.stale_fudge_ns;
  if (wv < nblk) load_blk(wv, cur);
  for (uint32_t b = wv; b < nblk; b += 4) {
    if (b + 4 < nblk) load_blk(b + 4, nxt);
    uint64_t s0 = 0, s1 = 0, carry = 0;
    uint32_t lits = 0;  // literal count of the block's lead encoding (neighbour rule, gx.h)
    uint32_t cnt = 0;   // present | stale << 16: what merging this block as-is counts
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint32_t i = b * GX_DIGEST_SLOTS + 2 * (64 * q + lane);
      const uint64_t w0 = cur[q].x, w1 = cur[q].y;
      const bool v0 = i < d.R, v1 = i + 1 < d.R;
      if (v0) {
        const uint64_t h = dig_hash(w0, i);
        s0 += h;
        s1 += h ^ (h >> 29);
      }
      if (v1) {
        const uint64_t h = dig_hash(w1, i + 1);
        s0 += h;
        s1 += h ^ (h >> 29);
      }
      uint64_t pw = __shfl_up(w1, 1, 64);  // the slot before 2 * (64q + lane)
      if (lane == 0) pw = carry;
      lits += (v0 && ((q == 0 && lane == 0) || w0 != pw)) + (v1 && w1 != w0);
      if (v0 && st_of(w0) != GX_ABSENT) cnt += 1u + ((uint32_t)(ts_of(w0) < thr) << 16);
      if (v1 && st_of(w1) != GX_ABSENT) cnt += 1u + ((uint32_t)(ts_of(w1) < thr) << 16);
      carry = __shfl(w1, 63, 64);
    }
    s0 = wave_sum(s0);
    s1 = wave_sum(s1);
    const unsigned long long lc = wave_sum((unsigned long long)cnt | ((unsigned long long)lits << 32));
    if (lane == 0) {
      bcnt[(size_t)k * nblk + b] = (uint32_t)lc;
      ulonglong2 dg = make_ulonglong2(s0, (s1 & ((1ull << 54) - 1)) | (uint64_t)(lc >> 32) << 54);
      own[(size_t)k * nblk + b] = dg;
      *reinterpret_cast<ulonglong2 *>(msg + 16 + 16ull * b) = dg;
    }
#pragma unroll
    for (int q = 0; q < 4; q++) cur[q] = nxt[q];
  }
}

// gx_lock_census: this shard's hosts that do not hold the ServicesState lock this round.
__global__ __launch_bounds__(256) void k_lock_census(Dev d, uint32_t *out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool free_ = i < d.Hl && !host_locked(d, d.lo + i);
  const unsigned long long m = __ballot(free_);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(out, (uint32_t)__popcll(m));
}
// gx_ae_skip_locked: the counts of a push-pull round whose every pair fails on the lock.
__global__ void k_ae_locked_note(Dev d, uint32_t n_first, uint32_t any) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  if (n_first) ctr_atomic(d, C_AE_LOCKED, n_first);
  if (any) atomicMin(&d.ctr->first_drop[shard_id()][1], (unsigned long long)d.round);
}

// Compare own digests with the partner's (message k of `in`): the blocks that differ, and who
// leads each (fewer literals; ties: the pair's first host). Per pair: lead and follow counts, the
// size of this side's lead message and of the partner's. A pair that does not run (failure
// detector: the initiator's decision) ships no blocks.
__global__ __launch_bounds__(256) void k_ae_mask(Dev d, const uint8_t *in, const ulonglong2 *own,
                                                  const uint32_t *pair_t, const uint32_t *host, const uint32_t *other,
                                                  const uint8_t *first, uint32_t nblk, uint32_t nmw, uint32_t *lmask,
                                                  uint32_t *fmask, uint16_t *lt, uint32_t *nlead, uint32_t *nfol,
                                                  uint64_t *lsz, uint64_t *isz, uint32_t *err, uint8_t *skip) {
  __shared__ unsigned long long s_n[4][3];
  const uint32_t k = blockIdx.x;
  const uint8_t *msg = in + (size_t)k * dig_stride(d, nblk);
  const uint32_t *hdr = reinterpret_cast<const uint32_t *>(msg);
  if (threadIdx.x == 0 && (hdr[0] != pair_t[k] || hdr[2] != nblk)) atomicOr(err, 1u);
  bool runs = !d.p.fd_enable || (first[k] ? ae_initiator_runs(d, host[k], other[k]) : (hdr[3] & 1u) != 0);
  // the ServicesState lock (gx.h lock_model): a side that holds it fails the exchange; with
  // lock_model = 0 the pair runs and its merges count as locked (skip bit 1)
  const bool lk = runs && (host_locked(d, host[k]) || (hdr[3] & 2u) != 0);
  if (lk && threadIdx.x == 0) {
    atomicMin(&d.ctr->first_drop[shard_id()][1], (unsigned long long)d.round);
    if (d.p.lock_model && first[k]) ctr_atomic(d, C_AE_LOCKED, 1);
  }
  if (lk && d.p.lock_model) runs = false;
  if (threadIdx.x == 0) skip[k] = (runs ? 0 : 1) | (lk && runs ? 2 : 0);
  unsigned long long n = 0, bl = 0, bi = 0;  // n: lead count | follow count << 32
  if (!runs) {  // block-uniform: a pair that does not run leads and follows nothing (its digests unread)
    for (uint32_t w = threadIdx.x; w < nmw; w += blockDim.x) {
      lmask[(size_t)k * nmw + w] = 0;
      fmask[(size_t)k * nmw + w] = 0;
    }
  } else {
    // one block per thread, 256 at a time: a wave's 64 blocks are two mask words (ballots)
    const uint32_t lane = threadIdx.x & 63, wvb = threadIdx.x >> 6;
    for (uint32_t b0 = 0; b0 < nblk; b0 += blockDim.x) {
      const uint32_t b = b0 + threadIdx.x;
      bool lead = false, fol = false;
      if (b < nblk) {
        const ulonglong2 x = own[(size_t)k * nblk + b];
        const ulonglong2 y = *reinterpret_cast<const ulonglong2 *>(msg + 16 + 16ull * b);
        const uint32_t lm = (uint32_t)(x.y >> 54), ly = (uint32_t)(y.y >> 54);
        lt[(size_t)k * nblk + b] = (uint16_t)ly;
        if (x.x != y.x || x.y != y.y) {
          lead = lm < ly || (lm == ly && first[k]);
          fol = !lead;
          if (lead) bl += 128 + 8ull * lm;
          else bi += 128 + 8ull * ly;
        }
      }
      const unsigned long long ml = __ballot(lead), mf = __ballot(fol);
      const uint32_t w0 = (b0 + 64 * wvb) >> 5;  // the wave's first mask word
      if (lane < 2 && w0 + lane < nmw) {
        lmask[(size_t)k * nmw + w0 + lane] = (uint32_t)(ml >> (32 * lane));
        fmask[(size_t)k * nmw + w0 + lane] = (uint32_t)(mf >> (32 * lane));
      }
      n += (unsigned long long)lead | ((unsigned long long)fol << 32);
    }
  }
  n = wave_sum(n);
  bl = wave_sum(bl);
  bi = wave_sum(bi);
  const uint32_t wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_n[wv][0] = n;
    s_n[wv][1] = bl;
    s_n[wv][2] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long tn = 0, tl = 0, ti = 0;
    for (int q = 0; q < 4; q++) {
      tn += s_n[q][0];
      tl += s_n[q][1];
      ti += s_n[q][2];
    }
    nlead[k] = (uint32_t)tn;
    nfol[k] = (uint32_t)(tn >> 32);
    lsz[k] = 16 + tl;
    isz[k] = 16 + ti;
  }
}

// Own flags of the padding past the row's end in mask word q of a block with n slots.
GXD uint64_t pad_mask(uint32_t n, uint32_t q) {
  return n >= 64 * (q + 1) ? 0ull : n <= 64 * q ? ~0ull : ~0ull << (n - 64 * q);
}
// Block-wide encoding of one block (gx.h "encoded block"): thread t holds slots t and t + 256
// (words w[], own flags own[], new-literal flags nw[]); writes the masks and the literals at enc.
GXD void enc_store(uint64_t *enc, const uint64_t *w, const bool *ownf, const bool *nw, unsigned long long *s_om,
                   unsigned long long *s_nm) {
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    if (nw[h]) {
      const uint32_t wi = 4 * h + wv;
      uint32_t rank = __popcll(s_nm[wi] & ((1ull << lane) - 1ull));
      for (uint32_t q = 0; q < wi; q++) rank += __popcll(s_nm[q]);
      enc[16 + rank] = w[h];
    }
  }
  if (t < 8) {
    enc[t] = s_om[t];
    enc[8 + t] = s_nm[t];
  }
}

// Lead messages (gx.h "lead"): the blocks this side leads, run-length coded, at off[k].
__global__ __launch_bounds__(256) void k_ae_lead_pack(Dev d, const uint32_t *host, const uint32_t *pair_t,
                                                       const uint32_t *lmask, const uint32_t *nlead,
                                                       const uint64_t *off, uint32_t nmw, uint8_t *out) {
  __shared__ unsigned long long s_om[8], s_nm[8];
  const uint32_t k = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  uint8_t *msg = out + off[k];
  if (t == 0) {
    uint32_t *hdr = reinterpret_cast<uint32_t *>(msg);
    hdr[0] = pair_t[k];
    hdr[1] = host[k];
    hdr[2] = nlead[k];
    hdr[3] = 0;
  }
  const uint64_t *row = vrow(d, host[k]);
  uint64_t o = 16;
  for (uint32_t mw = 0; mw < nmw; mw++) {
    uint32_t bits = lmask[(size_t)k * nmw + mw];
    while (bits) {
      const uint32_t blk = mw * 32 + (uint32_t)__builtin_ctz(bits);
      bits &= bits - 1;
      const uint32_t lo = blk * GX_DIGEST_SLOTS, n = lo + GX_DIGEST_SLOTS <= d.R ? GX_DIGEST_SLOTS : d.R - lo;
      uint64_t w[2];
      bool ownf[2], nw[2];
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const uint32_t s = 256 * h + t;
        const bool v = s < n;
        w[h] = v ? row[lo + s] : 0;
        const uint64_t p = v && s > 0 ? row[lo + s - 1] : 0;
        ownf[h] = !v;
        nw[h] = v && (s == 0 || w[h] != p);
        const unsigned long long m = __ballot(nw[h]);
        if (lane == 0) {
          s_nm[4 * h + wv] = m;
          s_om[4 * h + wv] = pad_mask(n, 4 * h + wv);
        }
      }
      __syncthreads();
      enc_store(reinterpret_cast<uint64_t *>(msg + o), w, ownf, nw, s_om, s_nm);
      uint32_t L = 0;
      for (int q = 0; q < 8; q++) L += __popcll(s_nm[q]);
      o += 128 + 8ull * L;
      __syncthreads();
    }
  }
}

// Return messages (gx.h "return"): for every block the partner leads, this side's words for the
// partner's merge; own slots where merging them would act exactly like the partner's own word.
// COUNT: sizes only (rsz[k]); else the messages at roff[k] and their size-table entries.
GXD bool ret_own(const Dev &d, uint64_t x, uint64_t y) {
  const bool xa = st_of(x) == GX_ABSENT, ya = st_of(y) == GX_ABSENT;
  if (xa || ya) return xa && ya;
  const int64_t thr = d.now - d.p.tombstone_lifespan_ns - d.p.stale_fudge_ns;
  const bool sx = ts_of(x) < thr, sy = ts_of(y) < thr;
  if (sy) return sx;
  return !sx && ts_of(y) <= ts_of(x);
}
// ---- wave-per-block lead and return encoding (nblk <= XS_MAXB) --------------------------------
// Every lead (follow) block's message offset is computed up front by a block scan into LDS, then
// the four waves encode blocks side by side with no barrier between blocks. Slot s of a block is
// lane s % 64 of word s / 64, so the own and neu mask words are plain wave ballots.
GXD uint64_t lanes_below(uint32_t lane) { return (1ull << lane) - 1ull; }
// a wave writes one encoded block: masks from lane 0, literals from the lanes that start a run
GXD void wave_enc_store(uint64_t *enc, const uint64_t *w, const bool *nwf, const uint64_t *om, const uint64_t *nm,
                        uint32_t lane) {
  uint32_t base = 0;
#pragma unroll
  for (int q = 0; q < 8; q++) {
    if (nwf[q]) enc[16 + base + __popcll(nm[q] & lanes_below(lane))] = w[q];
    base += __popcll(nm[q]);
  }
  if (lane < 8) {
    uint64_t a = 0, b = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      a = lane == (uint32_t)q ? om[q] : a;
      b = lane == (uint32_t)q ? nm[q] : b;
    }
    enc[lane] = a;
    enc[8 + lane] = b;
  }
}
__global__ __launch_bounds__(256) void k_ae_lead_pack_w(Dev d, const uint32_t *host, const uint32_t *pair_t,
                                                         const uint32_t *lmask, const uint32_t *nlead,
                                                         const uint64_t *off, uint32_t nmw, const ulonglong2 *own,
                                                         uint32_t nblk, uint8_t *out) {
  __shared__ uint32_t s_off[XS_MAXB];
  __shared__ uint16_t s_blk[XS_MAXB];
  __shared__ unsigned long long s_wave[4];
  const uint32_t k = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  uint8_t *msg = out + off[k];
  if (t == 0) {
    uint32_t *hdr = reinterpret_cast<uint32_t *>(msg);
    hdr[0] = pair_t[k];
    hdr[1] = host[k];
    hdr[2] = nlead[k];
    hdr[3] = 0;
  }
  const uint32_t *lm = lmask + (size_t)k * nmw;
  const ulonglong2 *dg = own + (size_t)k * nblk;
  const uint32_t c = (nblk + blockDim.x - 1) / blockDim.x, b0 = t * c, b1 = b0 + c < nblk ? b0 + c : nblk;
  uint32_t nl = 0, sz = 0;
  for (uint32_t b = b0; b < b1; b++)
    if ((lm[b >> 5] >> (b & 31)) & 1u) {
      nl++;
      sz += 128 + 8u * (uint32_t)(dg[b].y >> 54);  // the block's literal count (digest pass)
    }
  unsigned long long tot;
  const unsigned long long pre = block_excl_scan64((unsigned long long)nl | ((unsigned long long)sz << 32), s_wave, tot);
  uint32_t j = (uint32_t)pre, o = (uint32_t)(pre >> 32);
  for (uint32_t b = b0; b < b1; b++)
    if ((lm[b >> 5] >> (b & 31)) & 1u) {
      s_blk[j] = (uint16_t)b;
      s_off[j++] = o;
      o += 128 + 8u * (uint32_t)(dg[b].y >> 54);
    }
  __syncthreads();
  const uint32_t n_lead = (uint32_t)tot;
  const uint64_t *row = vrow(d, host[k]);
  for (uint32_t jj = wv; jj < n_lead; jj += 4) {
    const uint32_t b = s_blk[jj], lo = b * GX_DIGEST_SLOTS;
    const uint32_t nv = lo + GX_DIGEST_SLOTS <= d.R ? GX_DIGEST_SLOTS : d.R - lo;
    uint64_t w[8], om[8], nm[8];
    bool nwf[8];
#pragma unroll
    for (int q = 0; q < 8; q++) w[q] = 64u * q + lane < nv ? row[lo + 64u * q + lane] : 0;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint32_t sl = 64u * q + lane;
      uint64_t pw = __shfl_up(w[q], 1, 64);
      const uint64_t carry = q ? __shfl(w[q - 1], 63, 64) : 0;  // every lane shuffles (lane 63 must be active)
      if (lane == 0) pw = carry;
      const bool v = sl < nv;
      nwf[q] = v && (sl == 0 || w[q] != pw);
      om[q] = __ballot(!v);
      nm[q] = __ballot(nwf[q]);
    }
    wave_enc_store(reinterpret_cast<uint64_t *>(msg + 16 + s_off[jj]), w, nwf, om, nm, lane);
  }
}
// COUNT: the return message sizes (rsz) and every block's literal count (retL, in follow order);
// the pack pass lays the blocks out from those counts.
template <bool COUNT>
__global__ __launch_bounds__(256) void k_ae_ret_w(Dev d, const uint32_t *host, const uint32_t *pair_t,
                                                   const uint32_t *fmask, const uint32_t *nfol, const uint16_t *lt,
                                                   const uint8_t *lead, const uint64_t *ioff, uint32_t nblk,
                                                   uint32_t nmw, uint64_t *rsz, const uint64_t *roff,
                                                   const uint64_t *rtab, uint8_t *out, uint16_t *retL) {
  __shared__ uint32_t s_li[XS_MAXB], s_ro[XS_MAXB];
  __shared__ uint16_t s_blk[XS_MAXB];
  __shared__ unsigned long long s_wave[4];
  __shared__ unsigned long long s_sum;
  const uint32_t k = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint32_t nf = nfol[k];
  const uint8_t *lm = lead + ioff[k];
  uint8_t *msg = COUNT ? nullptr : out + roff[k];
  uint16_t *rl = retL + (size_t)k * nblk;
  const uint32_t hdr_bytes = 16 + 4u * (nf + (nf & 1u));
  if (t == 0) {
    s_sum = 0;
    if (!COUNT) {
      uint32_t *hdr = reinterpret_cast<uint32_t *>(msg);
      hdr[0] = pair_t[k];
      hdr[1] = host[k];
      hdr[2] = nf;
      hdr[3] = 0;
      if (nf & 1u) hdr[4 + nf] = 0;
      *reinterpret_cast<uint64_t *>(out + rtab[k]) = rsz[k];
    }
  }
  const uint32_t *fm = fmask + (size_t)k * nmw;
  const uint16_t *plt = lt + (size_t)k * nblk;
  const uint32_t c = (nblk + blockDim.x - 1) / blockDim.x, b0 = t * c, b1 = b0 + c < nblk ? b0 + c : nblk;
  uint32_t n = 0, lsz = 0;
  for (uint32_t b = b0; b < b1; b++)
    if ((fm[b >> 5] >> (b & 31)) & 1u) {
      n++;
      lsz += 128 + 8u * plt[b];
    }
  unsigned long long tot;
  const unsigned long long pre = block_excl_scan64((unsigned long long)n | ((unsigned long long)lsz << 32), s_wave, tot);
  uint32_t j = (uint32_t)pre, li_ = 16 + (uint32_t)(pre >> 32);
  const uint32_t j0 = j;
  uint32_t rs = 0;
  for (uint32_t b = b0; b < b1; b++)
    if ((fm[b >> 5] >> (b & 31)) & 1u) {
      s_blk[j] = (uint16_t)b;
      s_li[j] = li_;
      li_ += 128 + 8u * plt[b];
      if (!COUNT) rs += 128 + 8u * rl[j];
      j++;
    }
  if (!COUNT) {
    const unsigned long long rpre = block_excl_scan64(rs, s_wave, tot);
    uint32_t ro = hdr_bytes + (uint32_t)rpre;
    for (uint32_t q = j0; q < j; q++) {
      s_ro[q] = ro;
      ro += 128 + 8u * rl[q];
    }
  }
  __syncthreads();
  const uint64_t *row = vrow(d, host[k]);
  unsigned long long wsum = 0;
  for (uint32_t jj = wv; jj < nf; jj += 4) {
    const uint32_t b = s_blk[jj], lo = b * GX_DIGEST_SLOTS;
    const uint32_t nv = lo + GX_DIGEST_SLOTS <= d.R ? GX_DIGEST_SLOTS : d.R - lo;
    const uint64_t *xe = reinterpret_cast<const uint64_t *>(lm + s_li[jj]);  // the partner's lead block
    uint64_t xm[8], y[8], om[8], nm[8];
    bool ownf[8], nwf[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
      xm[q] = xe[8 + q];
      y[q] = 64u * q + lane < nv ? row[lo + 64u * q + lane] : 0;
    }
    uint32_t base = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const bool v = 64u * q + lane < nv;
      // the partner's word: the literal of the run holding this slot (its own bits are padding)
      const uint32_t rank = base + __popcll(xm[q] & ((2ull << lane) - 1ull)) - 1;
      ownf[q] = !v || ret_own(d, xe[16 + rank], y[q]);
      base += __popcll(xm[q]);
      om[q] = __ballot(ownf[q]);
    }
    uint32_t L = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint32_t sl = 64u * q + lane;
      uint64_t yp = __shfl_up(y[q], 1, 64);
      const uint64_t carry = q ? __shfl(y[q - 1], 63, 64) : 0;
      if (lane == 0) yp = carry;
      const bool op = sl == 0 || (lane ? (om[q] >> (lane - 1)) & 1ull : (q ? om[q - 1] >> 63 : 1ull));
      nwf[q] = !ownf[q] && (op || y[q] != yp);
      nm[q] = __ballot(nwf[q]);
      L += __popcll(nm[q]);
    }
    if (COUNT) {
      if (lane == 0) rl[jj] = (uint16_t)L;
      wsum += 128 + 8ull * L;
    } else {
      wave_enc_store(reinterpret_cast<uint64_t *>(msg + s_ro[jj]), y, nwf, om, nm, lane);
      if (lane == 0) reinterpret_cast<uint32_t *>(msg + 16)[jj] = L;
    }
  }
  if (COUNT) {
    if (lane == 0 && wsum) atomicAdd(&s_sum, wsum);
    __syncthreads();
    if (t == 0) rsz[k] = hdr_bytes + s_sum;
  }
}

template <bool COUNT>
__global__ __launch_bounds__(256) void k_ae_ret(Dev d, const uint32_t *host, const uint32_t *pair_t,
                                                 const uint32_t *fmask, const uint32_t *nfol, const uint16_t *lt,
                                                 const uint8_t *lead, const uint64_t *ioff, uint32_t nblk,
                                                 uint32_t nmw, uint64_t *rsz, const uint64_t *roff,
                                                 const uint64_t *rtab, uint8_t *out) {
  __shared__ unsigned long long s_om[8], s_nm[8], s_xm[8];
  const uint32_t k = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint32_t nf = nfol[k];
  const uint8_t *lm = lead + ioff[k];
  uint8_t *msg = COUNT ? nullptr : out + roff[k];
  if (!COUNT && t == 0) {
    uint32_t *hdr = reinterpret_cast<uint32_t *>(msg);
    hdr[0] = pair_t[k];
    hdr[1] = host[k];
    hdr[2] = nf;
    hdr[3] = 0;
    if (nf & 1u) hdr[4 + nf] = 0;
    *reinterpret_cast<uint64_t *>(out + rtab[k]) = rsz[k];
  }
  const uint64_t *row = vrow(d, host[k]);
  uint64_t li = 16, o = 16 + 4ull * (nf + (nf & 1u));
  uint32_t j = 0;
  for (uint32_t mw = 0; mw < nmw; mw++) {
    uint32_t bits = fmask[(size_t)k * nmw + mw];
    while (bits) {
      const uint32_t blk = mw * 32 + (uint32_t)__builtin_ctz(bits);
      bits &= bits - 1;
      const uint32_t lo = blk * GX_DIGEST_SLOTS, n = lo + GX_DIGEST_SLOTS <= d.R ? GX_DIGEST_SLOTS : d.R - lo;
      const uint64_t *xe = reinterpret_cast<const uint64_t *>(lm + li);  // the partner's lead block
      li += 128 + 8ull * lt[(size_t)k * nblk + blk];
      if (t < 8) s_xm[t] = xe[8 + t];
      __syncthreads();
      uint64_t y[2];
      bool ownf[2], nw[2];
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const uint32_t s = 256 * h + t, wi = 4 * h + wv;
        const bool v = s < n;
        y[h] = v ? row[lo + s] : 0;
        ownf[h] = true;
        if (v) {
          uint32_t rank = __popcll(s_xm[wi] & ((2ull << lane) - 1ull)) - 1;
          for (uint32_t q = 0; q < wi; q++) rank += __popcll(s_xm[q]);
          ownf[h] = ret_own(d, xe[16 + rank], y[h]);
        }
        const unsigned long long m = __ballot(ownf[h]);
        if (lane == 0) s_om[wi] = m;
      }
      __syncthreads();
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const uint32_t s = 256 * h + t;
        const bool op = s == 0 || ((s_om[(s - 1) >> 6] >> ((s - 1) & 63)) & 1ull);
        const uint64_t yp = s > 0 && s - 1 < n ? row[lo + s - 1] : 0;
        nw[h] = !ownf[h] && (op || y[h] != yp);
        const unsigned long long m = __ballot(nw[h]);
        if (lane == 0) s_nm[4 * h + wv] = m;
      }
      __syncthreads();
      uint32_t L = 0;
      for (int q = 0; q < 8; q++) L += __popcll(s_nm[q]);
      if (!COUNT) {
        enc_store(reinterpret_cast<uint64_t *>(msg + o), y, ownf, nw, s_om, s_nm);
        if (t == 0) reinterpret_cast<uint32_t *>(msg + 16)[j] = L;
      }
      o += 128 + 8ull * L;
      j++;
      __syncthreads();
    }
  }
  if (COUNT && t == 0) rsz[k] = o;
}

// Outbox plan on the device: block g lists, in entry order, this shard's packets (records or
// memberlist messages) whose receiver lives on shard g, after those bound for shards < g; the
// receiver's shard as in the host's contiguous blocks (floor(g * H / G)).
GXD uint32_t ob_dest(const Dev &d, size_t i) {
  const uint32_t len = d.msg_len[i], nfd = d.p.fd_enable ? d.fd_len[i] : 0u, dst = d.msg_dst[i];
  if (!(len || nfd) || (dst >= d.lo && dst < d.lo + d.Hl)) return d.G;
  uint32_t g = 0;
  while (g + 1 < d.G && (uint32_t)(((uint64_t)(g + 1) * d.H) / d.G) <= dst) g++;
  return g;
}
// Three launches over 256-entry chunks: per-chunk counts per shard, one block scans them into
// offsets (shard-major, chunk order), then each chunk places its entries by wave ballots.
GXD void ob_chunk_counts(const Dev &d, uint32_t gi, uint32_t *s_cnt) {  // s_cnt[4][G]
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (uint32_t g = 0; g < d.G; g++) {
    const unsigned long long m = __ballot(gi == g);
    if (lane == 0) s_cnt[wv * d.G + g] = (uint32_t)__popcll(m);
  }
}
__global__ __launch_bounds__(256) void k_ob_count(Dev d, uint32_t *cnt) {  // cnt[chunk][G]
  extern __shared__ uint32_t s_cnt[];
  const size_t ne = (size_t)d.Hl * d.KE, i = (size_t)blockIdx.x * 256 + threadIdx.x;
  ob_chunk_counts(d, i < ne ? ob_dest(d, i) : d.G, s_cnt);
  __syncthreads();
  if (threadIdx.x < d.G) {
    const uint32_t g = threadIdx.x;
    cnt[(size_t)blockIdx.x * d.G + g] = s_cnt[g] + s_cnt[d.G + g] + s_cnt[2 * d.G + g] + s_cnt[3 * d.G + g];
  }
}
// off[chunk][g] = entries bound for shards < g + entries for g in earlier chunks; tot[g] per shard
__global__ __launch_bounds__(256) void k_ob_scan(Dev d, const uint32_t *cnt, uint32_t nchunk, uint32_t *off,
                                                  uint32_t *tot) {
  __shared__ unsigned long long s_wave[4];
  unsigned long long base = 0;
  for (uint32_t g = 0; g < d.G; g++) {
    unsigned long long run = base;
    for (uint32_t c0 = 0; c0 < nchunk; c0 += blockDim.x) {
      const uint32_t c = c0 + threadIdx.x;
      const unsigned long long x = c < nchunk ? cnt[(size_t)c * d.G + g] : 0;
      unsigned long long t;
      const unsigned long long pre = block_excl_scan64(x, s_wave, t);
      if (c < nchunk) off[(size_t)c * d.G + g] = (uint32_t)(run + pre);
      run += t;
    }
    if (threadIdx.x == 0) tot[g] = (uint32_t)(run - base);
    base = run;
  }
}
__global__ __launch_bounds__(256) void k_ob_fill(Dev d, const uint32_t *off, uint32_t *entries) {
  extern __shared__ uint32_t s_cnt[];
  const size_t ne = (size_t)d.Hl * d.KE, i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t gi = i < ne ? ob_dest(d, i) : d.G;
  ob_chunk_counts(d, gi, s_cnt);
  __syncthreads();
  unsigned long long mine = 0;
  for (uint32_t g = 0; g < d.G; g++) {
    const unsigned long long b = __ballot(gi == g);
    if (gi == g) mine = b;
  }
  if (gi < d.G) {
    uint32_t rank = (uint32_t)__popcll(mine & ((1ull << lane) - 1ull));
    for (uint32_t w = 0; w < wv; w++) rank += s_cnt[w * d.G + gi];
    entries[off[(size_t)blockIdx.x * d.G + gi] + rank] = (uint32_t)i;
  }
}

// Outbox: fixed-size slots (16-B header + packet_cap records); slot index per local entry.
// gx_outbox_sizes_async: bytes per destination shard and the slot total, from k_ob_scan's counts
__global__ void k_ob_bytes(Dev d, const uint32_t *tot, unsigned long long *bytes, uint32_t *n_out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const uint64_t sb = 16 + 16ull * d.p.packet_cap + 16ull * (d.p.fd_enable ? d.p.fd_msg_cap : 0);
  uint32_t n = 0;
  for (uint32_t g = 0; g < d.G; g++) {
    bytes[g] = (unsigned long long)tot[g] * sb;
    n += tot[g];
  }
  *n_out = n;
}
// One packet slot (message entry e) into the wire buffer at dst (a 64-thread block).
GXD void pack_slot(const Dev &d, uint32_t e, uint8_t *dst) {
  const uint32_t fcap = d.p.fd_enable ? d.p.fd_msg_cap : 0;
  uint32_t len = d.msg_len[e], nfd = fcap ? d.fd_len[e] : 0;
  if (threadIdx.x == 0) {
    uint32_t *hdr = reinterpret_cast<uint32_t *>(dst);
    hdr[0] = d.msg_key[e];
    hdr[1] = d.msg_dst[e];
    hdr[2] = len;
    hdr[3] = nfd;
  }
  uint4 *fm = reinterpret_cast<uint4 *>(dst + 16 + 16ull * d.p.packet_cap);  // memberlist messages
  for (uint32_t x = threadIdx.x; x < fcap; x += blockDim.x) {
    uint4 w = make_uint4(0, 0, 0, 0);
    if (x < nfd) {
      const gx_fd_msg g = d.fdm[(size_t)e * fcap + x];
      w = make_uint4(g.incarnation, (uint32_t)g.node | ((uint32_t)g.from << 16), g.kind, 0);
    }
    fm[x] = w;
  }
  grec *recs = reinterpret_cast<grec *>(dst + 16);
  for (uint32_t x = threadIdx.x; x < d.p.packet_cap; x += blockDim.x) {
    grec g;
    if (x < len) {
      g = d.msg[(size_t)e * d.p.packet_cap + x];
    } else {
      g.w = 0;
      g.r = 0;
      g.pad = 0;
    }
    recs[x] = g;
  }
}
// n_dev: the slot count on the device (gx_outbox_sizes_async); slots past cap_slots are refused
__global__ void k_outbox_pack(Dev d, const uint32_t *entry, uint32_t n, uint8_t *out, const uint32_t *n_dev = nullptr,
                              uint32_t cap_slots = 0xffffffffu) {
  uint32_t i = blockIdx.x;
  if (n_dev) {
    n = *n_dev;
    if (i == 0 && threadIdx.x == 0 && n > cap_slots) atomicOr(&d.work_cnt[GX_WC_ERR], GX_ERR_INBOX);
    if (n > cap_slots) n = cap_slots;
  }
  if (i >= n) return;
  const size_t sb = 16 + 16ull * d.p.packet_cap + 16ull * (d.p.fd_enable ? d.p.fd_msg_cap : 0);
  pack_slot(d, entry[i], out + (size_t)i * sb);
}

// ------------------------------------------------------------ planned gossip exchange --
// Packet-slot bounds of the exchange, from the seeded sampler alone (gx_exchange_plan): for every
// round r of a batch and host u of the cluster, GossipMessages slots per sampled peer on another
// shard, counted per (shard of u, shard of the peer). Every shard computes the same matrix, so the
// collective's split sizes are known without waiting for the device.
struct XBound {
  uint32_t n[XPLAN_GMAX];  // slots this shard sends each shard this round
};
__global__ __launch_bounds__(256) void k_xplan(Dev d, int64_t r0, uint32_t *cnt) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x, rr = blockIdx.y;
  if (u >= d.H) return;
  const int64_t round = r0 + rr;
  // sample_peers of that round (its partition state)
  uint32_t base = 0, m = d.H;
  if (round >= d.p.partition_start && round < d.p.partition_end) {
    const uint32_t half = d.H / 2;
    base = u < half ? 0 : half;
    m = u < half ? half : d.H - half;
  }
  if (m < 2) return;
  const uint64_t h3 = mix64(mix64(mix64(d.p.seed ^ ((uint64_t)ST_PEER * 0xD1B54A32D192ED03ull)) ^ (uint64_t)round) ^ u);
  const uint32_t want = d.K < m - 1 ? d.K : m - 1, su = shard_of_d(d, u);
  uint32_t peers[16], c = 0;
  for (uint32_t at = 0; c < want && at < 64u * d.K; at++) {
    const uint32_t ix = unif(mix64(h3 ^ at), m - 1), self = u - base;
    const uint32_t p = base + (ix >= self ? ix + 1 : ix);
    bool dup = false;
    for (uint32_t i = 0; i < c; i++) dup |= peers[i] == p;
    if (!dup) peers[c++] = p;
  }
  for (uint32_t i = 0; i < c; i++) {
    const uint32_t sp = shard_of_d(d, peers[i]);
    if (sp != su) atomicAdd(&cnt[((size_t)rr * d.G + su) * d.G + sp], d.NG);
  }
}
// Slot i of the planned outbox: destination shard g's region holds bound.n[g] slots, its packets
// first (ob_fill's entries for g, tot[g] of them), then empty ones (sender key GX_SLOT_EMPTY).
__global__ void k_outbox_pack_planned(Dev d, const uint32_t *entry, const uint32_t *tot, XBound bound, uint8_t *out) {
  const uint32_t i = blockIdx.x;
  if (i == 0 && threadIdx.x == 0)  // every destination, also one whose region has no slot (cannot happen)
    for (uint32_t x = 0; x < d.G; x++)
      if (tot[x] > bound.n[x]) atomicOr(&d.work_cnt[GX_WC_ERR], GX_ERR_INBOX);
  uint32_t g = 0, acc = 0, eoff = 0;
  while (g < d.G && i >= acc + bound.n[g]) {
    acc += bound.n[g];
    eoff += tot[g];
    g++;
  }
  if (g >= d.G) return;
  const uint32_t j = i - acc;
  const size_t sb = 16 + 16ull * d.p.packet_cap + 16ull * (d.p.fd_enable ? d.p.fd_msg_cap : 0);
  uint8_t *dst = out + (size_t)i * sb;
  if (j < tot[g]) {
    pack_slot(d, entry[eoff + j], dst);
  } else if (threadIdx.x == 0) {
    uint32_t *hdr = reinterpret_cast<uint32_t *>(dst);
    hdr[0] = GX_SLOT_EMPTY;
    hdr[1] = hdr[2] = hdr[3] = 0;
  }
}

// Inbox: received slots -> message entries [Hl*K, Hl*K + n), registered in the receivers'
// inboxes. A slot is checked like the oracle's gx_inbox_unpack does: sender key < H*K and its
// sender on another shard, the key not seen before this round (one key per sender packet entry;
// a repeated key would give the merge two headers of equal rank), receiver on this shard, len <=
// packet_cap, n_fd <= fd_msg_cap, record keys < R. A bad slot is skipped and flagged
// (work_cnt[GX_WC_ERR]), and the next call that waits returns GX_EINVAL.
__global__ void k_inbox_unpack(Dev d, const uint8_t *in, uint32_t n) {
  uint32_t i = blockIdx.x;
  if (i >= n) return;
  const uint32_t fcap = d.p.fd_enable ? d.p.fd_msg_cap : 0;
  size_t sb = 16 + 16ull * d.p.packet_cap + 16ull * fcap;
  const uint8_t *src = in + (size_t)i * sb;
  const uint32_t *hdr = reinterpret_cast<const uint32_t *>(src);
  uint32_t key = hdr[0], dst = hdr[1], len = hdr[2], nfd = fcap ? hdr[3] : 0;
  if (key == GX_SLOT_EMPTY) return;  // an unused slot of a planned exchange (gx_outbox_pack_planned)
  size_t e = (size_t)d.Hl * d.KE + i;
  const grec *recs = reinterpret_cast<const grec *>(src + 16);
  bool bad = key >= d.H * d.KE || key / d.KE - d.lo < d.Hl || dst - d.lo >= d.Hl || len > d.p.packet_cap ||
             nfd > fcap;
  for (uint32_t x = threadIdx.x; !bad && x < len; x += blockDim.x) bad |= recs[x].r >= d.R;
  if (__ballot(bad) == 0) {  // a key seen twice this round: the later slot is refused
    const uint32_t stamp = (uint32_t)d.round + 1u;
    uint32_t dup = 0;
    if (threadIdx.x == 0) dup = atomicExch(&d.in_stamp[key], stamp) == stamp;
    bad = __shfl(dup, 0, 64) != 0;
  }
  if (bad) {
    if (threadIdx.x == 0) atomicOr(&d.work_cnt[GX_WC_ERR], GX_ERR_INBOX);
    return;
  }
  const uint32_t vi = dst - d.lo;
  // the receiver holds the ServicesState lock this round (gx.h lock_model): every record goes to
  // its pipeline unfiltered (k_merge_seg); lock_model = 0 merges them and counts them as locked
  const uint32_t rlw = gld(&d.hs[dst - d.lo].lock);
  const bool rlk = locked_in(d, rlw);
  if (rlk && threadIdx.x == 0 && len) {
    atomicMin(&d.ctr->first_drop[shard_id()][1], (unsigned long long)d.round);
    if (!d.p.lock_model) ctr_atomic(d, C_LOCKED_MERGES, len);
  }
  if (rlk && d.p.lock_model && GX_LOCK_BUF(rlw) >= d.C) {  // a full pipeline drops the records (send_planned)
    if (threadIdx.x == 0) {
      ctr_atomic(d, C_LOCK_DROP, len);
      d.msg_key[e] = key;
      d.msg_dst[e] = dst;
      d.msg_len[e] = 0;
      if (fcap) d.fd_len[e] = nfd;
    }
    const uint4 *fm = reinterpret_cast<const uint4 *>(src + 16 + 16ull * d.p.packet_cap);
    for (uint32_t x = threadIdx.x; x < nfd; x += blockDim.x) {
      const uint4 w = fm[x];
      gx_fd_msg g;
      g.incarnation = w.x;
      g.node = (uint16_t)(w.y & 0xffffu);
      g.from = (uint16_t)(w.y >> 16);
      g.kind = (uint8_t)w.z;
      g.pad[0] = g.pad[1] = g.pad[2] = 0;
      d.fdm[e * fcap + x] = g;
    }
    if (nfd && threadIdx.x == 0) inbox_header(d, dst - d.lo, inbox_claim(d, dst - d.lo), key, (uint32_t)e, 0u);
    return;
  }
  if (d.sfilt && !(rlk && d.p.lock_model)) {  // the receiver's filter: only live records are kept (compacted, see send_planned)
    const uint64_t *row = &d.view[(size_t)vi * d.R];
    const int64_t t_stale = d.now - d.p.tombstone_lifespan_ns - d.p.stale_fudge_ns;
    const int64_t t_gc = d.now - d.p.tombstone_lifespan_ns;
    grec *pk = &d.msg[e * d.p.packet_cap];
    uint32_t nlive = 0, nstale = 0;
    for (uint32_t x0 = 0; x0 < len; x0 += 64) {
      const uint32_t x = x0 + threadIdx.x;
      grec g;
      g.w = 0;
      g.r = 0;
      g.pad = 0;
      bool live = false;
      uint64_t w0 = 0;
      if (x < len) {
        g = recs[x];
        w0 = row[g.r];
        const int64_t ts = ts_of(g.w);
        const bool stale = ts < t_stale;
        const bool gc = st_of(w0) == GX_TOMBSTONE && ts_of(w0) < t_gc;
        live = !stale && (st_of(w0) == GX_ABSENT || ts > ts_of(w0) || gc);
        nstale += stale;
      }
      const unsigned long long m = __ballot(live);
      if (live) {
        const uint32_t at = nlive + (uint32_t)__popcll(m & ((1ull << threadIdx.x) - 1ull));
        pk[at] = g;
        d.msg_w0[e * d.p.packet_cap + at] = w0;
      }
      nlive += (uint32_t)__popcll(m);
    }
    nstale = (uint32_t)wave_sum(nstale);
    const uint4 *fm = reinterpret_cast<const uint4 *>(src + 16 + 16ull * d.p.packet_cap);
    for (uint32_t x = threadIdx.x; x < nfd; x += blockDim.x) {
      const uint4 w = fm[x];
      gx_fd_msg g;
      g.incarnation = w.x;
      g.node = (uint16_t)(w.y & 0xffffu);
      g.from = (uint16_t)(w.y >> 16);
      g.kind = (uint8_t)w.z;
      g.pad[0] = g.pad[1] = g.pad[2] = 0;
      d.fdm[e * fcap + x] = g;
    }
    if (threadIdx.x == 0) {
      d.msg_key[e] = key;
      d.msg_dst[e] = dst;
      d.msg_len[e] = nlive;
      if (fcap) d.fd_len[e] = nfd;
      if (nlive || nfd) inbox_header(d, vi, inbox_claim(d, vi), key, (uint32_t)e, nlive, GX_NOSLOT_W0);
      if (nlive) flag_live(d, vi, nlive);
      ctr_atomic(d, C_GOSSIP_MERGES, len);
      ctr_atomic(d, C_STALE, nstale);
      // 16 B per slot read, 8 B per receiver slot, 16 B per live record written, header + count
      kbytes(d, GX_K_MERGE, 16ull + 24ull * len + 16ull * nlive + ((nlive || nfd) ? 20ull : 0ull), 0);
    }
    return;
  }
  uint32_t pos = 0;
  if (threadIdx.x == 0 && (len || nfd)) pos = inbox_claim(d, vi);
  pos = __shfl(pos, 0, 64);
  grec *pk = (len || nfd) ? packet_recs(d, vi, pos, (uint32_t)e) : &d.msg[e * d.p.packet_cap];
  for (uint32_t x = threadIdx.x; x < len; x += blockDim.x) pk[x] = recs[x];
  const uint4 *fm = reinterpret_cast<const uint4 *>(src + 16 + 16ull * d.p.packet_cap);
  for (uint32_t x = threadIdx.x; x < nfd; x += blockDim.x) {
    const uint4 w = fm[x];
    gx_fd_msg g;
    g.incarnation = w.x;
    g.node = (uint16_t)(w.y & 0xffffu);
    g.from = (uint16_t)(w.y >> 16);
    g.kind = (uint8_t)w.z;
    g.pad[0] = g.pad[1] = g.pad[2] = 0;
    d.fdm[e * fcap + x] = g;
  }
  if (threadIdx.x == 0) {
    d.msg_key[e] = key;
    d.msg_dst[e] = dst;
    d.msg_len[e] = len;
    if (fcap) d.fd_len[e] = nfd;
    if (len || nfd) inbox_header(d, vi, pos, key, (uint32_t)e, len);
    if (rlk && d.sfilt && len) flag_live(d, vi, len);  // routes the locked receiver
  }
}

// Per-record min/max slot word over this shard's views, XOR 2^63 (signed-order reducible).
__global__ void k_view_minmax(Dev d, uint64_t *mn, uint64_t *mx) {
  uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= d.R) return;
  uint64_t a = ~0ull, b = 0;
  for (uint32_t v = 0; v < d.Hl; v++) {
    if (departed(d, d.lo + v)) continue;  // a crashed host's view is frozen and left out
    uint64_t w = d.view[(size_t)v * d.R + r];
    a = w < a ? w : a;
    b = w > b ? w : b;
  }
  mn[r] = a ^ (1ull << 63);
  mx[r] = b ^ (1ull << 63);
}

__global__ void k_owner_words(Dev d, uint64_t *out) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= d.R) return;
  const uint32_t o = owner_of(d, r);
  out[r] = o - d.lo < d.Hl ? d.view[(size_t)(o - d.lo) * d.R + r] : 0ull;
}

// ================================================================ convergence / digests ==
__global__ void k_converged(Dev d, unsigned long long *bad) {
  uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  bool dis = false;
  if (r < d.R) {  // the live views must agree; crashed hosts' views are left out
    uint32_t v0 = 0;
    while (v0 < d.Hl && departed(d, d.lo + v0)) v0++;
    uint64_t w0 = v0 < d.Hl ? d.view[(size_t)v0 * d.R + r] : 0;
    for (uint32_t v = v0 + 1; v < d.Hl; v++)
      if (!departed(d, d.lo + v) && d.view[(size_t)v * d.R + r] != w0) {
        dis = true;
        break;
      }
  }
  unsigned long long c = wave_sum(dis ? 1ull : 0ull);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(bad, c);
}

GXD uint64_t feed(uint64_t h, uint64_t x) { return mix64(h ^ x); }
GXD uint64_t feed_job(uint64_t h, const gx_job &j) {
  h = feed(h, j.a);
  return feed(h, (uint64_t)j.c | ((uint64_t)j.meta << 32));
}
__global__ void k_digest(Dev d, uint64_t *out) {
  uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;  // local index
  if (v >= d.Hl) return;
  const gx_host_state s = d.hs[v];
  uint64_t h = 0x243F6A8885A308D3ull;
  for (uint32_t i = s.fifo_head; i != s.fifo_stored; i++) h = feed_job(h, d.fifo[(size_t)v * d.Q + (i % d.Q)]);
  h = feed(h, 0xF1F0);
  h = feed(h, (uint64_t)(s.fifo_tail - s.fifo_stored) | ((uint64_t)s.fifo_stored << 32));
  for (uint32_t i = s.sleep_head; i != s.sleep_tail; i++) {
    const gx_sleeper z = d.sleep[(size_t)v * d.SQ + (i & (d.SQ - 1u))];
    h = feed(h, feed_job(z.wake, z.job));
  }
  h = feed(h, 0x51EE);
  h = feed(h, s.dq_len);
  for (uint32_t i = 0; i < s.dq_len; i++) {
    grec g = d.dq[(size_t)v * d.DQ + ((s.dq_head + i) & (d.DQ - 1))];
    h = feed(h, g.w);
    h = feed(h, g.r);
  }
  h = feed(h, 0xA7E4);
  for (uint32_t a = 0; a < d.A; a++) {
    if (!((d.arena_bits[(size_t)v * d.AW + (a >> 5)] >> (a & 31)) & 1u)) continue;
    uint32_t len = d.arena_len[(size_t)v * d.A + a];
    h = feed(h, a);
    h = feed(h, len);
    for (uint32_t i = 0; i < len; i++) {
      grec g = d.arena[((size_t)v * d.A + a) * d.L + i];
      h = feed(h, g.w);
      h = feed(h, g.r);
    }
  }
  h = feed(h, 0x10C6);  // the lock buffer, then the owners whose ExpireServer waits (gx.h lock_model)
  for (uint32_t k = 0; k < GX_LOCK_BUF(s.lock); k++) {
    const grec g = d.lkb[(size_t)v * d.C + k];
    h = feed(h, g.w);
    h = feed(h, g.r);
  }
  if (s.lock & GX_LOCK_PENDING_EXPIRE)
    for (uint32_t k = 0; k < d.PW; k++) {
      const uint32_t x = d.pexp[(size_t)v * d.PW + k];
      if (x) h = feed(h, (uint64_t)k << 32 | x);
    }
  h = feed(h, s.flags);
  h = feed(h, (uint64_t)s.bs_next);
  h = feed(h, (uint64_t)s.bt_next);
  h = feed(h, (uint64_t)s.last_bcast_ns);
  h = feed(h, s.running);
  out[v] = h;
}

// ============================================== catalog readers (EachServiceSorted, ByService) ==
// A view's present records (of one owner, or all: owner = 0xffffffff) compacted in key order: per
// 1024-slot chunk counts, one exclusive scan, then ordered writes by wave ballots.
#define VC_CHUNK 1024
GXD bool vc_take(const Dev &d, uint64_t w, uint32_t r, uint32_t owner) {
  return st_of(w) != GX_ABSENT && (owner == 0xffffffffu || owned_by(d, r, owner));
}
__global__ __launch_bounds__(256) void k_vc_count(Dev d, uint32_t vi, uint32_t owner, uint32_t *cnt) {
  __shared__ uint32_t s_n;
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  const uint64_t *row = &d.view[(size_t)vi * d.R];
  uint32_t n = 0;
  for (uint32_t k = threadIdx.x; k < VC_CHUNK; k += blockDim.x) {
    const uint32_t r = blockIdx.x * VC_CHUNK + k;
    n += r < d.R && vc_take(d, row[r], r, owner);
  }
  n = (uint32_t)wave_sum(n);
  if ((threadIdx.x & 63) == 0) atomicAdd(&s_n, n);
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = s_n;
}
__global__ __launch_bounds__(1024) void k_vc_scan(uint32_t *cnt, uint32_t nb) {  // exclusive, cnt[nb] = total
  __shared__ unsigned long long s_wave[16];
  unsigned long long carry = 0;
  for (uint32_t b0 = 0; b0 < nb; b0 += 1024) {
    const uint32_t b = b0 + threadIdx.x;
    const unsigned long long x = b < nb ? cnt[b] : 0;
    unsigned long long tot;
    const unsigned long long pre = block_excl_scan64(x, s_wave, tot);
    if (b < nb) cnt[b] = (uint32_t)(carry + pre);
    carry += tot;
  }
  if (threadIdx.x == 0) cnt[nb] = (uint32_t)carry;
}
__global__ __launch_bounds__(256) void k_vc_write(Dev d, uint32_t vi, uint32_t owner, const uint32_t *off,
                                                  uint64_t *keys, uint32_t *vals) {
  __shared__ uint32_t s_w[VC_CHUNK / 64];
  const uint64_t *row = &d.view[(size_t)vi * d.R];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t base = off[blockIdx.x];
  for (uint32_t k0 = 0; k0 < VC_CHUNK; k0 += blockDim.x) {
    const uint32_t r = blockIdx.x * VC_CHUNK + k0 + threadIdx.x;
    const uint64_t w = r < d.R ? row[r] : GX_SLOT_ABSENT;
    const bool t = r < d.R && vc_take(d, w, r, owner);
    const unsigned long long m = __ballot(t);
    if (lane == 0) s_w[wv] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t pre = 0, tot = 0;
    for (uint32_t q = 0; q < blockDim.x / 64; q++) {
      pre += q < wv ? s_w[q] : 0;
      tot += s_w[q];
    }
    if (t) {
      const uint32_t at = base + pre + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
      keys[at] = w >> GX_TS_SHIFT;  // Updated only: equal times keep key order (stable sort)
      vals[at] = r;
    }
    base += tot;
    __syncthreads();
  }
}
__global__ void k_vc_rank(const uint32_t *name_rank, const uint32_t *vals, uint32_t *keys, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) keys[i] = name_rank[vals[i]];
}
__global__ void k_vc_out(Dev d, uint32_t vi, const uint32_t *vals, uint32_t n, gx_service *out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t r = vals[i];
  const uint64_t w = d.view[(size_t)vi * d.R + r];
  gx_service g;
  g.updated_ns = ts_of(w) + d.epoch;
  g.host = r / d.S;
  g.svc = (uint16_t)(r % d.S);
  g.status = (uint8_t)st_of(w);
  g.flags = 0;
  out[i] = g;
}

// ========================================================= single-host ABI kernels (64 lanes) ==
// Lane 0 runs the scalar reference logic; all lanes join the counter flush.
__global__ void k_api_add(Dev d, const uint32_t *views, uint32_t fixed_view, const grec *recs, uint32_t n, int src,
                          uint32_t *acc_out) {
  Acc a;
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (uint32_t i = 0; i < n; i++) acc += add_entry(d, a, views ? views[i] : fixed_view, recs[i], src);
    *acc_out = acc;
  }
  acc_flush(d, a);
}
__global__ void k_api_expire(Dev d, uint32_t v, uint32_t o, uint32_t *out) {
  Acc a;
  if (threadIdx.x == 0) *out = expire_server(d, a, v, o);
  acc_flush(d, a);
}
__global__ void k_api_send(Dev d, uint32_t v, const grec *list, uint32_t n, uint32_t np) {
  Acc a;
  if (threadIdx.x == 0) {  // SendServices (services_state.go:579-604)
    a.c[C_SENDJOBS]++;
    const uint32_t m = n < d.L ? n : d.L;
    if (!fifo_stores(d, v)) {  // deferred: no list
      push_job(d, a, v, make_job(0, GX_LIST_NONE, meta_of(GX_JOB_SEND, 0, np)));
    } else {
      int slot = alloc_list(d, a, v);
      if (slot >= 0) {
        grec *dst = list_ptr(d, v, slot);
        for (uint32_t i = 0; i < m; i++) dst[i] = list[i];
      }
      commit_send(d, a, v, slot, m, np);
    }
  }
  acc_flush(d, a);
}
__global__ void k_api_bs(Dev d, uint32_t v, const grec *list, uint32_t n) {
  Acc a;
  if (threadIdx.x == 0) {
    uint64_t inc;
    bs_body_list(d, a, v, list, n, inc);
    gx_host_state *h = hst(d, v);
    h->lock = lock_snap(h->lock, h->flags, d.round, d.p.lock_readers != 0);  // a nil blocks the looper from now on
  }
  acc_flush(d, a);
}
__global__ void k_api_bt(Dev d, uint32_t v, uint64_t running, const grec *others, const uint32_t *n_others) {
  Acc a;
  if (threadIdx.x == 0) {
    uint32_t n = *n_others;
    bt_finish(d, a, v, running, others, n < d.L ? n : d.L);
    gx_host_state *h = hst(d, v);
    h->lock = lock_snap(h->lock, h->flags, d.round, d.p.lock_readers != 0);
  }
  acc_flush(d, a);
}
__global__ void k_api_tomb(Dev d, uint32_t v, uint64_t running, uint64_t *out_mask) {
  Acc a;
  if (threadIdx.x == 0) *out_mask = tombstone_services(d, a, v, running);
  acc_flush(d, a);
}
__global__ void k_api_getb(Dev d, uint32_t v, uint32_t limit, grec *out, uint32_t *n_out, uint32_t limit_bytes,
                           uint32_t overhead) {
  Acc a;
  gx_host_state hs = *hst(d, v);
  uint32_t l = get_broadcasts_team<64>(d, a, v, hs, limit, out, limit_bytes, overhead);
  hs.lock = lock_snap(hs.lock, hs.flags, d.round, d.p.lock_readers != 0);  // a looper's nil may have been taken
  if (threadIdx.x == 0) {
    *hst(d, v) = hs;
    *n_out = l;
  }
  acc_flush(d, a);
}
__global__ void k_api_msg_bytes(Dev d, const grec *recs, uint32_t n, uint32_t *out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = msg_bytes(d, recs[i]);
}
__global__ void k_fill_u16(uint16_t *p, size_t n, uint16_t v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}
// OR over this engine's views of the presence bits of owner o's S slots (gx_owner_slots_in_use):
// one thread per view, one atomic per wave.
__global__ void k_slots_in_use(Dev d, uint32_t o, unsigned long long *out) {
  const uint32_t vi = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long m = 0;
  if (vi < d.Hl) {
    const uint64_t *w = &d.view[(size_t)vi * d.R + (size_t)o * d.S];
    for (uint32_t s = 0; s < d.S; s++) m |= (unsigned long long)(st_of(w[s]) != GX_ABSENT) << s;
  }
  for (int k = 32; k > 0; k >>= 1) m |= __shfl_xor(m, k, 64);
  if ((threadIdx.x & 63) == 0 && m) atomicOr(out, m);
}
__global__ void k_api_is_new(Dev d, uint32_t v, uint64_t w, uint32_t r, uint32_t *out) {
  if (threadIdx.x == 0) *out = is_new(d, v, w, r);
}
__global__ void k_api_set_slot(Dev d, uint32_t v, uint32_t r, uint64_t w) {
  Acc a;
  if (threadIdx.x == 0) set_slot(d, a, v, &vrow(d, v)[r], w);
  acc_flush(d, a);
}
__global__ void k_api_mark(Dev d) {
  if (threadIdx.x == 0) mark_change(d);
}

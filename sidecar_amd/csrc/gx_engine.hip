// gx_engine.hip — sidecar-gx gossip-convergence engine for MI355X (gfx950).
//
// Implements include/gx.h. One engine object owns one GPU's slice of the simulated cluster and
// advances it one gossip round at a time (gx_run_rounds). Round phases and the kernels that run
// them (DESIGN.md "Round model", "Kernels"):
//   0+1 k_owner      wake re-armed SendServices passes; discovery churn; BroadcastServices tick
//                    (services_state.go:525-574) + TrackNewServices; flag BroadcastTombstones ticks
//   1   k_scan       TombstoneOthersServices full-view expiry scan (services_state.go:635-683),
//                    one 256-thread block streams one 4 MB view row, ordered compaction of tombstones
//   1   k_bt_finish  TombstoneServices + SendServices(TOMBSTONE_COUNT) or nil (services_state.go:606-633)
//   2   k_storm      NotifyLeave -> ExpireServer for every host of the other half (services_state.go:150-192)
//   3   k_send       peer sampling + GetBroadcasts/packPacket per peer (services_delegate.go:85-144,186-223)
//   3b  k_route_*    receiver-side CSR of this round's packets, sender-ordered (deterministic)
//   4   k_merge      gather-then-merge: one wave per receiver stages its inbound records in LDS,
//                    folds duplicates of a key in arrival order with the AddServiceEntry rule
//                    (services_state.go:293-347), writes each touched slot once, and compacts
//                    accepted foreign records into the receiver's broadcast FIFO with a wave ballot
//   5   k_ae         anti-entropy push-pull: one 256-thread block per host pair streams both views
//                    and merges each into the other (services_delegate.go:153-167, Merge :367-373)
// No MFMA: the work is int64 compare/select over HBM-resident views (memory-bound).
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "gx_device.hpp"

#define HIPCHK(x)                                                                          \
  do {                                                                                     \
    hipError_t _e = (x);                                                                   \
    if (_e != hipSuccess) {                                                                \
      fprintf(stderr, "gx: HIP error %s at %s:%d\n", hipGetErrorString(_e), __FILE__, __LINE__); \
      return GX_EIO;                                                                       \
    }                                                                                      \
  } while (0)

static uint32_t pow2_at_least(uint32_t x) {
  uint32_t v = 1;
  while (v < x) v <<= 1;
  return v;
}

// =============================================================================== kernels ==

// Ordered block-wide exclusive scan of a 0/1 flag (wave ballot + per-wave totals in LDS).
GXD uint32_t block_scan_flag(bool f, uint32_t *s_wave, uint32_t &total) {
  unsigned long long m = __ballot(f);
  uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  uint32_t pre = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
  if (lane == 0) s_wave[w] = (uint32_t)__popcll(m);
  __syncthreads();
  uint32_t off = 0, tot = 0;
  for (uint32_t i = 0; i < nw; i++) {
    uint32_t c = s_wave[i];
    if (i < w) off += c;
    tot += c;
  }
  __syncthreads();
  total = tot;
  return off + pre;
}

GXD unsigned long long wave_sum(unsigned long long x) {
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}

// Block reduction of a counter, then one atomic per block.
GXD void block_ctr(const Dev &d, int idx, unsigned long long x, unsigned long long *s_red) {
  x = wave_sum(x);
  uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  if (lane == 0) s_red[w] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (uint32_t i = 0; i < nw; i++) t += s_red[i];
    ctr_add(d, idx, t);
  }
  __syncthreads();
}

// -------------------------------------------------------------------------- init ---------
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
  size_t total = (size_t)d.H * d.R;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t v = (uint32_t)(i / d.R), r = (uint32_t)(i % d.R);
    uint64_t w = GX_SLOT_ABSENT;
    if (d.p.init_mode == GX_INIT_WARM || (d.p.init_mode == GX_INIT_OWN && r / d.S == v)) w = rec_word[r];
    d.view[i] = w;
  }
}

__global__ void k_init_hosts(Dev d) {
  uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= d.H) return;
  const gx_params &p = d.p;
  gx_host_state h = {};
  h.bs_next = (int64_t)(rng4(p.seed, ST_PHASE_BS, o, 0, 0) % p.alive_interval_rounds);
  h.bt_next = (int64_t)(rng4(p.seed, ST_PHASE_BT, o, 0, 0) % p.tombstone_interval_rounds);
  h.last_bcast_ns = p.init_mode == GX_INIT_WARM ? p.t0_ns : 0;
  h.running = d.S == 64 ? ~0ull : ((1ull << d.S) - 1);
  d.hs[o] = h;
  for (uint32_t s = 0; s < d.S; s++) d.own_status[(size_t)o * d.S + s] = GX_ALIVE;
}

__global__ void k_wake(Dev d) {
  uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v < d.H) wake_host(d, v);
}

// ---------------------------------------------------------------- phase 0+1: owner ticks --
__global__ __launch_bounds__(256) void k_owner(Dev d, grec *own_list) {
  uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= d.H) return;
  wake_host(d, o);
  gx_host_state *h = &d.hs[o];
  if (d.p.churn_ppm) {  // discovery churn: one service starts or stops
    uint64_t x = rng4(d.p.seed, ST_CHURN, (uint64_t)d.round, o, 0);
    if ((uint32_t)(x & 0xffffffffu) % 1000000u < d.p.churn_ppm) {
      uint32_t s = (uint32_t)((x >> 32) % d.S);
      h->running ^= 1ull << s;
      if ((h->running >> s) & 1ull) d.own_status[(size_t)o * d.S + s] = GX_ALIVE;
      ctr_add(d, C_CHURN, 1);
    }
  }
  if (!(h->flags & 1u) && h->bs_next <= d.round) {
    // fn(): the owner's running services, restamped by discovery at this tick
    grec *list = &own_list[(size_t)o * d.S];
    uint32_t n = 0;
    uint64_t run = h->running;
    for (uint32_t s = 0; s < d.S; s++)
      if ((run >> s) & 1ull) {
        list[n].w = pack(d.now, d.own_status[(size_t)o * d.S + s]);
        list[n].r = o * d.S + s;
        list[n].pad = 0;
        n++;
      }
    uint64_t inc = 0;
    bs_body_list(d, o, list, n, inc);
    if (inc) {
      h->bs_next = d.round + d.p.alive_interval_rounds;
      for (uint32_t i = 0; i < n; i++)
        if ((inc >> i) & 1ull) add_entry(d, o, list[i], SRC_LOCAL);  // TrackNewServices
    }
  }
  d.tick[o] = (!(h->flags & 2u) && h->bt_next <= d.round) ? 1 : 0;
}

// ------------------------------------------------- phase 1: TombstoneOthersServices scan --
// One 256-thread block per scanned view. list/cnt receive the first list_cap tombstoned records
// in key order and the total count.
__global__ __launch_bounds__(256) void k_scan(Dev d, grec *list_base, uint32_t list_stride, uint32_t list_cap,
                                               uint32_t *cnt_out, int only_host) {
  __shared__ uint32_t s_wave[4];
  __shared__ unsigned long long s_red[4];
  uint32_t o = only_host >= 0 ? (uint32_t)only_host : blockIdx.x;
  if (only_host < 0 && !d.tick[o]) return;
  uint64_t *row = &d.view[(size_t)o * d.R];
  grec *list = &list_base[only_host >= 0 ? 0 : (size_t)o * list_stride];
  uint32_t n_exp = 0;
  unsigned long long c_exp = 0, c_gc = 0;
  bool changed = false;
  unsigned long long c_wr = 0;
  for (uint32_t base = 0; base < d.R; base += blockDim.x) {
    uint32_t r = base + threadIdx.x;
    uint64_t w = r < d.R ? row[r] : GX_SLOT_ABSENT;
    bool ex, gc;
    uint64_t nw = expiry_word(d, w, ex, gc);
    if (nw != w) {
      row[r] = nw;
      changed = true;
      c_wr++;
    }
    c_exp += ex;
    c_gc += gc;
    uint32_t tot;
    uint32_t pos = block_scan_flag(ex, s_wave, tot);
    if (ex && n_exp + pos < list_cap) {
      grec g;
      g.w = nw;
      g.r = r;
      g.pad = 0;
      list[n_exp + pos] = g;
    }
    n_exp += tot;
  }
  if (threadIdx.x == 0) cnt_out[only_host >= 0 ? 0 : o] = n_exp;
  if (changed) mark_change(d);
  c_wr = wave_sum(c_wr);
  if ((threadIdx.x & 63) == 0) kbytes(d, GX_K_SCAN, c_wr * 8, 0);
  if (threadIdx.x == 0) kbytes(d, GX_K_SCAN, (unsigned long long)d.R * 8 + 16ull * (n_exp < list_cap ? n_exp : list_cap), d.R);
  block_ctr(d, C_EXPIRED, c_exp, s_red);
  block_ctr(d, C_GC, c_gc, s_red);
  block_ctr(d, C_SCANSLOTS, (threadIdx.x == 0) ? d.R : 0, s_red);
}

__global__ __launch_bounds__(256) void k_bt_finish(Dev d) {
  uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= d.H || !d.tick[o]) return;
  uint32_t n = d.scan_cnt[o];
  bt_finish(d, o, d.hs[o].running, &d.scan_list[(size_t)o * d.L], n < d.L ? n : d.L);
}

// ------------------------------------------------------------ phase 2: departure storm --
__global__ __launch_bounds__(256) void k_storm(Dev d) {
  __shared__ uint32_t s_wave[4];
  uint32_t v = blockIdx.x;
  uint32_t half = d.H / 2;
  uint32_t lo = v < half ? half : 0, hi = v < half ? d.H : half;
  gx_host_state *h = &d.hs[v];
  uint32_t tail0 = h->fifo_tail, count0 = tail0 - h->fifo_head;
  uint32_t room = count0 < d.Q - 2 ? d.Q - 2 - count0 : 0;
  uint32_t jobs = 0;
  bool changed = false;
  uint64_t tomb = pack(d.now, GX_TOMBSTONE);
  for (uint32_t base = lo; base < hi; base += blockDim.x) {
    uint32_t o = base + threadIdx.x;
    bool live = false;
    uint64_t mask = 0;
    if (o < hi) {
      uint64_t *row = &d.view[(size_t)v * d.R + (size_t)o * d.S];
      for (uint32_t s = 0; s < d.S; s++) {
        uint64_t w = row[s];
        if (st_of(w) == GX_ABSENT) continue;
        mask |= 1ull << s;
        if (st_of(w) != GX_TOMBSTONE) live = true;
      }
      if (live) {
        for (uint32_t s = 0; s < d.S; s++)
          if ((mask >> s) & 1ull && row[s] != tomb) {
            row[s] = tomb;
            changed = true;
          }
      }
    }
    uint32_t tot;
    uint32_t pos = block_scan_flag(live, s_wave, tot);
    if (live && jobs + pos < room) {
      gx_job j;
      j.a = (uint64_t)d.now;
      j.b = mask;
      j.c = o;
      j.meta = meta_of(GX_JOB_EXPIRE, 0, d.p.tombstone_count);
      j.wake = 0;
      j.aux = 0;
      d.fifo[(size_t)v * d.Q + ((tail0 + jobs + pos) % d.Q)] = j;
    }
    jobs += tot;
  }
  if (changed) mark_change(d);
  if (threadIdx.x == 0) {
    uint32_t ok = jobs < room ? jobs : room;
    h->fifo_tail = tail0 + ok;
    kbytes(d, GX_K_STORM, 8ull * (hi - lo) * d.S + 8ull * d.S * jobs + 32ull * ok, (unsigned long long)(hi - lo) * d.S);
    ctr_add(d, C_EXPSRV, jobs);
    ctr_add(d, C_QDROP, jobs - ok);
  }
}

// --------------------------------------------------------------------- phase 3: gossip send --
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

__global__ __launch_bounds__(256) void k_send(Dev d) {
  uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= d.H) return;
  uint32_t peers[16];
  uint32_t np = sample_peers(d, u, peers);
  uint32_t cap = d.p.packet_cap;
  for (uint32_t j = 0; j < d.K; j++) {
    d.msg_len[(size_t)u * d.K + j] = 0;
    d.msg_dst[(size_t)u * d.K + j] = 0xffffffffu;
  }
  for (uint32_t j = 0; j < np; j++) {
    uint32_t l = get_broadcasts(d, u, cap, &d.msg[((size_t)u * d.K + j) * cap]);
    d.msg_len[(size_t)u * d.K + j] = l;
    d.msg_dst[(size_t)u * d.K + j] = peers[j];
    if (l == 0 && d.p.gossip_stop_on_empty) break;
  }
}

// -------------------------------------------- phase 3b: receiver CSR, sender-ordered ------
__global__ void k_route_count(Dev d) {
  uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.H * d.K || d.msg_len[e] == 0) return;
  atomicAdd(&d.in_cnt[d.msg_dst[e]], 1u);
}

// Exclusive scan of H counts into in_cnt[0..H] (single block, 1024 threads).
__global__ __launch_bounds__(1024) void k_route_offsets(Dev d) {
  __shared__ uint32_t s_part[1024];
  uint32_t H = d.H, t = threadIdx.x;
  uint32_t per = (H + 1023) / 1024;
  uint32_t lo = t * per, hi = lo + per < H ? lo + per : H;
  uint32_t sum = 0;
  for (uint32_t i = lo; i < hi; i++) sum += d.in_cnt[i];
  s_part[t] = sum;
  __syncthreads();
  for (uint32_t off = 1; off < 1024; off <<= 1) {
    uint32_t x = t >= off ? s_part[t - off] : 0;
    __syncthreads();
    s_part[t] += x;
    __syncthreads();
  }
  uint32_t run = s_part[t] - sum;
  for (uint32_t i = lo; i < hi; i++) {
    uint32_t c = d.in_cnt[i];
    d.in_cnt[i] = run;
    run += c;
  }
  if (t == 1023) d.in_cnt[H] = s_part[1023];
}

__global__ void k_route_fill(Dev d) {
  uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.H * d.K || d.msg_len[e] == 0) return;
  uint32_t dst = d.msg_dst[e];
  uint32_t pos = atomicAdd(&d.in_cur[dst], 1u);
  d.in_fill[d.in_cnt[dst] + pos] = e;
}

// Deterministic order: rank of each entry (= sender * K + j) inside its receiver segment.
__global__ void k_route_rank(Dev d) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.in_cnt[d.H]) return;
  uint32_t e = d.in_fill[i];
  uint32_t dst = d.msg_dst[e];
  uint32_t lo = d.in_cnt[dst], hi = d.in_cnt[dst + 1];
  uint32_t rank = 0;
  for (uint32_t x = lo; x < hi; x++) rank += d.in_fill[x] < e;
  d.in_sorted[lo + rank] = e;
}

// ---------------------------------------------------------- phase 4: gather-then-merge --
#define MERGE_TILE 256
__global__ __launch_bounds__(64) void k_merge(Dev d) {
  __shared__ uint32_t s_key[MERGE_TILE];
  __shared__ uint64_t s_val[MERGE_TILE];
  __shared__ uint64_t s_acc[MERGE_TILE];
  __shared__ uint8_t s_accf[MERGE_TILE];
  __shared__ uint32_t s_start[65];
  __shared__ uint32_t s_ent[64];
  uint32_t v = blockIdx.x;
  uint32_t lane = threadIdx.x;
  uint32_t off = d.in_cnt[v], deg = d.in_cnt[v + 1] - off;
  if (deg == 0) return;
  uint32_t cap = d.p.packet_cap;
  gx_host_state *h = &d.hs[v];
  uint32_t tail0 = h->fifo_tail, count0 = tail0 - h->fifo_head;
  uint32_t room = count0 < d.Q - 2 ? d.Q - 2 - count0 : 0;
  uint32_t n_retx = 0;
  unsigned long long c_merge = 0, c_acc = 0, c_stale = 0, c_rd = 0, c_wr = 0;
  bool changed = false;
  uint64_t *row = &d.view[(size_t)v * d.R];
  for (uint32_t c0 = 0; c0 < deg; c0 += 64) {
    uint32_t cn = deg - c0 < 64 ? deg - c0 : 64;
    uint32_t ent = 0, len = 0;
    if (lane < cn) {
      ent = d.in_sorted[off + c0 + lane];
      len = d.msg_len[ent];
    }
    uint32_t incl = len;
    for (int o = 1; o < 64; o <<= 1) {
      uint32_t y = __shfl_up(incl, o, 64);
      if ((int)lane >= o) incl += y;
    }
    uint32_t total = __shfl(incl, 63, 64);
    s_start[lane] = incl - len;
    s_ent[lane] = ent;
    if (lane == 0) s_start[64] = total;
    __syncthreads();
    for (uint32_t t0 = 0; t0 < total; t0 += MERGE_TILE) {
      uint32_t tn = total - t0 < MERGE_TILE ? total - t0 : MERGE_TILE;
      // stage this tile's inbound records (arrival order) in LDS
      for (uint32_t i = lane; i < tn; i += 64) {
        uint32_t gi = t0 + i;
        uint32_t lo = 0, hi = cn - 1;  // last message with start <= gi
        while (lo < hi) {
          uint32_t mid = (lo + hi + 1) >> 1;
          if (s_start[mid] <= gi) lo = mid;
          else hi = mid - 1;
        }
        grec g = d.msg[(size_t)s_ent[lo] * cap + (gi - s_start[lo])];
        s_key[i] = g.r;
        s_val[i] = g.w;
        s_accf[i] = 0;
      }
      __syncthreads();
      // fold every key's occurrences in arrival order; one slot read + at most one write per key
      for (uint32_t i = lane; i < tn; i += 64) {
        uint32_t key = s_key[i];
        bool leader = true;
        for (uint32_t j = 0; j < i; j++)
          if (s_key[j] == key) {
            leader = false;
            break;
          }
        if (!leader) continue;
        uint64_t w0 = row[key], w = w0;
        c_rd++;
        for (uint32_t j = i; j < tn; j++) {
          if (s_key[j] != key) continue;
          bool a, st;
          w = merge_word(d, w, s_val[j], a, st);
          c_stale += st;
          if (a) {
            c_acc++;
            s_accf[j] = 1;
            s_acc[j] = w;
          }
        }
        if (w != w0) {
          row[key] = w;
          changed = true;
          c_wr++;
        }
      }
      c_merge += (lane == 0) ? tn : 0;
      __syncthreads();
      // ordered ballot compaction of accepted foreign records into the FIFO (retransmit)
      for (uint32_t b0 = 0; b0 < tn; b0 += 64) {
        uint32_t i = b0 + lane;
        bool f = i < tn && s_accf[i] && (s_key[i] / d.S != v);
        unsigned long long m = __ballot(f);
        uint32_t pos = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        if (f && n_retx + pos < room) {
          gx_job j;
          j.a = s_acc[i];
          j.b = 0;
          j.c = s_key[i];
          j.meta = meta_of(GX_JOB_RETX, 0, 1);
          j.wake = 0;
          j.aux = 0;
          d.fifo[(size_t)v * d.Q + ((tail0 + n_retx + pos) % d.Q)] = j;
        }
        n_retx += (uint32_t)__popcll(m);
      }
      __threadfence_block();
      __syncthreads();
    }
  }
  c_merge = wave_sum(c_merge);
  c_acc = wave_sum(c_acc);
  c_stale = wave_sum(c_stale);
  c_rd = wave_sum(c_rd);
  c_wr = wave_sum(c_wr);
  bool any = __ballot(changed) != 0;
  if (lane == 0) {
    uint32_t ok = n_retx < room ? n_retx : room;
    kbytes(d, GX_K_MERGE, 12ull * c_merge + 8ull * (c_rd + c_wr) + 32ull * ok + 8ull * deg, c_merge);
    h->fifo_tail = tail0 + ok;
    ctr_add(d, C_GOSSIP_MERGES, c_merge);
    ctr_add(d, C_GOSSIP_ACC, c_acc);
    ctr_add(d, C_STALE, c_stale);
    ctr_add(d, C_RETX, ok);
    ctr_add(d, C_QDROP, n_retx - ok);
    if (any) mark_change(d);
  }
}

// --------------------------------------------------------- phase 5: anti-entropy push-pull --
// Dense view-pair merge: dst <- src (and, when both, src <- dst's pre-exchange words).
GXD void ae_pair(const Dev &d, uint32_t a, uint32_t b, bool both, uint32_t *s_wave, unsigned long long *s_red) {
  uint64_t *A = &d.view[(size_t)a * d.R];
  uint64_t *B = &d.view[(size_t)b * d.R];
  gx_host_state *ha = &d.hs[a], *hb = &d.hs[b];
  uint32_t ta0 = ha->fifo_tail, ca0 = ta0 - ha->fifo_head;
  uint32_t tb0 = hb->fifo_tail, cb0 = tb0 - hb->fifo_head;
  uint32_t rooma = ca0 < d.Q - 2 ? d.Q - 2 - ca0 : 0, roomb = cb0 < d.Q - 2 ? d.Q - 2 - cb0 : 0;
  uint32_t na = 0, nb = 0;
  unsigned long long c_merge = 0, c_acc = 0, c_stale = 0, c_wr = 0;
  bool changed = false;
  for (uint32_t base = 0; base < d.R; base += blockDim.x) {
    uint32_t r = base + threadIdx.x;
    bool valid = r < d.R;
    uint64_t wa = valid ? A[r] : GX_SLOT_ABSENT;
    uint64_t wb = valid ? B[r] : GX_SLOT_ABSENT;
    bool fa = false, fb = false;
    uint64_t nwa = wa, nwb = wb;
    if (st_of(wb) != GX_ABSENT) {  // a.Merge(b): every present record of b
      bool ac, st;
      c_merge++;
      nwa = merge_word(d, wa, wb, ac, st);
      c_stale += st;
      if (ac) {
        c_acc++;
        fa = r / d.S != a;
      }
      if (nwa != wa) {
        A[r] = nwa;
        changed = true;
        c_wr++;
      }
    }
    if (both && st_of(wa) != GX_ABSENT) {  // b.Merge(a's snapshot)
      bool ac, st;
      c_merge++;
      nwb = merge_word(d, wb, wa, ac, st);
      c_stale += st;
      if (ac) {
        c_acc++;
        fb = r / d.S != b;
      }
      if (nwb != wb) {
        B[r] = nwb;
        changed = true;
        c_wr++;
      }
    }
    uint32_t tota, totb;
    uint32_t pa = block_scan_flag(fa, s_wave, tota);
    uint32_t pb = block_scan_flag(fb, s_wave, totb);
    if (fa && na + pa < rooma) {
      gx_job j;
      j.a = nwa;
      j.b = 0;
      j.c = r;
      j.meta = meta_of(GX_JOB_RETX, 0, 1);
      j.wake = 0;
      j.aux = 0;
      d.fifo[(size_t)a * d.Q + ((ta0 + na + pa) % d.Q)] = j;
    }
    if (fb && nb + pb < roomb) {
      gx_job j;
      j.a = nwb;
      j.b = 0;
      j.c = r;
      j.meta = meta_of(GX_JOB_RETX, 0, 1);
      j.wake = 0;
      j.aux = 0;
      d.fifo[(size_t)b * d.Q + ((tb0 + nb + pb) % d.Q)] = j;
    }
    na += tota;
    nb += totb;
  }
  if (changed) mark_change(d);
  c_wr = wave_sum(c_wr);
  if ((threadIdx.x & 63) == 0) kbytes(d, GX_K_AE, 8ull * c_wr, 0);
  block_ctr(d, C_AE_MERGES, c_merge, s_red);
  block_ctr(d, C_AE_ACC, c_acc, s_red);
  block_ctr(d, C_STALE, c_stale, s_red);
  if (threadIdx.x == 0) {
    uint32_t oka = na < rooma ? na : rooma, okb = nb < roomb ? nb : roomb;
    ha->fifo_tail = ta0 + oka;
    if (both) hb->fifo_tail = tb0 + okb;
    ctr_add(d, C_RETX, oka + (both ? okb : 0));
    ctr_add(d, C_QDROP, (na - oka) + (both ? nb - okb : 0));
    ctr_add(d, C_AESLOTS, (unsigned long long)d.R * (both ? 2 : 1));
    kbytes(d, GX_K_AE, 16ull * d.R + 32ull * (oka + (both ? okb : 0)), (unsigned long long)d.R * (both ? 2 : 1));
    if (both) ctr_add(d, C_AEX, 1);
  }
}

__global__ __launch_bounds__(256) void k_ae(Dev d, uint64_t key0, uint64_t key1) {
  __shared__ uint32_t s_wave[4];
  __shared__ unsigned long long s_red[4];
  uint32_t t = blockIdx.x, base = 0, m = d.H, q = t;
  uint64_t key = key0;
  if (d.partitioned) {
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
  uint32_t a = base + feistel_perm(key, 2 * q, m);
  uint32_t b = base + feistel_perm(key, 2 * q + 1, m);
  ae_pair(d, a, b, true, s_wave, s_red);
}

__global__ __launch_bounds__(256) void k_merge_views(Dev d, uint32_t dst, uint32_t src) {
  __shared__ uint32_t s_wave[4];
  __shared__ unsigned long long s_red[4];
  ae_pair(d, dst, src, false, s_wave, s_red);
}

// ------------------------------------------------------------------ convergence / digests --
__global__ void k_converged(Dev d, unsigned long long *bad) {
  uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  bool dis = false;
  if (r < d.R) {
    uint64_t w0 = d.view[r];
    for (uint32_t v = 1; v < d.H; v++)
      if (d.view[(size_t)v * d.R + r] != w0) {
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
  h = feed(h, j.b);
  h = feed(h, (uint64_t)j.c | ((uint64_t)j.meta << 32));
  return feed(h, (uint64_t)j.wake | ((uint64_t)j.aux << 32));
}
__global__ void k_digest(Dev d, uint64_t *out) {
  uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= d.H) return;
  const gx_host_state s = d.hs[v];
  uint64_t h = 0x243F6A8885A308D3ull;
  for (uint32_t i = s.fifo_head; i != s.fifo_tail; i++) h = feed_job(h, d.fifo[(size_t)v * d.Q + (i % d.Q)]);
  h = feed(h, 0xF1F0);
  for (uint32_t i = s.sleep_head; i != s.sleep_tail; i++) h = feed_job(h, d.sleep[(size_t)v * d.SQ + (i % d.SQ)]);
  h = feed(h, 0x51EE);
  h = feed(h, s.dq_len);
  for (uint32_t i = 0; i < s.dq_len; i++) {
    grec g = d.dq[(size_t)v * d.DQ + ((s.dq_head + i) & (d.DQ - 1))];
    h = feed(h, g.w);
    h = feed(h, g.r);
  }
  h = feed(h, 0xA7E4);
  for (uint32_t a = 0; a < d.A; a++) {
    if (!((s.arena_used >> a) & 1u)) continue;
    uint32_t len = d.arena_len[(size_t)v * d.A + a];
    h = feed(h, a);
    h = feed(h, len);
    for (uint32_t i = 0; i < len; i++) {
      grec g = d.arena[((size_t)v * d.A + a) * d.L + i];
      h = feed(h, g.w);
      h = feed(h, g.r);
    }
  }
  h = feed(h, s.flags);
  h = feed(h, (uint64_t)s.bs_next);
  h = feed(h, (uint64_t)s.bt_next);
  h = feed(h, (uint64_t)s.last_bcast_ns);
  h = feed(h, s.running);
  out[v] = h;
}

// ----------------------------------------------------------------- single-host ABI kernels --
__global__ void k_api_add(Dev d, const uint32_t *views, uint32_t fixed_view, const grec *recs, uint32_t n, int src,
                          uint32_t *acc) {
  uint32_t a = 0;
  for (uint32_t i = 0; i < n; i++) a += add_entry(d, views ? views[i] : fixed_view, recs[i], src);
  *acc = a;
}
__global__ void k_api_expire(Dev d, uint32_t v, uint32_t o, uint32_t *out) { *out = expire_server(d, v, o); }
__global__ void k_api_send(Dev d, uint32_t v, const grec *list, uint32_t n, uint32_t np) {
  int slot = alloc_list(d, v);
  if (slot < 0) return;
  uint32_t m = n < d.L ? n : d.L;
  grec *dst = list_ptr(d, v, slot);
  for (uint32_t i = 0; i < m; i++) dst[i] = list[i];
  commit_send(d, v, slot, m, np);
}
__global__ void k_api_bs(Dev d, uint32_t v, const grec *list, uint32_t n) {
  uint64_t inc;
  bs_body_list(d, v, list, n, inc);
}
__global__ void k_api_bt(Dev d, uint32_t v, uint64_t running, const grec *others, const uint32_t *n_others) {
  uint32_t n = *n_others;
  bt_finish(d, v, running, others, n < d.L ? n : d.L);
}
__global__ void k_api_tomb(Dev d, uint32_t v, uint64_t running, uint64_t *out_mask) {
  *out_mask = tombstone_services(d, v, running);
}
__global__ void k_api_getb(Dev d, uint32_t v, uint32_t limit, grec *out, uint32_t *n_out) {
  *n_out = get_broadcasts(d, v, limit, out);
}
__global__ void k_api_is_new(Dev d, uint32_t v, uint64_t w, uint32_t r, uint32_t *out) { *out = is_new(d, v, w, r); }
__global__ void k_api_set_slot(Dev d, uint32_t v, uint32_t r, uint64_t w) { set_slot(d, &d.view[(size_t)v * d.R + r], w); }
__global__ void k_api_mark(Dev d) { mark_change(d); }

// ================================================================================ host ==
struct TimedLaunch {
  int cls;
  hipEvent_t a, b;
};

struct gx_engine {
  Dev d;
  hipStream_t stream;
  int device;
  int timing;
  std::vector<TimedLaunch> pending_ev;
  double ms[GX_K_COUNT];
  uint64_t launches[GX_K_COUNT];
  grec *own_list;
  // small device scratch for single-host ABI calls
  void *api_dev;
  size_t api_dev_bytes;
  unsigned long long *conv_bad;
  uint64_t *digest_buf;
};

static int ensure_api(gx_engine *e, size_t bytes) {
  if (bytes <= e->api_dev_bytes) return GX_OK;
  if (e->api_dev) (void)hipFree(e->api_dev);
  e->api_dev = nullptr;
  e->api_dev_bytes = 0;
  size_t b = 1 << 20;
  while (b < bytes) b <<= 1;
  HIPCHK(hipMalloc(&e->api_dev, b));
  e->api_dev_bytes = b;
  return GX_OK;
}

static int64_t now_of(const gx_engine *e) { return e->d.p.t0_ns + e->d.round * e->d.p.round_ns; }
static void set_round_fields(gx_engine *e) {
  e->d.now = now_of(e);
  e->d.partitioned = e->d.round >= e->d.p.partition_start && e->d.round < e->d.p.partition_end;
}

struct LaunchTimer {
  gx_engine *e;
  int cls;
  hipEvent_t a, b;
  LaunchTimer(gx_engine *e_, int cls_) : e(e_), cls(cls_), a(nullptr), b(nullptr) {
    e->launches[cls]++;
    if (e->timing) {
      (void)hipEventCreate(&a);
      (void)hipEventCreate(&b);
      (void)hipEventRecord(a, e->stream);
    }
  }
  ~LaunchTimer() {
    if (e->timing) {
      (void)hipEventRecord(b, e->stream);
      e->pending_ev.push_back({cls, a, b});
    }
  }
};

static int drain_timing(gx_engine *e) {
  if (e->pending_ev.empty()) return GX_OK;
  HIPCHK(hipStreamSynchronize(e->stream));
  for (auto &t : e->pending_ev) {
    float ms = 0;
    (void)hipEventElapsedTime(&ms, t.a, t.b);
    e->ms[t.cls] += ms;
    (void)hipEventDestroy(t.a);
    (void)hipEventDestroy(t.b);
  }
  e->pending_ev.clear();
  return GX_OK;
}

static int sync_check(gx_engine *e) {
  HIPCHK(hipStreamSynchronize(e->stream));
  HIPCHK(hipGetLastError());
  return GX_OK;
}

static inline unsigned nblk(size_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

static int run_one_round(gx_engine *e) {
  Dev &d = e->d;
  set_round_fields(e);
  hipStream_t s = e->stream;
  {
    LaunchTimer t(e, GX_K_OWNER);
    k_owner<<<nblk(d.H, 256), 256, 0, s>>>(d, e->own_list);
  }
  {
    LaunchTimer t(e, GX_K_SCAN);
    k_scan<<<d.H, 256, 0, s>>>(d, d.scan_list, d.L, d.L, d.scan_cnt, -1);
    k_bt_finish<<<nblk(d.H, 256), 256, 0, s>>>(d);
  }
  if (d.p.storm_round >= 0 && d.round == d.p.storm_round && d.H >= 2) {
    LaunchTimer t(e, GX_K_STORM);
    k_storm<<<d.H, 256, 0, s>>>(d);
  }
  {
    LaunchTimer t(e, GX_K_SEND);
    k_send<<<nblk(d.H, 256), 256, 0, s>>>(d);
  }
  {
    LaunchTimer t(e, GX_K_ROUTE);
    HIPCHK(hipMemsetAsync(d.in_cnt, 0, sizeof(uint32_t) * (d.H + 1), s));
    HIPCHK(hipMemsetAsync(d.in_cur, 0, sizeof(uint32_t) * d.H, s));
    size_t ne = (size_t)d.H * d.K;
    if (ne) {
      k_route_count<<<nblk(ne, 256), 256, 0, s>>>(d);
      k_route_offsets<<<1, 1024, 0, s>>>(d);
      k_route_fill<<<nblk(ne, 256), 256, 0, s>>>(d);
      k_route_rank<<<nblk(ne, 256), 256, 0, s>>>(d);
    }
  }
  if (d.K) {
    LaunchTimer t(e, GX_K_MERGE);
    k_merge<<<d.H, 64, 0, s>>>(d);
  }
  if (d.p.ae_period_rounds && (uint64_t)d.round % d.p.ae_period_rounds == d.p.ae_phase) {
    uint32_t np;
    uint64_t key0, key1 = 0;
    if (d.partitioned) {
      uint32_t m0 = d.H / 2, m1 = d.H - m0;
      np = m0 / 2 + m1 / 2;
      key0 = rng4(d.p.seed, ST_AE, (uint64_t)d.round, 0, 0);
      key1 = rng4(d.p.seed, ST_AE, (uint64_t)d.round, m0, 0);
    } else {
      np = d.H / 2;
      key0 = rng4(d.p.seed, ST_AE, (uint64_t)d.round, 0, 0);
    }
    if (np) {
      LaunchTimer t(e, GX_K_AE);
      k_ae<<<np, 256, 0, s>>>(d, key0, key1);
    }
  }
  HIPCHK(hipGetLastError());
  d.round++;
  return GX_OK;
}

static int wake_all(gx_engine *e) {
  set_round_fields(e);
  k_wake<<<nblk(e->d.H, 256), 256, 0, e->stream>>>(e->d);
  HIPCHK(hipGetLastError());
  return GX_OK;
}

// ------------------------------------------------------------------------------ ABI ------
extern "C" {

int gx_abi_version(void) { return GX_ABI_VERSION; }
const char *gx_backend(void) { return "hip-gfx950"; }

void gx_params_default(gx_params *p) {
  memset(p, 0, sizeof(*p));
  p->n_hosts = 64;
  p->n_services = 8;
  p->fanout = 3;
  p->packet_cap = 32;
  p->pending_cap = 100;
  p->queue_cap = 1024;
  p->list_slots = 16;
  p->gossip_stop_on_empty = 1;
  p->alive_interval_rounds = 5;
  p->tombstone_interval_rounds = 10;
  p->retransmit_rounds = 5;
  p->alive_count = 5;
  p->tombstone_count = 10;
  p->init_mode = GX_INIT_EMPTY;
  p->t0_ns = 1700000000000000000ll;
  p->round_ns = 200000000ll;
  p->alive_lifespan_ns = 80000000000ll;
  p->draining_lifespan_ns = 600000000000ll;
  p->tombstone_lifespan_ns = 10800000000000ll;
  p->stale_fudge_ns = 60000000000ll;
  p->alive_broadcast_interval_ns = 60000000000ll;
  p->pass_increment_ns = 50;
  p->tombstone_bump_ns = 1000000000ll;
  p->seed = 0x5EEDull;
  p->aged_max_ns = 100000000000ll;
  p->storm_round = -1;
}

static int check_params(const gx_params *p) {
  if (!p || p->n_hosts < 1 || p->n_services < 1 || p->n_services > 64) return GX_EINVAL;
  if (p->fanout > 16 || p->packet_cap < 1 || p->packet_cap > 256 || p->pending_cap > 256) return GX_EINVAL;
  if (p->queue_cap < 3 || p->list_slots < 1 || p->list_slots > 32) return GX_EINVAL;
  if (p->alive_interval_rounds < 1 || p->tombstone_interval_rounds < 1) return GX_EINVAL;
  if (p->retransmit_rounds > 1000) return GX_EINVAL;
  if (p->alive_count < 1 || p->alive_count > 255 || p->tombstone_count < 1 || p->tombstone_count > 255) return GX_EINVAL;
  if (p->init_mode > GX_INIT_WARM) return GX_EINVAL;
  if (p->t0_ns < 0 || p->t0_ns >= GX_TS_LIMIT - ((int64_t)1 << 56) || p->round_ns <= 0) return GX_EINVAL;
  if ((uint64_t)p->n_hosts * p->n_services > 0xffffffffull) return GX_EINVAL;
  if (p->ae_period_rounds && p->ae_phase >= p->ae_period_rounds) return GX_EINVAL;
  return GX_OK;
}

int gx_destroy(gx_engine *e) {
  if (!e) return GX_EINVAL;
  (void)hipSetDevice(e->device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  for (auto &t : e->pending_ev) {
    (void)hipEventDestroy(t.a);
    (void)hipEventDestroy(t.b);
  }
  Dev &d = e->d;
  void *ptrs[] = {d.view, d.own_status, d.hs, d.fifo, d.sleep, d.dq, d.arena, d.arena_len, d.msg, d.msg_len,
                  d.msg_dst, d.in_cnt, d.in_cur, d.in_fill, d.in_sorted, d.scan_list, d.scan_cnt, d.tick,
                  d.ctr, e->own_list, e->api_dev, e->conv_bad, e->digest_buf};
  for (void *p : ptrs)
    if (p) (void)hipFree(p);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
  return GX_OK;
}

#define ALLOC(ptr, bytes)                                   \
  do {                                                      \
    if (hipMalloc((void **)&(ptr), (bytes)) != hipSuccess) { \
      (void)hipGetLastError();                              \
      gx_destroy(e);                                        \
      return GX_ENOMEM;                                     \
    }                                                       \
  } while (0)

int gx_create(const gx_params *p, gx_engine **out) {
  if (!out) return GX_EINVAL;
  int rc = check_params(p);
  if (rc) return rc;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || p->device < 0 || p->device >= ndev) return GX_EIO;
  HIPCHK(hipSetDevice(p->device));
  gx_engine *e = new gx_engine();
  memset(&e->d, 0, sizeof(e->d));
  e->device = p->device;
  e->timing = 0;
  memset(e->ms, 0, sizeof(e->ms));
  memset(e->launches, 0, sizeof(e->launches));
  e->own_list = nullptr;
  e->api_dev = nullptr;
  e->api_dev_bytes = 0;
  e->conv_bad = nullptr;
  e->digest_buf = nullptr;
  e->stream = nullptr;
  Dev &d = e->d;
  d.p = *p;
  d.H = p->n_hosts;
  d.S = p->n_services;
  d.R = p->n_hosts * p->n_services;
  d.Q = p->queue_cap;
  d.A = p->list_slots;
  d.L = p->packet_cap + p->pending_cap;
  d.K = p->fanout;
  d.SQ = pow2_at_least(64 > d.K * (p->retransmit_rounds + 1) ? 64 : d.K * (p->retransmit_rounds + 1));
  d.DQ = pow2_at_least(d.L + p->pending_cap + 64);
  d.round = 0;
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
    delete e;
    return GX_EIO;
  }
  size_t H = d.H, K = d.K ? d.K : 1;
  ALLOC(d.view, sizeof(uint64_t) * H * d.R);
  ALLOC(d.own_status, H * d.S);
  ALLOC(d.hs, sizeof(gx_host_state) * H);
  ALLOC(d.fifo, sizeof(gx_job) * H * d.Q);
  ALLOC(d.sleep, sizeof(gx_job) * H * d.SQ);
  ALLOC(d.dq, sizeof(grec) * H * d.DQ);
  ALLOC(d.arena, sizeof(grec) * H * d.A * d.L);
  ALLOC(d.arena_len, sizeof(uint32_t) * H * d.A);
  ALLOC(d.msg, sizeof(grec) * H * K * p->packet_cap);
  ALLOC(d.msg_len, sizeof(uint32_t) * H * K);
  ALLOC(d.msg_dst, sizeof(uint32_t) * H * K);
  ALLOC(d.in_cnt, sizeof(uint32_t) * (H + 1));
  ALLOC(d.in_cur, sizeof(uint32_t) * H);
  ALLOC(d.in_fill, sizeof(uint32_t) * H * K);
  ALLOC(d.in_sorted, sizeof(uint32_t) * H * K);
  ALLOC(d.scan_list, sizeof(grec) * H * d.L);
  ALLOC(d.scan_cnt, sizeof(uint32_t) * H);
  ALLOC(d.tick, H);
  ALLOC(d.ctr, sizeof(DevCtr));
  ALLOC(e->own_list, sizeof(grec) * H * d.S);
  ALLOC(e->conv_bad, sizeof(unsigned long long));
  ALLOC(e->digest_buf, sizeof(uint64_t) * H);
  hipStream_t s = e->stream;
  uint64_t *rec_word = nullptr;
  ALLOC(rec_word, sizeof(uint64_t) * d.R);
  HIPCHK(hipMemsetAsync(d.ctr, 0, sizeof(DevCtr), s));
  HIPCHK(hipMemsetAsync(d.arena_len, 0, sizeof(uint32_t) * H * d.A, s));
  HIPCHK(hipMemsetAsync(d.msg_len, 0, sizeof(uint32_t) * H * K, s));
  HIPCHK(hipMemsetAsync(d.tick, 0, H, s));
  set_round_fields(e);
  k_init_rec<<<nblk(d.R, 256), 256, 0, s>>>(d, rec_word);
  k_init_views<<<2048, 256, 0, s>>>(d, rec_word);
  k_init_hosts<<<nblk(d.H, 256), 256, 0, s>>>(d);
  rc = sync_check(e);
  (void)hipFree(rec_word);
  if (rc) {
    gx_destroy(e);
    return rc;
  }
  *out = e;
  return GX_OK;
}

int gx_set_round(gx_engine *e, int64_t round) {
  if (!e || round < e->d.round) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  e->d.round = round;
  int rc = wake_all(e);
  return rc ? rc : sync_check(e);
}

int gx_get_round(gx_engine *e, int64_t *round) {
  if (!e || !round) return GX_EINVAL;
  *round = e->d.round;
  return GX_OK;
}

int gx_enable_timing(gx_engine *e, int on) {
  if (!e) return GX_EINVAL;
  e->timing = on ? 1 : 0;
  return GX_OK;
}

int gx_run_rounds(gx_engine *e, uint32_t n_rounds) {
  if (!e) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  for (uint32_t i = 0; i < n_rounds; i++) {
    int rc = run_one_round(e);
    if (rc) return rc;
    if (e->pending_ev.size() > 4096) {
      rc = drain_timing(e);
      if (rc) return rc;
    }
  }
  int rc = wake_all(e);
  if (rc) return rc;
  return sync_check(e);
}

// ---------------------------------------------------------------------- record helpers --
static int to_grec(const gx_engine *e, const gx_service *s, grec *g) {
  if (s->host >= e->d.H || s->svc >= e->d.S || s->status > 6 || s->updated_ns < 0 || s->updated_ns >= GX_TS_LIMIT)
    return GX_EINVAL;
  g->w = pack(s->updated_ns, s->status);
  g->r = s->host * e->d.S + s->svc;
  g->pad = 0;
  return GX_OK;
}
static void to_svc(const gx_engine *e, const grec *g, gx_service *s) {
  s->updated_ns = ts_of(g->w);
  s->host = g->r / e->d.S;
  s->svc = (uint16_t)(g->r % e->d.S);
  s->status = (uint8_t)st_of(g->w);
  s->flags = 0;
}

// Converts caller records into a device grec array inside the api scratch (after `offset`).
static int stage_recs(gx_engine *e, const gx_service *svcs, uint32_t n, size_t offset, grec **dev_out) {
  std::vector<grec> tmp(n ? n : 1);
  for (uint32_t i = 0; i < n; i++)
    if (to_grec(e, &svcs[i], &tmp[i])) return GX_EINVAL;
  int rc = ensure_api(e, offset + sizeof(grec) * (n + 1));
  if (rc) return rc;
  grec *dev = (grec *)((char *)e->api_dev + offset);
  if (n) HIPCHK(hipMemcpyAsync(dev, tmp.data(), sizeof(grec) * n, hipMemcpyHostToDevice, e->stream));
  *dev_out = dev;
  return GX_OK;
}

static int api_add(gx_engine *e, const uint32_t *views, uint32_t fixed_view, const gx_service *svcs, uint32_t n,
                   int src, uint32_t *n_acc) {
  HIPCHK(hipSetDevice(e->device));
  if (views)
    for (uint32_t i = 0; i < n; i++)
      if (views[i] >= e->d.H) return GX_EINVAL;
  size_t vbytes = ((sizeof(uint32_t) * (n + 1)) + 255) & ~(size_t)255;
  grec *drec;
  int rc = stage_recs(e, svcs, n, vbytes + 256, &drec);
  if (rc) return rc;
  uint32_t *dviews = (uint32_t *)e->api_dev;
  uint32_t *dacc = (uint32_t *)((char *)e->api_dev + vbytes);
  if (views && n) HIPCHK(hipMemcpyAsync(dviews, views, sizeof(uint32_t) * n, hipMemcpyHostToDevice, e->stream));
  set_round_fields(e);
  k_api_add<<<1, 1, 0, e->stream>>>(e->d, views ? dviews : nullptr, fixed_view, drec, n, src, dacc);
  uint32_t acc = 0;
  HIPCHK(hipMemcpyAsync(&acc, dacc, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  rc = sync_check(e);
  if (rc) return rc;
  if (n_acc) *n_acc = acc;
  return GX_OK;
}

int gx_add_service_entries(gx_engine *e, const uint32_t *views, const gx_service *svcs, uint32_t n,
                           uint32_t *n_accepted) {
  if (!e || (n && (!views || !svcs))) return GX_EINVAL;
  return api_add(e, views, 0, svcs, n, SRC_LOCAL, n_accepted);
}

int gx_notify_msg(gx_engine *e, uint32_t host, const gx_service *recs, uint32_t n) {
  if (!e || host >= e->d.H || (n && !recs)) return GX_EINVAL;
  return api_add(e, nullptr, host, recs, n, SRC_GOSSIP, nullptr);
}

int gx_merge_remote_state(gx_engine *e, uint32_t view, const gx_service *svcs, uint32_t n) {
  if (!e || view >= e->d.H || (n && !svcs)) return GX_EINVAL;
  return api_add(e, nullptr, view, svcs, n, SRC_AE, nullptr);
}

int gx_merge(gx_engine *e, uint32_t dst, uint32_t src) {
  if (!e || dst >= e->d.H || src >= e->d.H) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  set_round_fields(e);
  k_merge_views<<<1, 256, 0, e->stream>>>(e->d, dst, src);
  return sync_check(e);
}

int gx_tombstone_others(gx_engine *e, uint32_t view, gx_service *out, uint32_t cap, uint32_t *n_out) {
  if (!e || view >= e->d.H || (cap && !out)) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  int rc = ensure_api(e, 256 + sizeof(grec) * (cap + 1));
  if (rc) return rc;
  uint32_t *dcnt = (uint32_t *)e->api_dev;
  grec *dlist = (grec *)((char *)e->api_dev + 256);
  set_round_fields(e);
  k_scan<<<1, 256, 0, e->stream>>>(e->d, dlist, 0, cap, dcnt, (int)view);
  uint32_t n = 0;
  HIPCHK(hipMemcpyAsync(&n, dcnt, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  rc = sync_check(e);
  if (rc) return rc;
  uint32_t m = n < cap ? n : cap;
  if (m) {
    std::vector<grec> tmp(m);
    HIPCHK(hipMemcpy(tmp.data(), dlist, sizeof(grec) * m, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < m; i++) to_svc(e, &tmp[i], &out[i]);
  }
  if (n_out) *n_out = n;
  return GX_OK;
}

int gx_tombstone_services(gx_engine *e, uint32_t host, const uint16_t *running, uint32_t n_running, gx_service *out,
                          uint32_t cap, uint32_t *n_out) {
  if (!e || host >= e->d.H || (n_running && !running) || (cap && !out)) return GX_EINVAL;
  uint64_t mask = 0;
  for (uint32_t i = 0; i < n_running; i++) {
    if (running[i] >= e->d.S) return GX_EINVAL;
    mask |= 1ull << running[i];
  }
  HIPCHK(hipSetDevice(e->device));
  int rc = ensure_api(e, 64);
  if (rc) return rc;
  set_round_fields(e);
  k_api_tomb<<<1, 1, 0, e->stream>>>(e->d, host, mask, (uint64_t *)e->api_dev);
  uint64_t m = 0;
  HIPCHK(hipMemcpyAsync(&m, e->api_dev, sizeof(uint64_t), hipMemcpyDeviceToHost, e->stream));
  rc = sync_check(e);
  if (rc) return rc;
  uint32_t n = 0;
  int64_t now = now_of(e);
  for (uint32_t s = 0; s < e->d.S; s++)
    if ((m >> s) & 1ull)
      for (int k = 0; k < 2; k++) {
        if (n < cap) {
          grec g;
          g.w = pack(now, GX_TOMBSTONE);
          g.r = host * e->d.S + s;
          to_svc(e, &g, &out[n]);
        }
        n++;
      }
  if (n_out) *n_out = n;
  return GX_OK;
}

int gx_expire_server(gx_engine *e, uint32_t view, uint32_t owner, int *expired) {
  if (!e || view >= e->d.H || owner >= e->d.H) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  int rc = ensure_api(e, 64);
  if (rc) return rc;
  set_round_fields(e);
  k_api_expire<<<1, 1, 0, e->stream>>>(e->d, view, owner, (uint32_t *)e->api_dev);
  uint32_t x = 0;
  HIPCHK(hipMemcpyAsync(&x, e->api_dev, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  rc = sync_check(e);
  if (rc) return rc;
  if (expired) *expired = (int)x;
  return GX_OK;
}

int gx_notify_leave(gx_engine *e, uint32_t view, uint32_t node) { return gx_expire_server(e, view, node, nullptr); }

int gx_send_services(gx_engine *e, uint32_t host, const gx_service *svcs, uint32_t n, uint32_t n_passes) {
  if (!e || host >= e->d.H || (n && !svcs) || n_passes < 1 || n_passes > 255) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  grec *drec;
  int rc = stage_recs(e, svcs, n, 0, &drec);
  if (rc) return rc;
  set_round_fields(e);
  k_api_send<<<1, 1, 0, e->stream>>>(e->d, host, drec, n, n_passes);
  return sync_check(e);
}

int gx_broadcast_services(gx_engine *e, uint32_t host, const gx_service *list, uint32_t n) {
  if (!e || host >= e->d.H || (n && !list) || n > 64) return GX_EINVAL;
  for (uint32_t i = 0; i < n; i++)
    if (list[i].host != host) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  grec *drec;
  int rc = stage_recs(e, list, n, 0, &drec);
  if (rc) return rc;
  set_round_fields(e);
  k_api_bs<<<1, 1, 0, e->stream>>>(e->d, host, drec, n);
  return sync_check(e);
}

int gx_broadcast_tombstones(gx_engine *e, uint32_t host, const gx_service *list, uint32_t n) {
  if (!e || host >= e->d.H || (n && !list)) return GX_EINVAL;
  uint64_t mask = 0;
  for (uint32_t i = 0; i < n; i++) {
    if (list[i].host != host || list[i].svc >= e->d.S) return GX_EINVAL;
    mask |= 1ull << list[i].svc;
  }
  HIPCHK(hipSetDevice(e->device));
  int rc = ensure_api(e, 256 + sizeof(grec) * (e->d.L + 1));
  if (rc) return rc;
  uint32_t *dcnt = (uint32_t *)e->api_dev;
  grec *dlist = (grec *)((char *)e->api_dev + 256);
  set_round_fields(e);
  k_scan<<<1, 256, 0, e->stream>>>(e->d, dlist, 0, e->d.L, dcnt, (int)host);
  k_api_bt<<<1, 1, 0, e->stream>>>(e->d, host, mask, dlist, dcnt);
  return sync_check(e);
}

int gx_is_new_service(gx_engine *e, uint32_t view, const gx_service *svc, int *out) {
  grec g;
  if (!e || !svc || !out || view >= e->d.H || to_grec(e, svc, &g)) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  int rc = ensure_api(e, 64);
  if (rc) return rc;
  k_api_is_new<<<1, 1, 0, e->stream>>>(e->d, view, g.w, g.r, (uint32_t *)e->api_dev);
  uint32_t x = 0;
  HIPCHK(hipMemcpyAsync(&x, e->api_dev, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  rc = sync_check(e);
  if (rc) return rc;
  *out = (int)x;
  return GX_OK;
}

int gx_get_broadcasts(gx_engine *e, uint32_t host, uint32_t limit, gx_service *out, uint32_t cap, uint32_t *n_out) {
  if (limit == GX_LIMIT_DEFAULT) limit = e ? e->d.p.packet_cap : 0;
  if (!e || host >= e->d.H || !n_out || limit > 256 || cap < limit || (limit && !out)) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  int rc = ensure_api(e, 256 + sizeof(grec) * 257);
  if (rc) return rc;
  uint32_t *dn = (uint32_t *)e->api_dev;
  grec *dpk = (grec *)((char *)e->api_dev + 256);
  set_round_fields(e);
  k_api_getb<<<1, 1, 0, e->stream>>>(e->d, host, limit, dpk, dn);
  uint32_t n = 0;
  HIPCHK(hipMemcpyAsync(&n, dn, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  rc = sync_check(e);
  if (rc) return rc;
  if (n) {
    std::vector<grec> tmp(n);
    HIPCHK(hipMemcpy(tmp.data(), dpk, sizeof(grec) * n, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; i++) to_svc(e, &tmp[i], &out[i]);
  }
  *n_out = n;
  return GX_OK;
}

int gx_local_state(gx_engine *e, uint32_t view, gx_service *out, uint32_t cap, uint32_t *n_out) {
  if (!e || view >= e->d.H || (cap && !out)) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  std::vector<uint64_t> row(e->d.R);
  HIPCHK(hipMemcpy(row.data(), &e->d.view[(size_t)view * e->d.R], sizeof(uint64_t) * e->d.R, hipMemcpyDeviceToHost));
  uint32_t n = 0;
  for (uint32_t r = 0; r < e->d.R; r++) {
    if (st_of(row[r]) == GX_ABSENT) continue;
    if (n < cap) {
      grec g;
      g.w = row[r];
      g.r = r;
      to_svc(e, &g, &out[n]);
    }
    n++;
  }
  if (n_out) *n_out = n;
  return GX_OK;
}

int gx_read_views(gx_engine *e, uint32_t lo, uint32_t hi, uint64_t *out) {
  if (!e || lo > hi || hi > e->d.H || (hi > lo && !out)) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipStreamSynchronize(e->stream));
  if (hi > lo)
    HIPCHK(hipMemcpy(out, &e->d.view[(size_t)lo * e->d.R], sizeof(uint64_t) * (size_t)(hi - lo) * e->d.R,
                     hipMemcpyDeviceToHost));
  return GX_OK;
}

int gx_write_views(gx_engine *e, uint32_t lo, uint32_t hi, const uint64_t *in) {
  if (!e || lo > hi || hi > e->d.H || (hi > lo && !in)) return GX_EINVAL;
  size_t n = (size_t)(hi - lo) * e->d.R;
  for (size_t i = 0; i < n; i++)
    if (st_of(in[i]) == 7 && in[i] != GX_SLOT_ABSENT) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipStreamSynchronize(e->stream));
  if (n) HIPCHK(hipMemcpy(&e->d.view[(size_t)lo * e->d.R], in, sizeof(uint64_t) * n, hipMemcpyHostToDevice));
  set_round_fields(e);
  k_api_mark<<<1, 1, 0, e->stream>>>(e->d);
  return sync_check(e);
}

int gx_write_slot(gx_engine *e, uint32_t view, const gx_service *svc) {
  if (!e || !svc || view >= e->d.H) return GX_EINVAL;
  uint64_t w;
  uint32_t r;
  if (svc->status == GX_ABSENT) {
    if (svc->host >= e->d.H || svc->svc >= e->d.S) return GX_EINVAL;
    w = GX_SLOT_ABSENT;
    r = svc->host * e->d.S + svc->svc;
  } else {
    grec g;
    if (to_grec(e, svc, &g)) return GX_EINVAL;
    w = g.w;
    r = g.r;
  }
  HIPCHK(hipSetDevice(e->device));
  set_round_fields(e);
  k_api_set_slot<<<1, 1, 0, e->stream>>>(e->d, view, r, w);
  return sync_check(e);
}

int gx_read_hosts(gx_engine *e, uint32_t lo, uint32_t hi, gx_host_state *out) {
  if (!e || lo > hi || hi > e->d.H || (hi > lo && !out)) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipStreamSynchronize(e->stream));
  if (hi > lo) HIPCHK(hipMemcpy(out, &e->d.hs[lo], sizeof(gx_host_state) * (hi - lo), hipMemcpyDeviceToHost));
  return GX_OK;
}

static int read_ring(gx_engine *e, const gx_job *base, uint32_t ring, uint32_t head, uint32_t n, gx_job *out,
                     uint32_t cap) {
  uint32_t m = n < cap ? n : cap;
  for (uint32_t i = 0; i < m;) {
    uint32_t idx = (head + i) % ring;
    uint32_t run = ring - idx;
    if (run > m - i) run = m - i;
    HIPCHK(hipMemcpy(&out[i], &base[idx], sizeof(gx_job) * run, hipMemcpyDeviceToHost));
    i += run;
  }
  return GX_OK;
}

int gx_read_queue(gx_engine *e, uint32_t host, gx_job *out, uint32_t cap, uint32_t *n_out) {
  if (!e || host >= e->d.H || (cap && !out)) return GX_EINVAL;
  gx_host_state h;
  int rc = gx_read_hosts(e, host, host + 1, &h);
  if (rc) return rc;
  uint32_t n = h.fifo_tail - h.fifo_head;
  rc = read_ring(e, &e->d.fifo[(size_t)host * e->d.Q], e->d.Q, h.fifo_head % e->d.Q, n, out, cap);
  if (rc) return rc;
  if (n_out) *n_out = n;
  return GX_OK;
}

int gx_read_sleepers(gx_engine *e, uint32_t host, gx_job *out, uint32_t cap, uint32_t *n_out) {
  if (!e || host >= e->d.H || (cap && !out)) return GX_EINVAL;
  gx_host_state h;
  int rc = gx_read_hosts(e, host, host + 1, &h);
  if (rc) return rc;
  uint32_t n = h.sleep_tail - h.sleep_head;
  rc = read_ring(e, &e->d.sleep[(size_t)host * e->d.SQ], e->d.SQ, h.sleep_head % e->d.SQ, n, out, cap);
  if (rc) return rc;
  if (n_out) *n_out = n;
  return GX_OK;
}

int gx_read_pending(gx_engine *e, uint32_t host, gx_service *out, uint32_t cap, uint32_t *n_out) {
  if (!e || host >= e->d.H || (cap && !out)) return GX_EINVAL;
  gx_host_state h;
  int rc = gx_read_hosts(e, host, host + 1, &h);
  if (rc) return rc;
  std::vector<grec> dq(e->d.DQ);
  HIPCHK(hipMemcpy(dq.data(), &e->d.dq[(size_t)host * e->d.DQ], sizeof(grec) * e->d.DQ, hipMemcpyDeviceToHost));
  for (uint32_t i = 0; i < h.dq_len && i < cap; i++) to_svc(e, &dq[(h.dq_head + i) & (e->d.DQ - 1)], &out[i]);
  if (n_out) *n_out = h.dq_len;
  return GX_OK;
}

int gx_read_list(gx_engine *e, uint32_t host, uint32_t slot, gx_service *out, uint32_t cap, uint32_t *n_out) {
  if (!e || host >= e->d.H || slot >= e->d.A || (cap && !out)) return GX_EINVAL;
  gx_host_state h;
  int rc = gx_read_hosts(e, host, host + 1, &h);
  if (rc) return rc;
  uint32_t n = 0;
  if ((h.arena_used >> slot) & 1u)
    HIPCHK(hipMemcpy(&n, &e->d.arena_len[(size_t)host * e->d.A + slot], sizeof(uint32_t), hipMemcpyDeviceToHost));
  uint32_t m = n < cap ? n : cap;
  if (m) {
    std::vector<grec> tmp(m);
    HIPCHK(hipMemcpy(tmp.data(), &e->d.arena[((size_t)host * e->d.A + slot) * e->d.L], sizeof(grec) * m,
                     hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < m; i++) to_svc(e, &tmp[i], &out[i]);
  }
  if (n_out) *n_out = n;
  return GX_OK;
}

int gx_host_digests(gx_engine *e, uint64_t *out) {
  if (!e || !out) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  k_digest<<<nblk(e->d.H, 256), 256, 0, e->stream>>>(e->d, e->digest_buf);
  HIPCHK(hipMemcpyAsync(out, e->digest_buf, sizeof(uint64_t) * e->d.H, hipMemcpyDeviceToHost, e->stream));
  return sync_check(e);
}

int gx_stats_get(gx_engine *e, gx_stats *out) {
  if (!e || !out) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  DevCtr c;
  HIPCHK(hipMemcpyAsync(&c, e->d.ctr, sizeof(c), hipMemcpyDeviceToHost, e->stream));
  int rc = sync_check(e);
  if (rc) return rc;
  memset(out, 0, sizeof(*out));
  out->round = e->d.round;
  out->gossip_merges = c.c[C_GOSSIP_MERGES];
  out->ae_merges = c.c[C_AE_MERGES];
  out->local_merges = c.c[C_LOCAL_MERGES];
  out->gossip_accepts = c.c[C_GOSSIP_ACC];
  out->ae_accepts = c.c[C_AE_ACC];
  out->local_accepts = c.c[C_LOCAL_ACC];
  out->stale_drops = c.c[C_STALE];
  out->retransmits = c.c[C_RETX];
  out->queue_drops = c.c[C_QDROP];
  out->list_drops = c.c[C_LDROP];
  out->sleep_drops = c.c[C_SDROP];
  out->pending_drops = c.c[C_PDROP];
  out->dequeues = c.c[C_DEQ];
  out->nil_batches = c.c[C_NIL];
  out->packets = c.c[C_PACKETS];
  out->records_sent = c.c[C_RECSENT];
  out->expired = c.c[C_EXPIRED];
  out->gc = c.c[C_GC];
  out->own_tombstones = c.c[C_OWNTOMB];
  out->expire_server = c.c[C_EXPSRV];
  out->send_jobs = c.c[C_SENDJOBS];
  out->ae_exchanges = c.c[C_AEX];
  out->churn_events = c.c[C_CHURN];
  out->scan_slots = c.c[C_SCANSLOTS];
  out->ae_slots = c.c[C_AESLOTS];
  out->last_change_round = (int64_t)c.last_change_p1 - 1;
  return GX_OK;
}

int gx_timing_get(gx_engine *e, gx_timing *out) {
  if (!e || !out) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  int rc = drain_timing(e);
  if (rc) return rc;
  DevCtr c;
  HIPCHK(hipMemcpyAsync(&c, e->d.ctr, sizeof(c), hipMemcpyDeviceToHost, e->stream));
  rc = sync_check(e);
  if (rc) return rc;
  memset(out, 0, sizeof(*out));
  for (int i = 0; i < GX_K_COUNT; i++) {
    out->ms[i] = e->ms[i];
    out->launches[i] = e->launches[i];
    out->bytes[i] = c.bytes[i];
    out->units[i] = c.units[i];
  }
  return GX_OK;
}

int gx_converged(gx_engine *e, int *converged, uint64_t *n_disagree) {
  if (!e) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipMemsetAsync(e->conv_bad, 0, sizeof(unsigned long long), e->stream));
  {
    LaunchTimer t(e, GX_K_CONVERGE);
    k_converged<<<nblk(e->d.R, 256), 256, 0, e->stream>>>(e->d, e->conv_bad);
  }
  unsigned long long bad = 0;
  HIPCHK(hipMemcpyAsync(&bad, e->conv_bad, sizeof(bad), hipMemcpyDeviceToHost, e->stream));
  int rc = sync_check(e);
  if (rc) return rc;
  if (converged) *converged = bad == 0;
  if (n_disagree) *n_disagree = bad;
  return GX_OK;
}

}  // extern "C"

// gx_device.hpp — device-side data layout and scalar semantics of the sidecar-gx engine.
//
// Layout in HBM (one engine = one GPU's cluster):
//   view      u64 [H][R]      R = H*S packed slots (ts << 3 | status), one row per host view
//   minexp    u64 [H]         lower bound of min over present slots of (ts + lifespan(status))
//   hs        gx_host_state[H] per-host broadcast-queue / looper bookkeeping (80 B)
//   fifo      gx_job [H][Q]   broadcast FIFO ring: the stored window of the blocked senders of
//                             state.Broadcasts (16 B jobs; later jobs are counted, gx.h gx_job)
//   sleep     gx_sleeper [H][SQ] SendServices passes sleeping TOMBSTONE_RETRANSMIT
//   dq        grec [H][DQ]    delegate pendingBroadcasts as a deque (push-front batch, pop packet)
//   arena     grec [H][A][L]  SendServices lists (L = packet_cap + pending_cap)
//   msg       grec [H][K][cap] this round's packets, msg_len/msg_dst [H][K]
//   in_hdr    uint4 [H][DI]   receiver inboxes: packet headers registered by the senders
//
// The scalar helpers below are the one-thread-per-host form of the reference semantics, used by
// the per-host round kernels (owner ticks, GetBroadcasts) and by the single-host ABI entry points.
// They count events into a per-thread accumulator (Acc) that each wave flushes once, so no kernel
// funnels thousands of atomics into one counter word. The hot data-parallel phases (gossip merge,
// anti-entropy, expiry scan, departure storm) have their own wave/block kernels in gx_engine.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gx.h"

#define GXD __device__ __forceinline__
#define GXHD __host__ __device__ __forceinline__

// Global (address space 1) loads and stores through pointers the compiler only knows as generic
// (taken from LDS or selected at run time): a flat access counts in lgkmcnt as well as vmcnt, so the
// next wait for an LDS read would also wait for it; global ones leave the loads in flight.
#define GX_GLOBAL __attribute__((address_space(1)))
typedef unsigned int gx_u32x4 __attribute__((ext_vector_type(4)));
template <class T>
GXD T gld(const T *p) {  // scalars
  return *(const GX_GLOBAL T *)p;
}
typedef unsigned int gx_u32x3 __attribute__((ext_vector_type(3)));
template <class T>
GXD void gst(T *p, T v) {  // scalars
  *(GX_GLOBAL T *)p = v;
}
GXD gx_u32x4 gld4(const void *p) { return *(const GX_GLOBAL gx_u32x4 *)p; }
// a record's word and key only (dwordx3): no dead destination register for the allocator to reuse
// while the load is in flight (that reuse makes it wait for the load on the spot)
GXD gx_u32x3 gld3(const void *p) { return *(const GX_GLOBAL gx_u32x3 *)p; }
GXD void gst4(void *p, gx_u32x4 v) { *(GX_GLOBAL gx_u32x4 *)p = v; }

struct grec {
  uint64_t w;  // packed (ts << 3) | status
  uint32_t r;  // record key = owner * S + svc
  uint32_t pad;
};
GXD grec gld_rec(const grec *p) {  // one global dwordx4 load
  const gx_u32x4 x = gld4(p);
  grec g;
  g.w = (uint64_t)x.x | ((uint64_t)x.y << 32);
  g.r = x.z;
  g.pad = x.w;
  return g;
}
GXD void gst_rec(grec *p, const grec &g) {
  gx_u32x4 x;
  x.x = (uint32_t)g.w;
  x.y = (uint32_t)(g.w >> 32);
  x.z = g.r;
  x.w = g.pad;
  gst4(p, x);
}

enum {
  C_GOSSIP_MERGES, C_AE_MERGES, C_LOCAL_MERGES, C_GOSSIP_ACC, C_AE_ACC, C_LOCAL_ACC, C_STALE,
  C_RETX, C_QDROP, C_LDROP, C_SDROP, C_PDROP, C_DEQ, C_NIL, C_PACKETS, C_RECSENT, C_EXPIRED,
  C_GC, C_OWNTOMB, C_EXPSRV, C_SENDJOBS, C_AEX, C_CHURN, C_SCANSLOTS, C_AESLOTS, C_BYTESENT,
  C_CAPCUT, C_CHG, C_QDEFER,
  // the ServicesState lock (gx.h lock_model)
  C_LOCKED_MERGES, C_LOCK_BUF, C_LOCK_DROP, C_LOCK_DRAIN, C_AE_LOCKED, C_NCTR
};
// Counters outside Acc (their own accumulators): packet loss and memberlist failure detection.
enum {
  C_LOST = C_NCTR, C_FD_PROBES, C_FD_PROBE_FAIL, C_FD_SUSPECT, C_FD_CONFIRM, C_FD_DEATH, C_FD_REFUTE,
  C_FD_ALIVE, C_FD_SENT, C_FD_RECV, C_FD_STATE_MERGE, C_EXP_DEFER, C_FEXP, C_AE_DEFER, C_AE_DEFER_LOST, C_FD_HQ, C_FD_HQ_DROP, C_NCTR_ALL
};
#define GX_NCTR_SLOTS 56
static_assert(C_NCTR_ALL <= GX_NCTR_SLOTS, "counter slots");

#define GX_SHARDS 64
// inbox slots per receiver, upper bound (gx_params.inbox_slots): the wave merge ranks up to this
// many headers in LDS; with GossipMessages > 1 the default (256) holds 17 senders' 15 packets
#define GX_DI_MAX 256
struct DevCtr {
  unsigned long long c[GX_SHARDS][GX_NCTR_SLOTS];   // counter shards (shard = block % 64)
  unsigned long long last_change_p1[GX_SHARDS][8];  // last round with a slot change + 1
  unsigned long long bytes[GX_SHARDS][16];          // algorithmic HBM bytes per kernel class
  unsigned long long units[GX_SHARDS][16];          // slots / records per kernel class
  unsigned long long first_drop[GX_SHARDS][8];      // [0] first round a LOST job was dequeued, [1] first
                                                    // round the lock held back work (min; ~0 none)
};

enum { SRC_GOSSIP = 0, SRC_AE = 1, SRC_LOCAL = 2 };
enum { ST_PEER = 1, ST_PHASE_BS = 2, ST_PHASE_BT = 3, ST_CHURN = 4, ST_INIT_TS = 5, ST_INIT_AGE = 6,
       ST_AE = 7, ST_FD_PHASE = 8, ST_FD_PERM = 9, ST_FD_RELAY = 10, ST_DEPART = 11, ST_PROBE = 12, ST_PP_PHASE = 13 };

#define XPLAN_BATCH 64  // rounds of planned-exchange slot bounds per k_xplan launch
#define XPLAN_GMAX 64   // shards the planned exchange supports

struct Dev {
  gx_params p;     // t0_ns epoch-relative (gx.h GX_TS_SHIFT)
  int64_t epoch;    // absolute time of slot time 0
  uint32_t H, S, R, Q, A, L, SQ, DQ, K;  // SQ and DQ are powers of two (ring index = position & (size - 1))
  uint32_t NG, KE;           // GossipMessages gathers per target; packet entries per host = K * NG (+ 2 probe)
  uint32_t KG;               // gossip packet entries per host, K * NG (the probe ping and ack follow, gx.h)
  uint32_t lo, Hl, G, gid;  // this engine owns hosts [lo, lo + Hl); per-host arrays are local
  uint32_t n_remote;        // packets received from other shards this round
  uint32_t *msg_key;        // [H*KE] global sender * KE + j * NG + n of each packet entry
  uint32_t *in_stamp;       // [H*KE] sharded: round + 1 when a received slot last carried the key
  int64_t round, now;
  int partitioned;
  uint64_t *view;
  unsigned long long *minexp;
  uint8_t *own_status;
  gx_host_state *hs;
  gx_job *fifo;
  gx_sleeper *sleep;
  grec *dq;
  grec *arena;
  uint32_t *arena_len;
  uint32_t AW;          // list bitmap words per host, ceil(A / 32)
  uint32_t *arena_bits; // [Hl][AW] live lists (slots >= A stay set); hs.arena_used bit w = word w full
  grec *msg;
  uint64_t *msg_w0;    // [H*K][cap] the receiver's slot word each live record was filtered against
  uint32_t *msg_len;
  uint32_t *msg_dst;
  // Receiver inboxes: a sender registers each packet straight into its receiver's
  // inbox with one atomic; the merge sorts a receiver's few headers by global sender key itself.
  uint32_t DI;         // inbox slots per receiver (<= GX_DI_MAX); packets past them go to the overflow list
  uint32_t DR;         // inbox slots whose records are stored inline (in_rec); the rest stay in msg
  // Per-round counters come in two buffers by round parity (set_round_fields): this round's, and
  // the next round's, which this round's owner phase zeroes (nothing reads it during this round),
  // so no kernel of a round has to wait for a reset of its counters.
  uint32_t *in_cnt;    // [Hl] packets registered per receiver this round
  uint32_t *in_cnt_nx; // [Hl] the same for the next round
  uint4 *in_hdr;       // [Hl][DI] {global key = sender * K + j, entry, len, slot}, arrival order
  uint4 *in_ovf;       // [H*K] {key, entry, len, local receiver} past a receiver's DI slots
  grec *in_rec;        // [Hl][DR][packet_cap] records of a receiver's first DR packets
  uint32_t *work_cnt;  // [0..1] expiry-scan worklist, [2..3] overflow list counts by round parity, [4] error bits
  uint32_t *wl_cnt, *wl_cnt_nx;    // this / next round's worklist count (into work_cnt)
  uint32_t *ovf_cnt, *ovf_cnt_nx;  // this / next round's overflow-list count
  uint32_t *work;      // [Hl] views whose expiry scan must stream the row this round
  // [Hl] live records registered for receiver vi this round (flag_live; the merge's routing hint,
  // 0 = nothing to merge), cleared by the merge
  uint32_t *mrec;
  grec *scan_list;     // [H][L] first L expired records of this round's scan
  uint32_t *scan_cnt;  // [H]
  uint8_t *tick;       // [H] BroadcastTombstones tick this round
  uint16_t *sbytes;    // [R] static encoded bytes per record key (every field but Updated/Status)
  gx_server_times *srvt;  // [Hl][H] Server.LastUpdated / LastChanged per (view, owner)
  int64_t *vlc;           // [Hl] state.LastChanged
  int32_t *ev_slot;       // [Hl] event log of a listening view, -1 = no listener
  gx_change_event *ev_log;  // [n_logs][ev_cap] ChangeEvents in processing order
  uint32_t *ev_cnt;       // [n_logs] events since the last delivery (may exceed ev_cap)
  uint32_t ev_cap;
  DevCtr *ctr;
  // memberlist failure detection (gx_fd.hpp), allocated when p.fd_enable; per-host arrays hold
  // this shard's Hl hosts (memp / dlp / fdhp), the message table also the received packets
  gx_member *mem;      // [Hl][H] member list of every host (the deadline field lives in fd_dl)
  int32_t *fd_dl;      // [Hl][H] suspicion deadlines, scanned by k_fd_tick
  gx_fd_host *fdh;     // [Hl]
  gx_fd_msg *fdm;      // [H*K][fd_msg_cap] memberlist messages of this round's packets
  uint32_t *fd_len;    // [H*K]
  uint32_t *fd_peers;  // [Hl*K] gossip targets (memberlist's kRandomNodes)
  uint32_t *fd_np;     // [Hl]
  uint64_t *fd_snap;   // [Hl][H] round-start member lists of push-pull (incarnation << 32 | state)
  int pair_split;      // push-pull pairs stay inside partition halves (scripted model)
  uint64_t divS;       // r / S as a 64x32 multiply-high (Lemire: M = (2^64 - 1) / S + 1), S > 1
  uint32_t logS;       // log2(S) when S is a power of two
  int departures;      // p.depart_round >= 0 && p.depart_ppm
  uint32_t nblk_ae;    // digest blocks per row, ceil(R / GX_DIGEST_SLOTS)
  uint64_t *snap;      // this round's k_send stores (round << 32 | work_cnt[GX_WC_SCANS]) here (pinned host memory), or null
  uint32_t sfilt;      // senders pre-filter inbound records for their local receivers (1 shard; see k_send)
  // the ServicesState lock held by a blocked looper (gx.h lock_model)
  uint32_t C;          // lock_buffer: records a locked host's inbound pipeline holds
  grec *lkb;           // [Hl][C] the records queued there, arrival order (count: hs.lock >> 8)
  uint32_t PW;         // words per host of pexp, ceil(H / 32)
  uint32_t *pexp;      // [Hl][PW] owners whose ExpireServer waits for the host's lock
  int in_round;        // a round phase is running: ExpireServer waits for the lock (ABI calls act directly)
  // gx.h lock_readers: push-pull merges of read-locked hosts waiting for their lock, in a pool of P
  // rows (host v uses slot v % P); each slot's host (GX_NOHOST = free), the pipeline places its merge
  // holds and the lowest claimant of the current batch. ro_flag[t]: pair t of the last push-pull
  // launch runs with a read-locked side (k_ae_ro takes it); ro_list: k_ae_ro's ordered list.
  uint32_t P;
  uint64_t *dpool;     // [P][R]
  uint32_t *dpool_host, *dpool_res, *dclaim;  // [P]
  uint8_t *ro_flag;    // [H]
  uint32_t *ro_list;   // [H]
  // gx.h fd_handoff_shared: memberlist messages waiting in each host's handoff queue (HQ places per
  // host, count gx_fd_host.hq_len), arrival order
  uint32_t HQ;
  gx_fd_msg *fdq;      // [Hl][HQ]
  // The planned exchange packed by k_send itself (gx_round_gossip_begin): a packet to another shard
  // is written straight into its slot of the send buffer. Set only for that launch.
  uint8_t *ob_buf;           // the send buffer (slots of 16 + 16 * packet_cap bytes), or null
  const uint32_t *ob_cnt;    // [G] slots this shard sends each shard this round (k_xplan's row, on the device)
  uint32_t *ob_claim;        // [XPLAN_GMAX] slots claimed per destination, [XPLAN_GMAX] blocks done; reset by the last block
  unsigned long long *kprof;  // diagnostics (env GX_KPROF): wall-clock phase marks of k_send per wave, or null
};

// ------------------------------------------------------------------- schedule RNG (seeded) --
GXHD uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
GXHD uint64_t rng4(uint64_t seed, uint64_t stream, uint64_t a, uint64_t b, uint64_t c) {
  uint64_t h = mix64(seed ^ (stream * 0xD1B54A32D192ED03ull));
  h = mix64(h ^ a);
  h = mix64(h ^ b);
  return mix64(h ^ c);
}
GXHD uint32_t unif(uint64_t x, uint32_t m) { return (uint32_t)(((x >> 32) * (uint64_t)m) >> 32); }
GXHD int st_of(uint64_t w) { return (int)(w & 7u); }
GXHD int64_t ts_of(uint64_t w) { return (int64_t)(w >> GX_TS_SHIFT); }
GXHD uint64_t pack(int64_t ts, int st) { return ((uint64_t)ts << GX_TS_SHIFT) | (uint64_t)st; }

// Push-pull pairing bijection on [0, m): 4-round keyed Feistel + cycle walking.
GXHD uint32_t feistel_perm(uint64_t key, uint32_t q, uint32_t m) {
  uint32_t b = 0;
  while ((1u << b) < m) b++;
  uint32_t hb = (b + 1) / 2;
  if (hb == 0) hb = 1;
  uint32_t hmask = (1u << hb) - 1;
  uint32_t x = q;
  do {
    uint32_t L = x >> hb, Rr = x & hmask;
    for (uint32_t i = 0; i < 4; i++) {
      uint32_t F = (uint32_t)(mix64(key ^ ((uint64_t)i << 32) ^ Rr)) & hmask;
      uint32_t t = Rr;
      Rr = L ^ F;
      L = t;
    }
    x = (L << hb) | Rr;
  } while (x >= m);
  return x;
}
// Its inverse: feistel_perm(key, feistel_inv(key, q, m), m) == q (each pass runs the four rounds
// backwards; cycle walking inverts by walking the inverse cycle).
GXHD uint32_t feistel_inv(uint64_t key, uint32_t q, uint32_t m) {
  uint32_t b = 0;
  while ((1u << b) < m) b++;
  uint32_t hb = (b + 1) / 2;
  if (hb == 0) hb = 1;
  uint32_t hmask = (1u << hb) - 1;
  uint32_t x = q;
  do {
    uint32_t L = x >> hb, Rr = x & hmask;
    for (int i = 3; i >= 0; i--) {  // round i: (L, R) -> (R, L ^ F_i(R))
      const uint32_t pr = L;
      L = Rr ^ ((uint32_t)(mix64(key ^ ((uint64_t)i << 32) ^ pr)) & hmask);
      Rr = pr;
    }
    x = (L << hb) | Rr;
  } while (x >= m);
  return x;
}

// Time after which TombstoneOthersServices would change this word (services_state.go:645-662):
// the slot is rewritten iff exp_time < now. ABSENT never expires.
GXHD unsigned long long exp_time(const gx_params &p, uint64_t w) {
  int st = st_of(w);
  if (st == GX_ABSENT) return ~0ull;
  int64_t life = st == GX_TOMBSTONE ? p.tombstone_lifespan_ns
                                    : (st == GX_DRAINING ? p.draining_lifespan_ns : p.alive_lifespan_ns);
  return (unsigned long long)(ts_of(w) + life);
}

// Host departures (crash) and network reachability a -> b. With the failure
// detector the partition is a network property; the scripted model samples within a side.
GXHD bool departed_at(const gx_params &p, int64_t round, uint32_t u) {
  if (p.depart_round < 0 || round < p.depart_round || !p.depart_ppm) return false;
  return (uint32_t)(rng4(p.seed, ST_DEPART, u, 0, 0) % 1000000ull) < p.depart_ppm;
}

// ------------------------------------------------------------------------------ counters --
GXD uint32_t shard_id() { return blockIdx.x & (GX_SHARDS - 1); }

GXD unsigned long long wave_sum(unsigned long long x) {
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}
GXD unsigned long long wave_min(unsigned long long x) {
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long y = __shfl_xor(x, o, 64);
    x = y < x ? y : x;
  }
  return x;
}

// Per-thread event counts; flushed once per wave (all 64 lanes must call acc_flush).
struct Acc {
  unsigned c[C_NCTR];
  bool changed;
  bool locked;  // the ServicesState lock held back (or, lock_model = 0, would have held back) work
  GXD Acc() : changed(false), locked(false) {
#pragma unroll
    for (int i = 0; i < C_NCTR; i++) c[i] = 0;
  }
};

GXD void ctr_atomic(const Dev &d, int i, unsigned long long v) {
  if (v) atomicAdd(&d.ctr->c[shard_id()][i], v);
}
GXD void mark_change(const Dev &d) {
  atomicMax(&d.ctr->last_change_p1[shard_id()][0], (unsigned long long)(d.round + 1));
}
GXD void kbytes(const Dev &d, int k, unsigned long long b, unsigned long long u) {
  if (b) atomicAdd(&d.ctr->bytes[shard_id()][k], b);
  if (u) atomicAdd(&d.ctr->units[shard_id()][k], u);
}
GXD void acc_flush(const Dev &d, const Acc &a) {
#pragma unroll  // constant indices keep Acc in registers (a rolled loop moves it to scratch)
  for (int i = 0; i < C_NCTR; i++) {
    if (__ballot(a.c[i] != 0) == 0) continue;  // most counters are zero in most waves
    unsigned long long x = wave_sum((unsigned long long)a.c[i]);
    if ((threadIdx.x & 63) == 0) ctr_atomic(d, i, x);
  }
  bool any = __ballot(a.changed) != 0;
  if ((threadIdx.x & 63) == 0 && any) mark_change(d);
  if (__ballot(a.locked) != 0 && (threadIdx.x & 63) == 0)
    atomicMin(&d.ctr->first_drop[shard_id()][1], (unsigned long long)d.round);
}

// Local index of an owned host (global id v in [lo, lo + Hl)).
GXD uint32_t li(const Dev &d, uint32_t v) { return v - d.lo; }
// Owner of record key r (r / S) without a runtime 32-bit division; exact for every 32-bit r.
GXD uint32_t owner_of(const Dev &d, uint32_t r) { return d.S == 1 ? r : (uint32_t)__umul64hi(d.divS, (uint64_t)r); }
// r belongs to owner o (r / S == o) as one range compare
GXD bool owned_by(const Dev &d, uint32_t r, uint32_t o) { return r - o * d.S < d.S; }
GXD bool departed(const Dev &d, uint32_t u) { return d.departures && departed_at(d.p, d.round, u); }

// Orders a wave's LDS and global accesses across its lanes (a team lives inside one wave).
GXD void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// ------------------------------------------------------------------------ receiver inboxes --
#define GX_ERR_INBOX 1u  // work_cnt[4]: a received packet slot failed validation (k_inbox_unpack)
#define GX_WC_ERR 4
#define GX_WC_SCANS 5  // work_cnt[5]: views streamed by expiry scans so far (wraps; differences only)
#define GX_WC_N 8
// Register a packet (global sender key, message entry) in local receiver vi's inbox: one atomic
// on the receiver's count; returns the inbox position (slot). The header itself (with the record
// count) is written by inbox_header once the packet is packed.
GXD uint32_t inbox_claim(const Dev &d, uint32_t vi) { return atomicAdd(&d.in_cnt[vi], 1u); }
// slot: where the records are (packet_recs): the inbox position (inline for the first DR), or
// 0xffffffff for the message entry
GXD void inbox_header(const Dev &d, uint32_t vi, uint32_t pos, uint32_t key, uint32_t entry, uint32_t len,
                      uint32_t slot) {
  if (pos < d.DI) d.in_hdr[(size_t)vi * d.DI + pos] = make_uint4(key, entry, len, slot);
  else d.in_ovf[atomicAdd(d.ovf_cnt, 1u)] = make_uint4(key, entry, len, vi);
}
GXD void inbox_header(const Dev &d, uint32_t vi, uint32_t pos, uint32_t key, uint32_t entry, uint32_t len) {
  inbox_header(d, vi, pos, key, entry, len, pos);
}
GXD void inbox_put(const Dev &d, uint32_t vi, uint32_t key, uint32_t entry, uint32_t len) {
  inbox_header(d, vi, inbox_claim(d, vi), key, entry, len);
}
// Where the records of a packet registered at inbox position `slot` live: inline in the receiver's
// inbox for its first DR packets, else in the sender's message entry.
GXD grec *packet_recs(const Dev &d, uint32_t vi, uint32_t slot, uint32_t entry) {
  return slot < d.DR ? &d.in_rec[((size_t)vi * d.DR + slot) * d.p.packet_cap] : &d.msg[(size_t)entry * d.p.packet_cap];
}
// Overflowed inboxes (more than DI packets): the header of receiver vi with the smallest key
// above `after` (-1: the first). O(DI + overflow list) per call; the merge then walks the inbox in
// key order one header at a time. Keys are distinct (one packet per sender slot).
GXD uint4 inbox_next(const Dev &d, uint32_t vi, int64_t after) {
  uint4 best = make_uint4(0xffffffffu, 0u, 0u, 0u);
  bool found = false;
  const uint32_t cnt = d.in_cnt[vi], n = cnt < d.DI ? cnt : d.DI;
  for (uint32_t i = 0; i < n; i++) {
    const uint4 h = d.in_hdr[(size_t)vi * d.DI + i];
    if ((int64_t)h.x > after && (!found || h.x < best.x)) {
      best = h;
      found = true;
    }
  }
  const uint32_t no = *d.ovf_cnt;
  for (uint32_t i = 0; i < no; i++) {
    const uint4 h = d.in_ovf[i];
    if (h.w == vi && (int64_t)h.x > after && (!found || h.x < best.x)) {
      best = make_uint4(h.x, h.y, h.z, 0xffffffffu);  // past DI: records in the message entry
      found = true;
    }
  }
  return best;
}
// n live records were registered for local receiver vi (no return value: the senders never wait
// for it). The merge folds exactly the receivers with a count and routes them by it (k_merge_seg).
GXD void flag_live(const Dev &d, uint32_t vi, uint32_t n) { atomicAdd(&d.mrec[vi], n); }
// memberlist state of this engine's host v (rows are shard-local, like the views)
GXD gx_member *memp(const Dev &d, uint32_t v, uint32_t m) { return &d.mem[(size_t)li(d, v) * d.H + m]; }
GXD int32_t *dlp(const Dev &d, uint32_t v, uint32_t m) { return &d.fd_dl[(size_t)li(d, v) * d.H + m]; }
GXD gx_fd_host *fdhp(const Dev &d, uint32_t v) { return &d.fdh[li(d, v)]; }
GXD bool reach(const Dev &d, uint32_t a, uint32_t b) {
  if (departed(d, a) || departed(d, b)) return false;
  return !(d.partitioned && ((a < d.H / 2) != (b < d.H / 2)));
}
GXD uint64_t *vrow(const Dev &d, uint32_t v) { return &d.view[(size_t)li(d, v) * d.R]; }
GXD gx_host_state *hst(const Dev &d, uint32_t v) { return &d.hs[li(d, v)]; }

GXD void set_slot(const Dev &d, Acc &a, uint32_t v, uint64_t *slot, uint64_t nw) {
  if (*slot != nw) {
    *slot = nw;
    a.changed = true;
    atomicMin(&d.minexp[li(d, v)], exp_time(d.p, nw));
  }
}

// ------------------------------------------------ the ServicesState lock --
// BroadcastServices blocks on its nil holding state.RLock() (services_state.go:535-536,569),
// BroadcastTombstones holding state.Lock() (:610-611,628). Host v is locked for round n iff one of
// them was blocked at the start of round n: bit (n & 1) of its lock word (gx.h gx_host_state.lock),
// written for round n + 1 when v's round-n GetBroadcasts calls end, so every phase of a round reads
// one value and another host's team may read it while v's team rewrites the other bit.
GXD bool locked_in(const Dev &d, uint32_t lockw) { return GX_LOCK_AT(lockw, d.round) != 0u; }
GXD bool host_locked(const Dev &d, uint32_t v) { return locked_in(d, gld(&hst(d, v)->lock)); }
// the lock word with bit `round & 1` set from the loopers' state
// (and with gx.h lock_readers, bit 4 + (round & 1) from BroadcastTombstones' write lock alone)
GXD uint32_t lock_snap(uint32_t lockw, uint32_t flags, int64_t round, bool rw) {
  const uint32_t b = 1u << (round & 1), w = 16u << (round & 1);
  lockw = (lockw & ~b) | ((flags & 3u) ? b : 0u);
  return rw ? (lockw & ~w) | ((flags & 2u) ? w : 0u) : lockw;
}
// gx.h lock_readers: host v holds the lock this round and LocalState's RLock would still succeed
// (services_delegate.go:148 behind BroadcastServices' read lock, services_state.go:535): the write
// lock did not hold it at the round's start and no writer waits (no record in the pipeline, no
// waiting ExpireServer or merge, no BroadcastTombstones tick due). Oracle: ro_side.
#define GX_NOHOST 0xffffffffu
GXD bool ro_side(const Dev &d, uint32_t v) {
  const gx_host_state *h = hst(d, v);
  const uint32_t lw = gld(&h->lock);
  return d.p.lock_readers && locked_in(d, lw) && !GX_LOCK_W_AT(lw, d.round) && GX_LOCK_BUF(lw) == 0u &&
         !(lw & (GX_LOCK_PENDING_EXPIRE | GX_LOCK_DEFER_MERGE)) && h->bt_next > d.round;
}
// a locked pair whose locked sides are all read-locked with no writer waiting: it runs (k_ae_ro)
GXD bool ro_pair(const Dev &d, uint32_t a, uint32_t b) {
  return d.p.lock_readers && (!host_locked(d, a) || ro_side(d, a)) && (!host_locked(d, b) || ro_side(d, b));
}
// the inbound pipeline's room for gossip records of local host vi with lock word lw: a waiting merge
// holds min(n, 26) of its places (gx.h GX_LOCK_DEFER_RES). Oracle: pipe_cap.
GXD uint32_t pipe_cap(const Dev &d, uint32_t vi, uint32_t lw) {
  if (!(lw & GX_LOCK_DEFER_MERGE)) return d.C;
  const uint32_t res = d.dpool_res[(d.lo + vi) % d.P];
  return d.C > res ? d.C - res : 0u;
}
GXD void note_locked(const Dev &d) { atomicMin(&d.ctr->first_drop[shard_id()][1], (unsigned long long)d.round); }

// --------------------------------------------------- change bookkeeping --
GXD gx_server_times *srv_times(const Dev &d, uint32_t v, uint32_t o) {
  return &d.srvt[(size_t)li(d, v) * d.H + o];
}
// ChangeEvent at position pos of view v's log (listening views only).
GXD void ev_put(const Dev &d, int32_t k, uint32_t pos, uint32_t r, uint64_t nw, int prev) {
  if (pos >= d.ev_cap) return;
  gx_change_event ev;
  ev.service.updated_ns = ts_of(nw);
  ev.service.host = r / d.S;
  ev.service.svc = (uint16_t)(r % d.S);
  ev.service.status = (uint8_t)st_of(nw);
  ev.service.flags = 0;
  ev.time_ns = ts_of(nw);
  ev.previous_status = (uint32_t)prev;
  ev.pad = 0;
  d.ev_log[(size_t)k * d.ev_cap + pos] = ev;
}
// ServiceChanged (services_state.go:195-199) from a path that owns view v alone (one thread).
GXD void svc_changed(const Dev &d, Acc &a, uint32_t v, uint32_t r, uint64_t nw, int prev) {
  int64_t ts = ts_of(nw);
  gx_server_times *t = srv_times(d, v, owner_of(d, r));
  t->last_updated_ns = ts;
  t->last_changed_ns = ts;
  d.vlc[li(d, v)] = ts;
  a.c[C_CHG]++;
  int32_t k = d.ev_slot[li(d, v)];
  if (k >= 0) ev_put(d, k, d.ev_cnt[k]++, r, nw, prev);
}

// ----------------------------------------------------------------------- broadcast FIFO --
// The unbuffered Broadcasts channel's blocked senders (services_state.go:94): the reference never
// refuses one, so every push is accepted. The first Q jobs are stored; a job pushed while the
// stored window is full, or behind a deferred job, is deferred (counted in place, contents
// dropped); a looper's nil keeps its position (gx.h gx_job).
GXD gx_job make_job(uint64_t a, uint32_t c, uint32_t meta) {
  gx_job j;
  j.a = a;
  j.c = c;
  j.meta = meta;
  return j;
}
GXHD uint32_t meta_of(int kind, uint32_t pass, uint32_t np) { return GX_JOB_META((uint32_t)kind, pass, np, 0); }
// Jobs a push of several may store at the tail: the window's free room, or 0 behind deferred jobs.
GXD uint32_t fifo_room(const Dev &d, uint32_t head, uint32_t tail, uint32_t stored) {
  return stored == tail ? d.Q - (stored - head) : 0u;
}

// List arena: the lowest free slot, a two-level bitmap (hs.arena_used bit w = bitmap word w full).
// The bitmap word is read and written by one lane of the host's team (lane0).
GXD uint32_t *list_bits(const Dev &d, uint32_t vi, uint32_t w) { return &d.arena_bits[(size_t)vi * d.AW + w]; }
GXD void list_release(const Dev &d, uint32_t vi, uint32_t &arena_used, uint32_t slot, bool lane0) {
  if (slot >= d.A) return;  // GX_LIST_NONE: a SendServices job queued deferred holds no list
  // (a non-returning atomic: the sends do not wait for the word; only this host's team touches it)
  if (lane0) atomicAnd(list_bits(d, vi, slot >> 5), ~(1u << (slot & 31)));
  arena_used &= ~(1u << (slot >> 5));
}
// Allocates on the team-uniform register copy `arena_used`; -1 when every slot is live. Every
// lane of the team of T lanes calls it; the team's lane 0 loads and stores the word.
template <int T = 1>
GXD int list_alloc(const Dev &d, uint32_t vi, uint32_t &arena_used, bool lane0) {
  const uint32_t wfree = ~arena_used & (d.AW >= 32 ? 0xffffffffu : ((1u << d.AW) - 1u));
  if (!wfree) return -1;
  const uint32_t w = (uint32_t)__builtin_ctz(wfree);
  uint32_t *p = list_bits(d, vi, w);
  // atomic (L2) accesses: list_release clears bits with a non-returning atomic, which a plain load
  // of the same launch could miss in the vector L1
  uint32_t word = lane0 ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
  if (T > 1) word = (uint32_t)__shfl((int)word, 0, T);
  const uint32_t b = (uint32_t)__builtin_ctz(~word), nw = word | (1u << b);
  if (lane0) __hip_atomic_store(p, nw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (nw == 0xffffffffu) arena_used |= 1u << w;
  return (int)(w * 32 + b);
}
GXD void free_list_r(const Dev &d, uint32_t vi, gx_host_state &hs, const gx_job &j, bool lane0) {
  if (GX_JOB_KIND(j.meta) == GX_JOB_SEND) list_release(d, vi, hs.arena_used, j.c & 0xffff, lane0);
}

// The FIFO pushes of one host, on its register copy `hs` (the whole team holds the same copy;
// lane 0 stores).
GXD void push_job_r(const Dev &d, Acc &a, uint32_t v, gx_host_state &hs, const gx_job &j, bool lane0) {
  const uint32_t kind = GX_JOB_KIND(j.meta);
  if (kind == GX_JOB_NIL_BS) hs.nil_pos_bs = hs.fifo_tail;
  else if (kind == GX_JOB_NIL_BT) hs.nil_pos_bt = hs.fifo_tail;
  if (fifo_room(d, hs.fifo_head, hs.fifo_tail, hs.fifo_stored)) {
    if (lane0) d.fifo[(size_t)li(d, v) * d.Q + (hs.fifo_tail % d.Q)] = j;
    hs.fifo_stored++;
  } else {
    if (lane0) a.c[C_QDEFER]++;
    free_list_r(d, li(d, v), hs, j, lane0);  // only a LOST dequeue could reach it
  }
  hs.fifo_tail++;
}
GXD void push_sleep_r(const Dev &d, Acc &a, uint32_t v, gx_host_state &hs, const gx_job &j, uint32_t wake,
                      bool lane0) {
  if (hs.sleep_tail - hs.sleep_head >= d.SQ) {
    if (lane0) a.c[C_SDROP]++;
    free_list_r(d, li(d, v), hs, j, lane0);
    return;
  }
  if (lane0) {  // two 16-B stores: the job, then wake and padding
    gx_sleeper *z = &d.sleep[(size_t)li(d, v) * d.SQ + (hs.sleep_tail & (d.SQ - 1u))];
    gx_u32x4 x0, x1;
    x0.x = (uint32_t)j.a;
    x0.y = (uint32_t)(j.a >> 32);
    x0.z = j.c;
    x0.w = j.meta;
    x1.x = wake;
    x1.y = x1.z = x1.w = 0u;
    gst4(&z->job, x0);
    gst4(&z->wake, x1);
  }
  hs.sleep_tail++;
}
// Scalar forms (one thread owns host v's bookkeeping), field by field (a copy of the whole
// bookkeeping struct would go through scratch memory).
GXD void push_job(const Dev &d, Acc &a, uint32_t v, const gx_job &j) {
  gx_host_state *h = hst(d, v);
  const uint32_t kind = GX_JOB_KIND(j.meta), tail = h->fifo_tail, stored = h->fifo_stored;
  if (kind == GX_JOB_NIL_BS) h->nil_pos_bs = tail;
  else if (kind == GX_JOB_NIL_BT) h->nil_pos_bt = tail;
  if (fifo_room(d, h->fifo_head, tail, stored)) {
    d.fifo[(size_t)li(d, v) * d.Q + (tail % d.Q)] = j;
    h->fifo_stored = stored + 1;
  } else {
    a.c[C_QDEFER]++;
    if (kind == GX_JOB_SEND) {  // only a LOST dequeue could reach it
      uint32_t au = h->arena_used;
      list_release(d, li(d, v), au, j.c & 0xffff, true);
      h->arena_used = au;
    }
  }
  h->fifo_tail = tail + 1;
}
GXD void free_list(const Dev &d, uint32_t v, const gx_job &j) {
  gx_host_state *h = hst(d, v);
  uint32_t au = h->arena_used;
  if (GX_JOB_KIND(j.meta) == GX_JOB_SEND) list_release(d, li(d, v), au, j.c & 0xffff, true);
  h->arena_used = au;
}

// TimedLooper re-arm (services_state.go:585-601): due passes re-enter the FIFO tail.
GXD void wake_host(const Dev &d, Acc &a, uint32_t v) {
  gx_host_state *h = hst(d, v);
  while (h->sleep_head != h->sleep_tail) {
    const gx_sleeper &z = d.sleep[(size_t)li(d, v) * d.SQ + (h->sleep_head & (d.SQ - 1u))];
    if ((int64_t)z.wake > d.round) break;
    const gx_job j = z.job;
    h->sleep_head++;
    push_job(d, a, v, j);
  }
}

// Take the FIFO head (fifo_head != fifo_tail) on the register copy: a stored job, or, past the
// stored window, a looper's nil at its kept position, else LOST (the caller counts it). `pj`:
// the head job when the caller loaded it ahead (stored jobs only).
GXD gx_job pop_job_r(const Dev &d, uint32_t vi, gx_host_state &hs, const gx_job *pj) {
  const uint32_t p = hs.fifo_head++;
  if (p != hs.fifo_stored) return pj ? *pj : d.fifo[(size_t)vi * d.Q + (p % d.Q)];
  hs.fifo_stored = hs.fifo_head;  // the stored window restarts behind the deferred job
  uint32_t kind = GX_JOB_LOST;
  if ((hs.flags & 1u) && p == hs.nil_pos_bs) kind = GX_JOB_NIL_BS;
  else if ((hs.flags & 2u) && p == hs.nil_pos_bt) kind = GX_JOB_NIL_BT;
  return make_job(0, 0, meta_of((int)kind, 0, 1));
}
GXD void count_lost(const Dev &d, Acc &a, bool lane0) {
  if (!lane0) return;
  a.c[C_QDROP]++;
  atomicMin(&d.ctr->first_drop[shard_id()][0], (unsigned long long)d.round);
}

// (base + k) % q for base < q and k < q, without a division
GXD uint32_t ring_add(uint32_t base, uint32_t k, uint32_t q) {
  const uint32_t x = base + k;
  return x >= q ? x - q : x;
}

// Lowest free list slot, or -1 (the caller queues a LOST job: list_drops).
GXD int alloc_list(const Dev &d, Acc &a, uint32_t v) {
  gx_host_state *h = hst(d, v);
  uint32_t au = h->arena_used;
  const int slot = list_alloc(d, li(d, v), au, true);
  if (slot < 0) a.c[C_LDROP]++;
  h->arena_used = au;
  return slot;
}
GXD grec *list_ptr(const Dev &d, uint32_t v, uint32_t slot) {
  return &d.arena[((size_t)li(d, v) * d.A + slot) * d.L];
}
// SendServices job over an allocated, filled list (services_state.go:579-604); slot < 0: the list
// did not fit, the job is queued LOST.
GXD void commit_send(const Dev &d, Acc &a, uint32_t v, int slot, uint32_t n, uint32_t npasses) {
  if (slot >= 0) d.arena_len[(size_t)li(d, v) * d.A + slot] = n;
  push_job(d, a, v, slot >= 0 ? make_job(0, (uint32_t)slot | (n << 16), meta_of(GX_JOB_SEND, 0, npasses))
                              : make_job(0, 0, meta_of(GX_JOB_LOST, 0, 1)));
}
// Whether the next push of host v is stored (a deferred SendServices job takes no list).
GXD bool fifo_stores(const Dev &d, uint32_t v) {
  const gx_host_state *h = hst(d, v);
  return fifo_room(d, h->fifo_head, h->fifo_tail, h->fifo_stored) != 0;
}

GXD uint32_t job_len(const Dev &d, const gx_job &j) {
  uint32_t kind = GX_JOB_KIND(j.meta);
  if (kind == GX_JOB_RETX) return 1;
  if (kind == GX_JOB_SEND) return j.c >> 16;
  if (kind == GX_JOB_EXPIRE) return (uint32_t)__popcll(j.a);
  return 0;
}


// GetBroadcasts(overhead, limit) + packPacket (services_delegate.go:85-144, :186-223).
// ---------------------------------------------------------- encoded message length (f-1) --
// len(Service.Encode()) (service/service_ffjson.go:370-436): the static fields come from the
// per-record table; "Updated" is time.Time.MarshalJSON = quoted RFC3339Nano in UTC:
// "YYYY-MM-DDTHH:MM:SS" + ("." + fraction without trailing zeros, omitted when zero) + "Z";
// "Status" is FormatBits2 decimal.
GXHD uint32_t json_time_len(int64_t ts) {
  int64_t f = ts % 1000000000ll;
  if (f < 0) f += 1000000000ll;
  if (f == 0) return 22;
  uint32_t n = 9;
  while (f % 10 == 0) {
    f /= 10;
    n--;
  }
  return 23 + n;
}
GXHD uint32_t dec_len(uint32_t x) { return x >= 100 ? 3 : x >= 10 ? 2 : 1; }
GXD uint32_t msg_bytes(const Dev &d, const grec &g) {
  return d.sbytes[g.r] + json_time_len(ts_of(g.w)) + dec_len((uint32_t)st_of(g.w));
}

// Position of the n-th (0-based) set bit of m (n < popcount(m)).
GXD uint32_t nth_set_bit(uint64_t m, uint32_t n) {
  uint32_t pos = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    uint64_t low = m & ((1ull << w) - 1);
    uint32_t c = (uint32_t)__popcll(low);
    if (n >= c) {
      n -= c;
      m >>= w;
      pos += w;
    } else {
      m = low;
    }
  }
  return pos;
}
// Inclusive scan over the T lanes of a team (tl = lane within the team).
template <int T>
GXD uint32_t team_incl_scan(uint32_t x, uint32_t tl) {
#pragma unroll
  for (int o = 1; o < T; o <<= 1) {
    uint32_t y = __shfl_up(x, o, T);
    if ((int)tl >= o) x += y;
  }
  return x;
}

// GetBroadcasts (services_delegate.go:85-144) with packPacket (:186-223) by a team of T lanes
// per host: the control state is the team-uniform register copy `hs`, the records move
// lane-parallel. broadcast = batch ++ pendingBroadcasts is read as a virtual sequence (batch
// record i from the job, then the pending ring); only the batch records that stay pending are
// written to the ring. limit = record budget (the packet buffer); limit_bytes > 0 adds the byte
// budget + overhead. Every lane of the team calls it; ring writes are fenced before the next call.
// pj: the job at the FIFO head when the caller loaded it ahead of the call (LDS), else null.
template <int T>
GXD uint32_t get_broadcasts_team(const Dev &d, Acc &a, uint32_t v, gx_host_state &hs, uint32_t limit,
                                 grec *packet, uint32_t limit_bytes, uint32_t overhead,
                                 const gx_job *pj = nullptr, const uint64_t *rrow = nullptr,
                                 uint32_t rvi = 0) {
  const uint32_t lane = threadIdx.x & 63, tl = lane & (T - 1), tw = lane / T;
  const bool lane0 = tl == 0;
  const uint32_t mask = d.DQ - 1;
  grec *dq = &d.dq[(size_t)li(d, v) * d.DQ];
  gx_job j = make_job(0, 0, 0);
  uint32_t m = 0;
  if (hs.fifo_head != hs.fifo_tail) {  // case broadcast = <-d.state.Broadcasts (:94)
    j = pop_job_r(d, li(d, v), hs, pj);
    if (lane0) a.c[C_DEQ]++;
    m = job_len(d, j);
    uint32_t kind = GX_JOB_KIND(j.meta), pass = GX_JOB_PASS(j.meta), np = GX_JOB_NPASSES(j.meta);
    if (kind == GX_JOB_LOST) {  // a deferred job reached the head: its batch is unknown
      count_lost(d, a, lane0);
    } else if (kind == GX_JOB_NIL_BS) {  // the BroadcastServices looper unblocks (services_state.go:569)
      if (lane0) a.c[C_NIL]++;
      hs.flags &= ~1u;
      hs.bs_next = d.round + d.p.alive_interval_rounds;
    } else if (kind == GX_JOB_NIL_BT) {  // ... BroadcastTombstones (:628)
      if (lane0) a.c[C_NIL]++;
      hs.flags &= ~2u;
      hs.bt_next = d.round + d.p.tombstone_interval_rounds;
    } else if (kind == GX_JOB_SEND || kind == GX_JOB_EXPIRE) {
      if (pass + 1 < np) {  // the looper re-arms (services_state.go:585-601)
        gx_job nj = j;
        nj.meta = GX_JOB_META(kind, pass + 1, np, GX_JOB_OWNER(j.meta));
        if (d.p.retransmit_rounds == 0) push_job_r(d, a, v, hs, nj, lane0);
        else push_sleep_r(d, a, v, hs, nj, (uint32_t)(d.round + d.p.retransmit_rounds), lane0);
      } else {
        free_list_r(d, li(d, v), hs, j, lane0);  // the list is read below; nothing reallocates it in this call
      }
    }
  } else if (hs.dq_len == 0) {  // default: nothing pending (:96-98)
    return 0;
  }
  const uint32_t head = hs.dq_head, n = m + hs.dq_len;
  const uint32_t kind = GX_JOB_KIND(j.meta), pass = GX_JOB_PASS(j.meta);
  const uint64_t dw = ((uint64_t)pass * (uint64_t)d.p.pass_increment_ns) << GX_TS_SHIFT;
  auto item = [&](uint32_t i) -> grec {  // element i of batch ++ pendingBroadcasts
    grec g;
    g.pad = 0;
    if (i >= m) return dq[(head + (i - m)) & mask];
    if (kind == GX_JOB_RETX) {
      g.w = j.a;
      g.r = j.c;
    } else if (kind == GX_JOB_SEND) {  // Updated + pass * 50ns (services_state.go:588-599)
      grec s = list_ptr(d, v, j.c & 0xffff)[i];
      g.w = s.w + dw;
      g.r = s.r;
    } else {  // EXPIRE: the i-th tombstoned service of the owner, at the call's now
      g.w = pack(d.p.t0_ns + (int64_t)j.c * d.p.round_ns, GX_TOMBSTONE) + dw;
      g.r = GX_JOB_OWNER(j.meta) * d.S + nth_set_bit(j.a, i);
    }
    return g;
  };
  // packPacket (:186-223): the greedy prefix within the limit
  const uint32_t nmax = n < limit ? n : limit;
  uint32_t l = nmax;
  if (limit_bytes) {
    uint64_t total = 0;
    l = 0;
    const uint64_t tmask = T == 64 ? ~0ull : ((1ull << T) - 1);
    for (uint32_t c0 = 0; c0 < nmax; c0 += T) {
      uint32_t i = c0 + tl;
      uint32_t b = i < nmax ? msg_bytes(d, item(i)) + overhead : 0;
      uint32_t incl = team_incl_scan<T>(b, tl);
      bool fits = i < nmax && total + incl <= limit_bytes;  // total+len(message)+overhead > limit (:195)
      // prefix sums rise, so the fitting lanes are a prefix of the team
      uint32_t k = (uint32_t)__popcll((__ballot(fits) >> (tw * T)) & tmask);
      if (k) total += __shfl(incl, (int)k - 1, T);
      l += k;
      uint32_t chunk = nmax - c0 < T ? nmax - c0 : T;
      if (k < chunk) break;
    }
    if (lane0) {
      if (l == nmax && nmax < n && total + msg_bytes(d, item(nmax)) + overhead <= limit_bytes) a.c[C_CAPCUT]++;
      a.c[C_BYTESENT] += (unsigned)total;
    }
  }
  // Ring position p is read and written only by team lane p % T (T divides DQ), so a record that
  // a call leaves pending is seen by the same lane in the next call without a fence; batch records
  // (list arena, job) and packet slots are not written and read back here, any lane moves them.
  // Send-side filter (rrow: the local receiver's view row): a record that is stale, or no newer
  // than the receiver's slot, is a no-op in the receiver's merge whatever the other packets hold
  // (see k_merge). Phases 0-3 only raise a slot's timestamp, except the expiry scan's GC of a
  // tombstone older than the tombstone lifespan, which is read as absent; so a record this sees
  // as a no-op is one, and the receiver is flagged for k_merge only when some record is live.
  // The senders count the receivers' gossip merges and stale drops (k_merge then does not).
  uint32_t nlv = 0, fm = 0, fs = 0;
  const int64_t t_stale = d.now - d.p.tombstone_lifespan_ns - d.p.stale_fudge_ns;
  const int64_t t_gc = d.now - d.p.tombstone_lifespan_ns;
  auto filt = [&](const grec &g) {
    const uint64_t w0 = rrow[g.r];
    const int64_t ts = ts_of(g.w);
    const bool stale = ts < t_stale;
    const bool gc = st_of(w0) == GX_TOMBSTONE && ts_of(w0) < t_gc;
    nlv += !stale && (st_of(w0) == GX_ABSENT || ts > ts_of(w0) || gc);
    fm++;
    fs += stale;
  };
  const uint32_t lb = l < m ? l : m;
  for (uint32_t i = tl; i < lb; i += T) {
    const grec g = item(i);
    packet[i] = g;
    if (rrow) filt(g);
  }
  if (l > m)  // the pending prefix, ring positions head .. head + l - m - 1, by their owner lanes
    for (uint32_t q = (tl - head) & (T - 1); q < l - m; q += T) {
      const grec g = dq[(head + q) & mask];
      packet[m + q] = g;
      if (rrow) filt(g);
    }
  if (rrow) {
    a.c[C_GOSSIP_MERGES] += fm;
    a.c[C_STALE] += fs;
    if (nlv) flag_live(d, rvi, nlv);  // each lane its live records
  }
  // leftover = broadcast[l:]; batch records that stay pending go in front of the old head
  uint32_t nh;
  if (l < m) {
    uint32_t k = m - l;
    nh = (head - k) & mask;
    for (uint32_t q = (tl - nh) & (T - 1); q < k; q += T) dq[(nh + q) & mask] = item(l + q);
  } else {
    nh = (head + (l - m)) & mask;
  }
  hs.dq_head = nh;
  hs.dq_len = n - l;
  if (hs.dq_len > d.p.pending_cap) {  // pendingBroadcasts = leftover[:MAX_PENDING_LENGTH]
    if (lane0) a.c[C_PDROP] += hs.dq_len - d.p.pending_cap;
    hs.dq_len = d.p.pending_cap;
  }
  if (l && lane0) {
    a.c[C_PACKETS]++;
    a.c[C_RECSENT] += l;
  }
  // Byte mode reads ring records on any lane (the byte scan), and with no retransmit sleep a
  // re-armed job is pushed to the FIFO and may be dequeued by the next call: those need the fence.
  if (limit_bytes || d.p.retransmit_rounds == 0) __threadfence_block();
  return l;
}

// ------------------------------------------------------------------------ merge rule (a-5) --
// AddServiceEntry core on one slot word (services_state.go:293-347): returns the new word and
// sets acc when the record was stored; stale when IsStale dropped it (service.go:68-72).
GXD uint64_t merge_word(const Dev &d, uint64_t old, uint64_t u, bool &acc, bool &stale) {
  int64_t ts = ts_of(u);
  acc = false;
  stale = false;
  if (ts < d.now - d.p.tombstone_lifespan_ns - d.p.stale_fudge_ns) {
    stale = true;
    return old;
  }
  if (st_of(old) == GX_ABSENT) {  // !server.HasService: insert (:317-320)
    acc = true;
    return u;
  }
  if (ts > ts_of(old)) {  // Invalidates: strictly newer (:321)
    int st = st_of(u);
    if (st_of(old) == GX_DRAINING && st == GX_ALIVE) st = GX_DRAINING;  // (:329-331)
    acc = true;
    return pack(ts, st);
  }
  return old;
}

GXD bool add_entry(const Dev &d, Acc &a, uint32_t v, grec u, int src) {
  a.c[src == SRC_GOSSIP ? C_GOSSIP_MERGES : src == SRC_AE ? C_AE_MERGES : C_LOCAL_MERGES]++;
  uint64_t *slot = &vrow(d, v)[u.r];
  bool acc, stale;
  uint64_t nw = merge_word(d, *slot, u.w, acc, stale);
  if (stale) {
    a.c[C_STALE]++;
    return false;
  }
  if (!acc) return false;
  uint64_t old = *slot;
  set_slot(d, a, v, slot, nw);
  if (st_of(old) == GX_ABSENT) {
    svc_changed(d, a, v, u.r, nw, GX_UNKNOWN);  // ServiceChanged(&newSvc, UNKNOWN, ...) (:319)
  } else {
    srv_times(d, v, u.r / d.S)->last_updated_ns = ts_of(nw);  // server.LastUpdated (:323)
    if (st_of(old) != st_of(nw)) svc_changed(d, a, v, u.r, nw, st_of(old));  // (:338-340)
  }
  a.c[src == SRC_GOSSIP ? C_GOSSIP_ACC : src == SRC_AE ? C_AE_ACC : C_LOCAL_ACC]++;
  if (u.r / d.S != v) {  // retransmit foreign records only (services_state.go:377-392)
    push_job(d, a, v, make_job(nw, u.r, meta_of(GX_JOB_RETX, 0, 1)));
    a.c[C_RETX]++;
  }
  return true;
}

// Expiry rule of TombstoneOthersServices on one slot (services_state.go:645-679).
GXD uint64_t expiry_word(const Dev &d, uint64_t w, bool &expired, bool &gc) {
  expired = false;
  gc = false;
  int st = st_of(w);
  if (st == GX_ABSENT) return w;
  int64_t ts = ts_of(w);
  if (st == GX_TOMBSTONE) {
    if (ts < d.now - d.p.tombstone_lifespan_ns) {
      gc = true;
      return GX_SLOT_ABSENT;
    }
    return w;
  }
  int64_t life = st == GX_DRAINING ? d.p.draining_lifespan_ns : d.p.alive_lifespan_ns;
  if (ts < d.now - life) {
    expired = true;
    return pack(ts + d.p.tombstone_bump_ns, GX_TOMBSTONE);
  }
  return w;
}

// TombstoneServices(self, list) on the owner's own slots (services_state.go:685-715).
// Returns the mask of services tombstoned (each contributes the record twice).
GXD uint64_t tombstone_services(const Dev &d, Acc &a, uint32_t o, uint64_t running) {
  uint64_t *row = &vrow(d, o)[(size_t)o * d.S];
  uint64_t m = 0;
  for (uint32_t s = 0; s < d.S; s++) {
    if ((running >> s) & 1ull) continue;  // running: no slot read (each read waits on the last store)
    uint64_t w = row[s];
    if (st_of(w) == GX_ABSENT || st_of(w) == GX_TOMBSTONE) continue;
    set_slot(d, a, o, &row[s], pack(d.now, GX_TOMBSTONE));  // svc.Tombstone() (service.go:91-94)
    svc_changed(d, a, o, o * d.S + s, row[s], st_of(w));     // (:703-705)
    m |= 1ull << s;
  }
  a.c[C_OWNTOMB] += (unsigned)__popcll(m);
  return m;
}

// ExpireServer (services_state.go:150-192) for one (viewer, owner).
GXD bool expire_server(const Dev &d, Acc &a, uint32_t v, uint32_t o) {
  uint64_t *row = &vrow(d, v)[(size_t)o * d.S];
  const uint64_t nw = pack(d.now, GX_TOMBSTONE);
  uint64_t mask = 0, diff = 0;
  bool live = false;
  for (uint32_t s = 0; s < d.S; s++) {
    const uint64_t w = row[s];
    int st = st_of(w);
    if (st == GX_ABSENT) continue;
    mask |= 1ull << s;
    if (w != nw) diff |= 1ull << s;
    if (st != GX_TOMBSTONE) live = true;
  }
  if (!live) return false;  // no server / no services / no live services (:154-170)
  // Tombstone() + ServiceChanged for every record (:176-181). Every record gets the same word and
  // the same owner, so the per-record bookkeeping (set_slot's expiry bound, svc_changed's server
  // times and view LastChanged) collapses to one update each; the ChangeEvents (listening views
  // only) go out in record order, before the slots are overwritten. The slot stores then issue
  // back to back, with no load between them.
  const int32_t k = d.ev_slot[li(d, v)];
  if (k >= 0)
    for (uint32_t s = 0; s < d.S; s++)
      if ((mask >> s) & 1ull) ev_put(d, k, d.ev_cnt[k]++, o * d.S + s, nw, st_of(row[s]));
  for (uint32_t s = 0; s < d.S; s++)
    if ((diff >> s) & 1ull) row[s] = nw;
  if (diff) {
    a.changed = true;
    atomicMin(&d.minexp[li(d, v)], exp_time(d.p, nw));
  }
  gx_server_times *t = srv_times(d, v, o);
  t->last_updated_ns = ts_of(nw);
  t->last_changed_ns = ts_of(nw);
  d.vlc[li(d, v)] = ts_of(nw);
  a.c[C_CHG] += (unsigned)__popcll(mask);
  a.c[C_EXPSRV]++;
  push_job(d, a, v, make_job(mask, (uint32_t)d.round, GX_JOB_META(GX_JOB_EXPIRE, 0, d.p.tombstone_count, o)));
  return true;
}

// NotifyLeave -> go ExpireServer(node) (services_delegate.go:173-176) inside a round phase:
// ExpireServer takes state.Lock() (services_state.go:151), so on a locked host the call waits (a
// bit in pexp); the waiting calls run in owner order at the end of the owner phase of the host's
// first unlocked round (run_pending_expires). One thread owns host v here.
GXD void notify_leave(const Dev &d, Acc &a, uint32_t v, uint32_t o) {
  gx_host_state *h = hst(d, v);
  if (d.p.lock_model && d.in_round && locked_in(d, h->lock)) {
    d.pexp[(size_t)li(d, v) * d.PW + (o >> 5)] |= 1u << (o & 31);
    h->lock |= GX_LOCK_PENDING_EXPIRE;
    ctr_atomic(d, C_EXP_DEFER, 1);
    return;
  }
  expire_server(d, a, v, o);
}
GXD void run_pending_expires(const Dev &d, Acc &a, uint32_t v) {
  uint32_t *w = &d.pexp[(size_t)li(d, v) * d.PW];
  for (uint32_t k = 0; k < d.PW; k++) {
    uint32_t x = w[k];
    if (!x) continue;
    w[k] = 0;
    for (; x; x &= x - 1) expire_server(d, a, v, k * 32 + (uint32_t)__builtin_ctz(x));
  }
  hst(d, v)->lock &= ~GX_LOCK_PENDING_EXPIRE;
}

GXD bool is_new(const Dev &d, uint32_t o, uint64_t sw, uint32_t r) {
  uint64_t w = vrow(d, o)[r];
  return st_of(w) == GX_ABSENT || (st_of(sw) != GX_TOMBSTONE && st_of(sw) != st_of(w));
}

// BroadcastServices looper body (services_state.go:525-574) over fn() = list (n <= 64).
// Sets inc = bit i for each list element handed to SendServices (0 = a nil was sent).
GXD void bs_body_list(const Dev &d, Acc &a, uint32_t o, const grec *list, uint32_t n, uint64_t &inc_out) {
  gx_host_state *h = hst(d, o);
  bool refresh = (d.now - d.p.alive_broadcast_interval_ns) > h->last_bcast_ns;  // (:547)
  bool any_new = false;
  uint64_t inc = 0;
  for (uint32_t i = 0; i < n; i++) {
    if (is_new(d, o, list[i].w, list[i].r)) {  // IsNewService (:509-521)
      any_new = true;
      inc |= 1ull << i;
    } else if (refresh) {
      inc |= 1ull << i;
    }
  }
  inc_out = inc;
  if (inc) {
    h->last_bcast_ns = d.now;
    a.c[C_SENDJOBS]++;
    uint32_t m = 0;
    for (uint32_t i = 0; i < n && m < d.L; i++) m += (inc >> i) & 1ull;
    if (!fifo_stores(d, o)) {  // deferred: no list
      push_job(d, a, o, make_job(0, GX_LIST_NONE, meta_of(GX_JOB_SEND, 0, any_new ? d.p.alive_count : 1)));
    } else {
      int slot = alloc_list(d, a, o);
      if (slot >= 0) {
        grec *dst = list_ptr(d, o, slot);
        uint32_t k = 0;
        for (uint32_t i = 0; i < n && k < d.L; i++)
          if ((inc >> i) & 1ull) dst[k++] = list[i];
      }
      commit_send(d, a, o, slot, m, any_new ? d.p.alive_count : 1);  // ALIVE_COUNT if new (:555-558)
    }
  } else {
    push_job(d, a, o, make_job(0, 0, meta_of(GX_JOB_NIL_BS, 0, 1)));  // Broadcasts <- nil (:569)
    h->flags |= 1u;  // the looper blocks until the nil is consumed
  }
}

// Second half of the BroadcastTombstones body (services_state.go:613-629), after the view scan
// left the first L expired records (key order) in `others`.
GXD void bt_finish(const Dev &d, Acc &a, uint32_t o, uint64_t running, const grec *others, uint32_t n_others) {
  gx_host_state *h = hst(d, o);
  uint64_t own = tombstone_services(d, a, o, running);
  uint32_t n_own = 2u * (uint32_t)__popcll(own);
  if (n_own + n_others > 0) {
    a.c[C_SENDJOBS]++;
    int slot = fifo_stores(d, o) ? alloc_list(d, a, o) : -2;  // a deferred job takes no list
    const uint32_t len = n_own + n_others < d.L ? n_own + n_others : d.L;
    if (slot == -2) push_job(d, a, o, make_job(0, GX_LIST_NONE, meta_of(GX_JOB_SEND, 0, d.p.tombstone_count)));
    else if (slot < 0) commit_send(d, a, o, slot, len, d.p.tombstone_count);
    if (slot >= 0) {
      grec *dst = list_ptr(d, o, slot);
      uint32_t m = 0;
      uint64_t w = pack(d.now, GX_TOMBSTONE);
      for (uint32_t s = 0; s < d.S && m < d.L; s++)
        if ((own >> s) & 1ull)
          for (int k = 0; k < 2 && m < d.L; k++) {  // each own tombstone twice (:707-710)
            dst[m].w = w;
            dst[m].r = o * d.S + s;
            dst[m].pad = 0;
            m++;
          }
      for (uint32_t i = 0; i < n_others && m < d.L; i++) dst[m++] = others[i];  // own ++ others (:618)
      commit_send(d, a, o, slot, m, d.p.tombstone_count);
    }
    h->bt_next = d.round + d.p.tombstone_interval_rounds;
  } else {
    push_job(d, a, o, make_job(0, 0, meta_of(GX_JOB_NIL_BT, 0, 1)));  // Broadcasts <- nil (:628)
    h->flags |= 2u;
  }
}

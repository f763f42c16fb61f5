// gx_engine.hip — sidecar-gx gossip-convergence engine for MI355X (gfx950).
//
// Implements include/gx.h. One engine object owns one GPU's slice of the simulated cluster and
// advances it one gossip round at a time (gx_run_rounds). Round phases and the kernels that run
// them (DESIGN.md "Round model", "Kernels"):
//   0+1 k_owner      a team of S lanes per host: wake re-armed SendServices passes; discovery churn;
//                    BroadcastServices tick (services_state.go:525-574) + TrackNewServices; the
//                    BroadcastTombstones tick lists the views whose expiry scan can change anything
//   1   k_scan       TombstoneOthersServices full-view expiry scan (services_state.go:635-683) over
//                    that worklist: one 256-thread block streams one 4 MB view row, ordered compaction
//   1   k_bt_finish  TombstoneServices + SendServices(TOMBSTONE_COUNT) or nil (services_state.go:606-633);
//                    folded into k_send unless another phase queues jobs in between (storm, detector)
//   2   k_storm      NotifyLeave -> ExpireServer for every host of the other half (services_state.go:150-192)
//   3   k_send       peer sampling + GetBroadcasts/packPacket per peer (services_delegate.go:85-144,186-223);
//                    each packet is registered in its receiver's inbox with one atomic
//   4   k_merge      gather-then-merge: one wave per receiver sorts its inbox by sender key, takes its
//                    inbound records straight from the packets, folds duplicates of a key in arrival
//                    order with the AddServiceEntry rule (services_state.go:293-347), writes each
//                    touched slot once, and compacts accepted foreign records into the receiver's
//                    broadcast FIFO with a wave ballot
//   5   k_ae         anti-entropy push-pull: one 256-thread block per host pair streams both views
//                    and merges each into the other (services_delegate.go:153-167, Merge :367-373)
// No MFMA: the work is int64 compare/select over HBM-resident views (memory-bound).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <deque>
#include <string>
#include <vector>


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

#include "gx_kernels.hpp"
#include "gx_fd.hpp"
#include "gx_codec.hpp"

// ================================================================================ host ==
struct TimedLaunch {
  int cls;
  hipEvent_t a, b;
};

struct gx_engine {
  Dev d;
  hipStream_t stream;      // where all device work goes (own_stream, or the caller's: gx_set_stream)
  hipStream_t own_stream;
  // shard-local push-pull pairs run on side_stream, between side_start (recorded on `stream` after
  // the rows are packed) and side_done (joined back into `stream` before anything reads them)
  hipStream_t side_stream;
  hipEvent_t side_start, side_done;
  bool side_pending;
  // Where a round's expiry scans run (round_send_impl): in k_send's prologue (one launch with the
  // owner ticks and the sends; a block streams its own listed views, fine while almost no view
  // needs a scan) or, while views do get scanned, in k_owner + k_scan + k_send, where k_scan
  // streams the listed rows with the whole chip. Decided from the device's count of scanned views
  // (work_cnt[GX_WC_SCANS]) read back without stalling the device: a snapshot is copied to pinned
  // memory every second round and consumed two snapshots later (scan_probe_begin). Both placements give
  // the same results; only the time differs.
  bool scan_heavy;
  uint64_t *scan_snap;      // [2] pinned host copies of (round << 32 | work_cnt[GX_WC_SCANS]), written by k_send
  uint64_t *scan_snap_dev;  // the same memory as the device addresses it
  uint32_t scan_tag[2];     // the round each slot's snapshot was asked for
  uint32_t scan_k, scan_last;
  uint32_t *in_cnt_buf;     // [2][Hl] inbox counts by round parity (Dev::in_cnt, in_cnt_nx)
  int async_phases;         // sharded phase calls return without waiting (gx_set_stream)
  int device;
  int timing;
  std::vector<TimedLaunch> pending_ev;
  std::vector<uint32_t> pp_host;  // GX_PP_INITIATE: this round's exchanges, batch by batch (a then b)
  uint32_t *pp_dev;
  int32_t *pp_prow;               // all -1: every exchange is local
  uint32_t *name_rank;            // [R] ByService: rank of each record's Service.Name (gx_set_service_names)
  double ms[GX_K_COUNT];
  uint64_t launches[GX_K_COUNT];
  uint64_t host_bytes[GX_K_COUNT], host_units[GX_K_COUNT];  // codec classes (gx_codec_host.hpp)
  struct CodecState *codec;
  // sharded rounds: outbox entry list and push-pull plan (device), rebuilt per round
  uint32_t *ob_entries;
  uint32_t *ob_counts;  // [G] packets per destination shard, then [chunks][G] counts and offsets
  uint32_t n_ob;
  bool ob_async;        // the outbox slot count is on the device only (gx_outbox_sizes_async)
  uint32_t *ob_total;   // [1] that count
  uint32_t *ae_pa, *ae_pb, *ae_pack_host, *ae_pack_t, *ae_pack_other;
  uint8_t *ae_pack_first, *ae_skip;  // this side is the pair's initiator; the pair does not run
  uint64_t *fd_rsnap;                // [pairs][H] partner member lists received with the digests
  int32_t *ae_prow;
  uint8_t *ae_pcount;
  uint32_t n_plan, n_pack, n_plan_rows;
  // push-pull digests / delta (per cross pair k, in pack order = receive order)
  uint32_t nblk, nmw;
  ulonglong2 *ae_dig;  // [Hl][nblk] own digests
  uint32_t *ae_mask;   // [Hl][nmw] differing blocks this side leads
  uint32_t *ae_fmask;  // [Hl][nmw] differing blocks the partner leads
  uint16_t *ae_lt;     // [Hl][nblk] the partner's literal counts (its digests)
  uint16_t *ae_retL;   // [Hl][nblk] literal counts of this side's return blocks (follow order)
  uint32_t *ae_bcnt;   // [Hl][nblk] own blocks: present | stale << 16 (digest pass)
  uint32_t *ae_cnt;    // [Hl] blocks this side leads
  uint32_t *ae_nfol;   // [Hl] blocks the partner leads
  uint64_t *ae_sz;     // [4][Hl] lead message size, partner's lead size, return size, scratch
  uint64_t *ae_off;    // [4][Hl] lead offsets, lead inbox offsets, return offsets, return table entries
  uint64_t *ae_rioff;  // [Hl] return inbox offsets
  uint32_t *ae_err;
  std::vector<uint32_t> pack_gstart;  // pack index range per destination shard
  std::vector<uint64_t> delta_off_h;
  uint64_t delta_total, lead_in_total, ret_total;
  int ae_delta_round, ae_ret_round;
  int ae_planned_round;
  int64_t ae_local_round;
  // listeners: host-side channels fed from the per-view device event logs
  struct Listener {
    uint32_t view, id, cap;
    std::deque<gx_change_event> ring;
  };
  std::vector<Listener> listeners;
  std::vector<uint32_t> log_views;  // view of each device event log
  uint64_t listener_drops;
  // small device scratch for single-host ABI calls
  void *api_dev;
  size_t api_dev_bytes;
  unsigned long long *conv_bad;
  uint64_t *digest_buf;
  size_t kprof_n;  // diagnostics: u64 marks in d.kprof (env GX_KPROF)
  // planned gossip exchange (gx_exchange_plan): slot bounds of XPLAN_BATCH rounds computed ahead on
  // xplan_stream into pinned host memory, two batches (the current one and the next)
  hipStream_t xplan_stream;
  uint32_t *xplan_dev;           // [2][XPLAN_BATCH][G][G] (k_send of a packing round reads its row)
  uint32_t *xplan_host;          // [2][XPLAN_BATCH][G][G] pinned
  int64_t xplan_start[2];
  uint64_t xplan_waits[2];       // diagnostics: calls whose batch was not ready yet (a host wait) / all calls
  hipEvent_t xplan_ev[2];
  hipEvent_t xplan_join;         // a batch is rewritten after the rounds queued before it (xplan_launch)
  int64_t xbound_round;          // the round xbound holds
  XBound xbound;                 // this shard's slots per destination this round
  const uint32_t *xbound_dev;    // the same row on the device
  uint32_t *ob_claim;            // Dev::ob_claim (gx_round_gossip_begin packing in k_send)
  // the worklist expiry scan's row split (k_scan_split / k_scan_join): chunks per row, chunk length,
  // each chunk's first L expirations and its result
  uint32_t scan_nch;
  grec *scan_tmp;
  ScanChunk *scan_chunk;
};

static void codec_free(gx_engine *e);  // gx_codec_host.hpp

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

static bool own(const gx_engine *e, uint32_t v) { return v >= e->d.lo && v < e->d.lo + e->d.Hl; }
// push-pull also merges memberlist state (mergeState)
static bool pp_state(const Dev &d) { return d.p.fd_enable && d.p.fd_push_pull_state; }
static int64_t now_of(const gx_engine *e) { return e->d.p.t0_ns + e->d.round * e->d.p.round_ns; }
// slot time -> absolute for server times and state.LastChanged: 0 = never set (time.Unix(0, 0),
// services_state.go:62-63,95)
static int64_t abs_tm(const gx_engine *e, int64_t t) { return t ? t + e->d.epoch : 0; }
static void set_round_fields(gx_engine *e) {
  Dev &d = e->d;
  const uint32_t par = (uint32_t)(d.round & 1);
  d.in_cnt = e->in_cnt_buf + (size_t)par * d.Hl;
  d.in_cnt_nx = e->in_cnt_buf + (size_t)(par ^ 1u) * d.Hl;
  d.wl_cnt = d.work_cnt + par;
  d.wl_cnt_nx = d.work_cnt + (par ^ 1u);
  d.ovf_cnt = d.work_cnt + 2 + par;
  d.ovf_cnt_nx = d.work_cnt + 2 + (par ^ 1u);
  e->d.now = now_of(e);
  e->d.partitioned = e->d.round >= e->d.p.partition_start && e->d.round < e->d.p.partition_end;
  e->d.pair_split = e->d.partitioned && !e->d.p.fd_enable;
}

struct LaunchTimer {
  gx_engine *e;
  int cls;
  hipEvent_t a, b;
  hipStream_t st;
  LaunchTimer(gx_engine *e_, int cls_, hipStream_t s_ = nullptr) : e(e_), cls(cls_), a(nullptr), b(nullptr), st(s_ ? s_ : e_->stream) {
    e->launches[cls]++;
    if (e->timing) {
      (void)hipEventCreate(&a);
      (void)hipEventCreate(&b);
      (void)hipEventRecord(a, st);
    }
  }
  ~LaunchTimer() {
    if (e->timing) {
      (void)hipEventRecord(b, st);
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

// Deliver the device event logs into the listeners' channels (non-blocking sends: a full
// channel drops the event, services_state.go:230-236) and reset the logs. Channels are drained
// only between ABI calls, so each listener receives a prefix of its view's events.
static int deliver_events(gx_engine *e) {
  size_t nlog = e->log_views.size();
  if (!nlog) return GX_OK;
  std::vector<uint32_t> cnt(nlog);
  HIPCHK(hipMemcpy(cnt.data(), e->d.ev_cnt, sizeof(uint32_t) * nlog, hipMemcpyDeviceToHost));
  bool any = false;
  for (uint32_t c : cnt) any |= c != 0;
  if (!any) return GX_OK;
  for (size_t k = 0; k < nlog; k++) {
    if (!cnt[k]) continue;
    uint32_t n = cnt[k] < e->d.ev_cap ? cnt[k] : e->d.ev_cap;
    std::vector<gx_change_event> ev(n);
    HIPCHK(hipMemcpy(ev.data(), &e->d.ev_log[k * e->d.ev_cap], sizeof(gx_change_event) * n, hipMemcpyDeviceToHost));
    for (auto &x : ev) {
      x.service.updated_ns += e->d.epoch;
      x.time_ns = abs_tm(e, x.time_ns);
    }
    for (auto &l : e->listeners) {
      if (l.view != e->log_views[k]) continue;
      uint32_t room = l.cap - (uint32_t)l.ring.size();
      uint32_t take = cnt[k] < room ? cnt[k] : room;  // take <= n: ev_cap >= every capacity
      for (uint32_t i = 0; i < take; i++) l.ring.push_back(ev[i]);
      e->listener_drops += cnt[k] - take;
    }
  }
  HIPCHK(hipMemset(e->d.ev_cnt, 0, sizeof(uint32_t) * nlog));
  return GX_OK;
}

// A received packet slot that failed validation (k_inbox_unpack: the oracle's gx_inbox_unpack
// checks) was skipped on the device; the next call that waits reports it, once.
static int take_device_error(gx_engine *e) {
  if (e->d.G < 2) return GX_OK;
  uint32_t err = 0;
  HIPCHK(hipMemcpy(&err, &e->d.work_cnt[GX_WC_ERR], sizeof(err), hipMemcpyDeviceToHost));
  if (!err) return GX_OK;
  HIPCHK(hipMemset(&e->d.work_cnt[GX_WC_ERR], 0, sizeof(err)));
  return GX_EINVAL;
}

// The shard-local push-pull merges rejoin the engine's stream (gx_ae_merge_local).
static int join_side(gx_engine *e) {
  if (!e->side_pending) return GX_OK;
  HIPCHK(hipStreamWaitEvent(e->stream, e->side_done, 0));
  e->side_pending = false;
  return GX_OK;
}

// The push-pull exchange stages read sizes back without waiting for the shard-local merges on
// side_stream (they touch rows no exchange stage reads); gx_ae_merge / gx_round_end join them.
static int sync_main(gx_engine *e) {
  HIPCHK(hipStreamSynchronize(e->stream));
  HIPCHK(hipGetLastError());
  return take_device_error(e);
}

static int sync_check(gx_engine *e) {
  int jr = join_side(e);
  if (jr) return jr;
  HIPCHK(hipStreamSynchronize(e->stream));
  HIPCHK(hipGetLastError());
  int rc = take_device_error(e);
  if (rc) return rc;
  return e->log_views.empty() ? GX_OK : deliver_events(e);
}

// End of a sharded phase call: with async phases (and no listeners to feed) the caller's stream
// orders the next step, so only launch errors are checked here.
static int phase_done(gx_engine *e) {
  if (e->async_phases && e->log_views.empty()) {
    HIPCHK(hipGetLastError());
    return GX_OK;
  }
  return sync_check(e);
}

static inline unsigned nblk(size_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

// Phases 0-3 (wake, owners, expiry scan, storm, GetBroadcasts) for this engine's hosts.
// k_owner with a team of T >= S lanes per host (lane s = service s)
template <int T>
static void launch_owner(const Dev &d, hipStream_t s) {
  k_owner<T><<<nblk(d.Hl, 256 / T), 256, 0, s>>>(d);  // 64- and 128-thread blocks measured 13.6 / 12.6 vs 12.5 us
}
// teams of the smallest power of two >= S (16 -> 32 -> 64 lanes measured 12.3 / 17.4 / 29.2 us at cfg 5)
static void owner_launch(const Dev &d, hipStream_t s) {
  if (d.S <= 1) launch_owner<1>(d, s);
  else if (d.S <= 2) launch_owner<2>(d, s);
  else if (d.S <= 4) launch_owner<4>(d, s);
  else if (d.S <= 8) launch_owner<8>(d, s);
  else if (d.S <= 16) launch_owner<16>(d, s);
  else if (d.S <= 32) launch_owner<32>(d, s);
  else launch_owner<64>(d, s);
}
#define SCAN_GRID 2048  // worklist blocks: every listed row of a round streams at once, a quick exit when none do

// Every second round: takes the scanned-view count of the snapshot two probes back, if the device
// has written it by now (the slot carries the round it was asked for; nothing waits for it: with the
// device further behind, the last decision stands), and has this round's k_send store a new one
// (Dev::snap, one 8-B store to pinned host memory, no event in the stream). A view scanned between
// the two consumed snapshots selects the k_scan placement.
static int scan_probe_begin(gx_engine *e) {
  e->d.snap = nullptr;
  if (e->d.round % 2) return GX_OK;
  const uint32_t i = e->scan_k & 1u;
  if (e->scan_k >= 2) {
    const uint64_t v = __atomic_load_n(&e->scan_snap[i], __ATOMIC_ACQUIRE);
    if ((uint32_t)(v >> 32) == e->scan_tag[i]) {
      e->scan_heavy = (uint32_t)v != e->scan_last;
      e->scan_last = (uint32_t)v;
    }
  }
  e->scan_tag[i] = (uint32_t)e->d.round;
  e->d.snap = &e->scan_snap_dev[i];
  return GX_OK;
}
static int scan_probe_end(gx_engine *e) {
  if (!e->d.snap) return GX_OK;
  e->scan_k++;
  e->d.snap = nullptr;
  return GX_OK;
}

// Phases 0-3 (wake, owners, expiry scan, storm, GetBroadcasts) for this engine's hosts.
static int round_send_impl(gx_engine *e) {
  Dev &d = e->d;
  set_round_fields(e);
  d.in_round = 1;  // ExpireServer waits for a held lock (gx.h lock_model); reset after the launches
  struct InRound {
    Dev &d;
    ~InRound() { d.in_round = 0; }
  } in_round_guard{d};
  {
    int rc = scan_probe_begin(e);
    if (rc) return rc;
  }
  d.n_remote = 0;
  hipStream_t s = e->stream;
  if (d.p.probe_piggyback) {  // the probe ping and ack calls come before the owner phase (gx.h)
    LaunchTimer t(e, GX_K_SEND);
    // phase 0 first: inside a gx_run_rounds call the due sleepers re-enter the FIFOs in the owner
    // tick (the oracle's ph_wake opens the round), which runs after these calls
    k_wake<<<nblk(d.Hl, 64), 64, 0, s>>>(d);
    k_probe<4><<<nblk(d.Hl, 64), 256, 0, s>>>(d);
  }
  bool vec = (d.R % 2) == 0;
  const bool storm = d.p.storm_round >= 0 && d.round == d.p.storm_round && d.H >= 2;
  // BroadcastTombstones' SendServices is queued before the detector's and the storm's jobs
  const bool bt_apart = d.p.fd_enable || storm;
  // a round without the detector or the storm: owner ticks, expiry scans and sends in one launch
  // (S <= 16: owner teams of the send's 4 lanes with up to 4 services each)
  const bool fused = !bt_apart && d.K && d.S <= 16 && !e->scan_heavy;
  // planned GetBroadcasts (send_planned): record budget, no detector or departures, re-armed
  // passes sleep; teams of 4 lanes per host
  const bool plan = !d.p.limit_bytes && d.p.retransmit_rounds > 0 && !d.departures && !d.p.fd_enable;
  if (fused && plan) {
    LaunchTimer t(e, GX_K_SEND);
    const unsigned g = nblk(d.Hl, 64);
    const bool ev = !e->log_views.empty();
#define GX_TSP(SPL)                                                                                               \
  (vec ? (ev ? k_send<4, false, true, true, true, SPL, true> : k_send<4, false, true, true, false, SPL, true>)    \
       : (ev ? k_send<4, false, true, false, true, SPL, true> : k_send<4, false, true, false, false, SPL, true>)) \
      <<<g, 256, 0, s>>>(d, 1)
    if (d.S <= 4) GX_TSP(1);
    else if (d.S <= 8) GX_TSP(2);
    else GX_TSP(4);
#undef GX_TSP
    HIPCHK(hipGetLastError());
    return scan_probe_end(e);
  }
  if (fused) {
    LaunchTimer t(e, GX_K_SEND);
    const unsigned g = nblk(d.Hl, 64);
    const bool ev = !e->log_views.empty();
#define GX_TS(X, SPL)                                                                                    \
  (vec ? (ev ? k_send<4, X, true, true, true, SPL> : k_send<4, X, true, true, false, SPL>)             \
       : (ev ? k_send<4, X, true, false, true, SPL> : k_send<4, X, true, false, false, SPL>))<<<g, 256, 0, s>>>(d, 1)
#define GX_TICK_SEND(SPL) \
  if (d.departures) GX_TS(true, SPL); else GX_TS(false, SPL)
    if (d.S <= 4) {
      GX_TICK_SEND(1);
    } else if (d.S <= 8) {
      GX_TICK_SEND(2);
    } else {
      GX_TICK_SEND(4);
    }
#undef GX_TICK_SEND
#undef GX_TS
    HIPCHK(hipGetLastError());
    return scan_probe_end(e);
  }
  {
    LaunchTimer t(e, GX_K_OWNER);
    owner_launch(d, s);
  }
  // with the tick finished in k_send, the expiry scans run in k_send's prologue (no k_scan launch)
  const bool scan_in_send = !bt_apart && d.K && !e->scan_heavy;
  if (!scan_in_send) {
    LaunchTimer t(e, GX_K_SCAN);
    const bool ev = !e->log_views.empty();
    const unsigned grid = d.Hl < SCAN_GRID ? d.Hl : SCAN_GRID;
    if (vec && !ev && e->scan_nch > 1) {  // rows split over blocks, then joined per view
      k_scan_split<true><<<SCAN_GRID, 256, GX_SCAN_WAVE ? 4 * sizeof(grec) * d.L : 0, s>>>(d, e->scan_tmp, e->scan_chunk,
                                                                                         e->scan_nch);
      k_scan_join<<<grid, 256, 0, s>>>(d, e->scan_tmp, e->scan_chunk, e->scan_nch);
    } else {
      (vec ? (ev ? k_scan<true, true> : k_scan<true, false>) : (ev ? k_scan<false, true> : k_scan<false, false>))
          <<<grid, 256, 0, s>>>(d, d.scan_list, d.L, d.L, d.scan_cnt, -1);
    }
    if (bt_apart) k_bt_finish<<<nblk(d.Hl, 256), 256, 0, s>>>(d);
  }
  if (d.p.fd_enable) {  // suspicion timers -> deadNode -> NotifyLeave; probe ticks
    LaunchTimer t(e, GX_K_FD);
    k_fd_tick<<<d.Hl, 64, 0, s>>>(d);
  }
  if (storm) {
    LaunchTimer t(e, GX_K_STORM);
    const bool ev = !e->log_views.empty();
    // nontemporal row stream: 30.3 -> 27.9 ms at cfg 5 (profiles/ab/storm_nt_ab_r02.log)
    if (d.S >= 2 && 64 % d.S == 0)
      (ev ? k_storm_p2<true, true> : k_storm_p2<false, true>)<<<d.Hl, 256, 0, s>>>(d);
    else (ev ? k_storm<true> : k_storm<false>)<<<d.Hl, 256, 0, s>>>(d);
  }
  {
    LaunchTimer t(e, GX_K_SEND);
    if (d.p.fd_enable) k_fd_send<<<nblk(d.Hl, 64), 64, 0, s>>>(d);  // memberlist's targets + messages
    // 4 lanes per host: measured best of 1/4/8/16/64 (profiles/send_team.sh)
    const bool ev = !e->log_views.empty();
    const unsigned g = nblk(d.Hl, 64);
    // teams of 2 / 8 lanes measured 25.6 / 28.7 vs 21.1 us (profiles/r02/gossip/send_team_ab.log)
    if (plan) {
      if (scan_in_send)
        (vec ? (ev ? k_send<4, false, true, true, true, 0, true> : k_send<4, false, true, true, false, 0, true>)
             : (ev ? k_send<4, false, true, false, true, 0, true> : k_send<4, false, true, false, false, 0, true>))
            <<<g, 256, 0, s>>>(d, 1);
      else
        k_send<4, false, false, false, false, 0, true><<<g, 256, 0, s>>>(d, bt_apart ? 0 : 1);
    } else if (scan_in_send) {
      if (d.departures)
        (vec ? (ev ? k_send<4, true, true, true, true> : k_send<4, true, true, true, false>)
             : (ev ? k_send<4, true, true, false, true> : k_send<4, true, true, false, false>))<<<g, 256, 0, s>>>(d, 1);
      else
        (vec ? (ev ? k_send<4, false, true, true, true> : k_send<4, false, true, true, false>)
             : (ev ? k_send<4, false, true, false, true> : k_send<4, false, true, false, false>))<<<g, 256, 0, s>>>(d, 1);
    } else if (d.p.fd_enable || d.departures) {
      k_send<4, true><<<g, 256, 0, s>>>(d, bt_apart ? 0 : 1);
    } else {
      k_send<4, false><<<g, 256, 0, s>>>(d, bt_apart ? 0 : 1);
    }
  }
  HIPCHK(hipGetLastError());
  return scan_probe_end(e);
}

#ifndef GX_LOCK_APPEND
#define GX_LOCK_APPEND 1
#endif
// with k_lock_append taking the locked receivers, the merge's 64-receiver blocks are faster again:
// cfg 5 lock on, filling 80.7 -> 77.9 us, full 32.8 -> 30.6 us (profiles/r06/ab/merge_nr64_lapp_cfg5.jsonl)
#ifndef GX_MERGE_LAPP_NR64
#define GX_MERGE_LAPP_NR64 1
#endif
#ifndef GX_LOCK_APPEND_HL
#define GX_LOCK_APPEND_HL 32768
#endif
#ifndef GX_MERGE_SMALL_HL
#define GX_MERGE_SMALL_HL 16384  // 16 receivers per block below this many local hosts: merge 2.0 -> 1.1 ms (cfg 2)
                                 // and 2.4 -> 1.5 ms (cfg 4) over 60 rounds lock off (profiles/r05/ab/merge_nr16_*)
#endif
// Phase 4: gather-then-merge of every receiver's inbox (local and received packets).
static int round_merge_impl(gx_engine *e) {
  Dev &d = e->d;
  set_round_fields(e);
  d.in_round = 1;
  struct InRound {
    Dev &d;
    ~InRound() { d.in_round = 0; }
  } in_round_guard{d};
  hipStream_t s = e->stream;
  if (d.p.lock_readers) {  // waiting push-pull merges of hosts unlocked now, before their pipelines
    LaunchTimer t(e, GX_K_AE);
    const bool vec = (d.R % 2) == 0, ev = !e->log_views.empty();
    (vec ? (ev ? k_defer_drain<true, true> : k_defer_drain<true, false>)
         : (ev ? k_defer_drain<false, true> : k_defer_drain<false, false>))<<<d.P, 256, 0, s>>>(d);
  }
  if (d.K) {
    LaunchTimer t(e, GX_K_MERGE);
    const bool ev = !e->log_views.empty();
    // receivers routed by their live records. GossipMessages > 1: inboxes of hundreds of live
    // records, each folded by a whole wave tile by tile, so more waves in flight (16 receivers per
    // block, 4 waves per SIMD: 10% faster than 3 in the GM 15 accepting stretch,
    // profiles/r03/ab/merge_wpe_gm15.jsonl); else 64 receivers per block (3% faster at cfg 5)
    // ... and when 64 receivers per block leave most CUs idle (a shard, a small cluster): a block's
    // waves fold their receivers one item after another, so fewer per block shortens the launch
    // ... and with the lock modelled (round 6): a locked receiver's pipeline append is a short
    // dependent chain, and 64 receivers per block run a wave's four of them one after another; 16 per
    // block spread them over more waves (cfg 5, locked gossip rounds 93.7 -> 87.7 us; lock off the
    // 64-receiver blocks stay 3-5% faster, profiles/r06/ab/merge_nr16_cfg5.jsonl)
    // locked receivers' pipeline appends first, at high occupancy (k_lock_append), where k_merge_seg's
    // item waves would take several passes over the receivers: cfg 5 (32768 receivers) lock-on gossip
    // rounds 88.1 -> 79.8 us, a round whose pipelines are all full 30.0 -> 32.3 us (the launch with
    // nothing to append); at 16384 receivers (cfg 3) the extra launch cost 7.7 us per round, and
    // with GossipMessages 15 most locked inboxes exceed a segment (+4%), so neither takes it
    // (profiles/r06/ab/lock_append_*.jsonl)
    const bool lapp = GX_LOCK_APPEND && d.p.lock_model && !d.p.fd_handoff_shared && d.NG == 1 && d.Hl >= GX_LOCK_APPEND_HL;
    if (lapp) k_lock_append<<<nblk(d.Hl, 16), 256, 0, s>>>(d);
    const bool small = d.NG > 1 || d.Hl < GX_MERGE_SMALL_HL || (d.p.lock_model && !(GX_MERGE_LAPP_NR64 && lapp));
    const unsigned g = nblk(d.Hl, small ? 16u : (unsigned)MERGE_NR);
    if (small) {
      if (d.R < (1u << 26)) (ev ? k_merge_seg<true, true, 16, MERGE_WPE_GM> : k_merge_seg<true, false, 16, MERGE_WPE_GM>)<<<g, 64 * MERGE_WAVES, 0, s>>>(d);
      else (ev ? k_merge_seg<false, true, 16, MERGE_WPE_GM> : k_merge_seg<false, false, 16, MERGE_WPE_GM>)<<<g, 64 * MERGE_WAVES, 0, s>>>(d);
    } else if (d.R < (1u << 26)) {
      (ev ? k_merge_seg<true, true> : k_merge_seg<true, false>)<<<g, 64 * MERGE_WAVES, 0, s>>>(d);
    } else {
      (ev ? k_merge_seg<false, true> : k_merge_seg<false, false>)<<<g, 64 * MERGE_WAVES, 0, s>>>(d);
    }
  }
  if (d.p.fd_enable && d.K) {  // the packets' memberlist messages, after the catalog merge
    LaunchTimer t(e, GX_K_FD);
    k_fd_recv<<<nblk(d.Hl, 64), 64, 0, s>>>(d);
  }
  HIPCHK(hipGetLastError());
  return GX_OK;
}

// lock off, cfg 2's window (two push-pull rounds): 0.94 ms as built; two tiles in flight 1.01, plain
// row loads and stores 0.98, two tiles at 3 waves per SIMD 1.08 (profiles/r06/ab/ae_cfg2_variants.jsonl)
#ifndef GX_AE_PF_OFF
#define GX_AE_PF_OFF 1  // lock off: tiles in flight per pair
#endif
#ifndef GX_AE_NT_OFF
#define GX_AE_NT_OFF true  // lock off: nontemporal row loads and stores
#endif
#ifndef GX_AE_PF_LOCK
#define GX_AE_PF_LOCK 1  // 2 tiles in flight spill (92 B scratch): 0.98 vs 0.71 ms at cfg 5 lock on (profiles/r05/ab/ae_pf_lock.jsonl)
#endif
static bool ae_round(const gx_engine *e) {
  const Dev &d = e->d;
  if (d.p.ae_period_rounds && d.p.push_pull_stagger) return true;  // some host's staggered timer, every round
  return d.p.ae_period_rounds && (uint64_t)d.round % d.p.ae_period_rounds == d.p.ae_phase;
}
// gx.h push_pull_stagger: host i's push-pull timer fires in the rounds of its seeded phase
static bool pp_initiates(const Dev &d, uint32_t i) {
  if (!d.p.push_pull_stagger) return true;
  return (uint64_t)d.round % d.p.ae_period_rounds == rng4(d.p.seed, ST_PP_PHASE, i, 0, 0) % d.p.ae_period_rounds;
}

// GX_PP_INITIATE (unsharded engines): every live host starts one exchange with a partner drawn
// at random on its side; the exchanges run in initiator order, in batches of exchanges with no
// host in common (an exchange goes into the batch after the last one holding either of its hosts).
// The oracle's pp_batches computes the same batches; each batch is one k_ae_plan launch over its
// pair list (local pairs: both sides merge the other's pre-exchange row).
static bool ae_partner(const Dev &d, uint32_t i, uint32_t *out) {
  uint32_t base = 0, m = d.H;
  if (d.partitioned && !d.p.fd_enable) {
    const uint32_t half = d.H / 2;
    base = i < half ? 0 : half;
    m = i < half ? half : d.H - half;
  }
  if (m < 2) return false;
  const uint64_t x = rng4(d.p.seed, ST_AE, (uint64_t)d.round, i, 1);
  const uint32_t idx = unif(x, m - 1), self = i - base;
  *out = base + (idx >= self ? idx + 1 : idx);
  return true;
}
// gx.h lock_readers: the read-locked exchanges of the last push-pull launch (k_ae_ro)
static void ae_ro_launch(gx_engine *e, const uint32_t *pa, const uint32_t *pb, uint64_t key0, uint64_t key1, uint32_t np) {
  const Dev &d = e->d;
  const bool vec = (d.R % 2) == 0, ev = !e->log_views.empty();
  (vec ? (ev ? k_ae_ro<true, true> : k_ae_ro<true, false>) : (ev ? k_ae_ro<false, true> : k_ae_ro<false, false>))<<<1, 256, 0, e->stream>>>(
      d, pa, pb, key0, key1, np);
}
static int ae_initiate(gx_engine *e) {
  Dev &d = e->d;
  const bool dep = d.departures;
  std::vector<uint32_t> last(d.H, 0), bat, ia, ib;
  uint32_t nb = 0;
  for (uint32_t i = 0; i < d.H; i++) {
    uint32_t b;
    if (!pp_initiates(d, i) || (dep && departed_at(d.p, d.round, i)) || !ae_partner(d, i, &b) ||
        (dep && departed_at(d.p, d.round, b)))
      continue;
    const uint32_t k = 1 + std::max(last[i], last[b]);
    last[i] = last[b] = k;
    ia.push_back(i);
    ib.push_back(b);
    bat.push_back(k - 1);
    nb = std::max(nb, k);
  }
  const size_t n = ia.size();
  if (!n) return GX_OK;
  std::vector<uint32_t> off(nb + 1, 0);
  for (uint32_t x : bat) off[x + 1]++;
  for (uint32_t q = 0; q < nb; q++) off[q + 1] += off[q];
  std::vector<uint32_t> cur(off.begin(), off.end() - 1);
  e->pp_host.assign(2 * n, 0);
  for (size_t t = 0; t < n; t++) {  // stable: initiator order inside a batch
    const uint32_t at = cur[bat[t]]++;
    e->pp_host[at] = ia[t];
    e->pp_host[n + at] = ib[t];
  }
  HIPCHK(hipMemcpyAsync(e->pp_dev, e->pp_host.data(), sizeof(uint32_t) * 2 * n, hipMemcpyHostToDevice, e->stream));
  const bool vec = (d.R % 2) == 0, ev = !e->log_views.empty();
  AeIn none;
  memset(&none, 0, sizeof(none));
  LaunchTimer t(e, GX_K_AE);
  for (uint32_t q = 0; q < nb; q++) {
    const uint32_t *pa = e->pp_dev + off[q], *pb = e->pp_dev + n + off[q];
    const unsigned np = off[q + 1] - off[q];
    if (ev) (vec ? k_ae_plan_ev<true> : k_ae_plan_ev<false>)<<<np, 256, 0, e->stream>>>(d, pa, pb, e->pp_prow, nullptr, none, nullptr);
    else (vec ? k_ae_plan<true> : k_ae_plan<false>)<<<np, 256, 0, e->stream>>>(d, pa, pb, e->pp_prow, nullptr, none, nullptr);
    if (d.p.lock_readers) ae_ro_launch(e, pa, pb, 0, 0, np);  // the batch's read-locked exchanges
  }
  return GX_OK;
}

// Phase 5 on an unsharded engine: pairs derived on device.
static int ae_whole_impl(gx_engine *e) {
  Dev &d = e->d;
  set_round_fields(e);
  hipStream_t s = e->stream;
  bool vec = (d.R % 2) == 0;
  if (ae_round(e) && d.p.push_pull_mode == GX_PP_INITIATE) {
    int rc = ae_initiate(e);
    if (rc) return rc;
  } else if (ae_round(e)) {
    uint32_t np;
    uint64_t key0, key1 = 0;
    if (d.pair_split) {
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
      // PF = 1: deeper prefetch measured within noise (profiles/ae_variants.sh)
      // the ChangeEvent variant only while some view has a listener
      const bool ev = !e->log_views.empty();
      // nontemporal row loads and stores: -1% over the bench window (profiles/ab/ae_nt_ab_r02.log)
      // under the lock model chunks of pairs per block (ae_round_pairs): a round whose pairs a lock
      // skips costs one round trip per chunk, not a block per pair
      if (vec && !ev && d.p.lock_model)
        k_ae_chunk<true, GX_AE_PF_LOCK, true, true><<<ae_grid(np, 1), 256, 0, s>>>(d, key0, key1, np);
      else if (vec && !ev) k_ae<true, GX_AE_PF_OFF, GX_AE_NT_OFF, GX_AE_NT_OFF><<<np, 256, 0, s>>>(d, key0, key1);
      else if (vec) k_ae_ev<true><<<np, 256, 0, s>>>(d, key0, key1);
      else if (!ev) k_ae<false><<<np, 256, 0, s>>>(d, key0, key1);
      else k_ae_ev<false><<<np, 256, 0, s>>>(d, key0, key1);
    }
    if (np && pp_state(d)) {  // pushPull's membership half (mergeState), from round-start lists
      LaunchTimer t(e, GX_K_FD);
      k_fd_pushpull_pair<<<np, 128, 0, s>>>(d, key0, key1);  // both directions in lockstep: no snapshot
    }
    if (np && d.p.lock_readers) {  // the read-locked exchanges (after the membership half reads ro_flag)
      LaunchTimer t(e, GX_K_AE);
      ae_ro_launch(e, nullptr, nullptr, key0, key1, np);
    }
  }
  HIPCHK(hipGetLastError());
  return GX_OK;
}

static int run_one_round(gx_engine *e) {
  int rc = round_send_impl(e);
  if (!rc) rc = round_merge_impl(e);
  if (!rc) rc = ae_whole_impl(e);
  if (!rc) e->d.round++;
  return rc;
}

static int wake_all(gx_engine *e) {
  set_round_fields(e);
  k_wake<<<nblk(e->d.Hl, 64), 64, 0, e->stream>>>(e->d);
  HIPCHK(hipGetLastError());
  return GX_OK;
}

// ------------------------------------------------------------------------------ ABI ------
extern "C" {

int gx_abi_version(void) { return GX_ABI_VERSION; }

int gx_set_stream(gx_engine *e, void *stream, int mode) {
  if (!e || (mode & ~(GX_STREAM_CALLER | GX_STREAM_ASYNC))) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  if (e->side_pending) HIPCHK(hipStreamSynchronize(e->side_stream));
  e->side_pending = false;
  HIPCHK(hipStreamSynchronize(e->stream));  // work queued so far completes first
  e->stream = (mode & GX_STREAM_CALLER) ? (hipStream_t)stream : e->own_stream;
  e->async_phases = (mode & GX_STREAM_ASYNC) ? 1 : 0;
  return GX_OK;
}
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
  p->overhead_bytes = 3;
  p->fd_probe_rounds = 5;
  p->fd_indirect_checks = 3;
  p->fd_msg_cap = 16;
  p->fd_msg_bytes = 64;
  p->fd_gossip_dead_rounds = 150;
  p->depart_round = -1;
  p->fd_push_pull_state = 1;
  p->lock_model = 1;
  p->lock_buffer = 1024 + 1 + 25 + 1 + 25 + 1;  // gx.h lock_model: handoff queue .. AddServiceEntry
  gx_fd_defaults(p);
}

// memberlist's size-derived parameters: util.go retransmitLimit / suspicionTimeout,
// suspicion.go remainingSuspicionTime (include/gx.h).
int gx_fd_defaults(gx_params *p) {
  if (!p || p->n_hosts < 1 || p->fd_probe_rounds < 1 || p->round_ns <= 0) return GX_EINVAL;
  const int suspicion_mult = 4, max_mult = 6, retransmit_mult = 4;
  const double n = (double)p->n_hosts;
  uint32_t limit = (uint32_t)(retransmit_mult * (int)ceil(log10(n + 1.0)));
  p->fd_retransmit_limit = limit > GX_FD_MAX_TX ? GX_FD_MAX_TX : limit;
  const double node_scale = fmax(1.0, log10(fmax(1.0, n)));
  const int64_t interval = (int64_t)p->fd_probe_rounds * p->round_ns;
  const int64_t tmin = (int64_t)suspicion_mult * (int64_t)(node_scale * 1000.0) * interval / 1000;
  const int64_t tmax = (int64_t)max_mult * tmin;
  int k = suspicion_mult - 2;
  if ((int)p->n_hosts - 2 < k) k = 0;
  p->fd_suspicion_k = (uint32_t)k;
  for (int c = 0; c < 8; c++) {
    int64_t t = tmin;
    if (c == 0) {
      t = k < 1 ? tmin : tmax;
    } else if (c <= k) {
      const double frac = log((double)c + 1.0) / log((double)k + 1.0);
      const double raw = (double)tmax / 1e9 - frac * ((double)tmax / 1e9 - (double)tmin / 1e9);
      t = (int64_t)floor(1000.0 * raw) * 1000000ll;
      if (t < tmin) t = tmin;
    }
    p->fd_suspicion_rounds[c] = (uint32_t)((t + p->round_ns - 1) / p->round_ns);
  }
  return GX_OK;
}

static int check_params(const gx_params *p) {
  if (!p || p->n_hosts < 1 || p->n_services < 1 || p->n_services > 64) return GX_EINVAL;
  if (p->fanout > 16 || p->packet_cap < 1 || p->packet_cap > 256 || p->pending_cap > 256) return GX_EINVAL;
  if (p->queue_cap < 1 || p->list_slots < 1 || p->list_slots > GX_MAX_LIST_SLOTS) return GX_EINVAL;
  if (p->n_hosts > GX_MAX_HOSTS) return GX_EINVAL;  // gx_job owner field
  if (p->alive_interval_rounds < 1 || p->tombstone_interval_rounds < 1) return GX_EINVAL;
  if (p->retransmit_rounds > 1000) return GX_EINVAL;
  if (p->alive_count < 1 || p->alive_count > GX_JOB_MAX_PASSES || p->tombstone_count < 1 ||
      p->tombstone_count > GX_JOB_MAX_PASSES)
    return GX_EINVAL;
  if (p->init_mode > GX_INIT_WARM) return GX_EINVAL;
  if (p->t0_ns < 0 || p->t0_ns > ((int64_t)1 << 62) || p->round_ns <= 0) return GX_EINVAL;
  {  // lifespans stay far inside the half window before t0 (gx.h GX_TS_SHIFT)
    const int64_t lim = (int64_t)1 << 58;
    for (int64_t x : {p->alive_lifespan_ns, p->draining_lifespan_ns, p->tombstone_lifespan_ns, p->stale_fudge_ns,
                      p->aged_max_ns})
      if (x < 0 || x > lim) return GX_EINVAL;
  }
  if ((uint64_t)p->n_hosts * p->n_services > 0xffffffffull) return GX_EINVAL;
  if (p->ae_period_rounds && p->ae_phase >= p->ae_period_rounds) return GX_EINVAL;
  if (p->limit_bytes > (1u << 24) || p->overhead_bytes > (1u << 16)) return GX_EINVAL;
  if (p->n_shards > 1 && (p->shard_id >= p->n_shards || p->n_shards > p->n_hosts || p->n_shards > 64)) return GX_EINVAL;
  if (p->depart_ppm > 1000000u) return GX_EINVAL;
  if (p->gossip_messages > 16) return GX_EINVAL;
  if (p->push_pull_mode > GX_PP_INITIATE || (p->push_pull_mode == GX_PP_INITIATE && (p->n_shards > 1 || p->fd_enable)))
    return GX_EINVAL;
  if (p->inbox_slots > GX_DI_MAX) return GX_EINVAL;
  if (p->lock_model > 1 || p->lock_buffer < 1 || p->lock_buffer > 65535) return GX_EINVAL;
  if (p->lock_model && (((uint64_t)p->n_hosts + (p->n_shards > 1 ? p->n_shards : 1) - 1) / (p->n_shards > 1 ? p->n_shards : 1)) *
                               p->lock_buffer * 16ull > GX_LOCK_BUF_MAX_BYTES)
    return GX_EINVAL; // the pipelines' records (gx.h lock_buffer)
  if (p->probe_piggyback > 1 || (p->probe_piggyback && (p->fd_enable || p->n_shards > 1 || p->fd_probe_rounds < 1)))
    return GX_EINVAL;
  if (p->push_pull_stagger > 1 || (p->push_pull_stagger && (p->push_pull_mode != GX_PP_INITIATE || !p->ae_period_rounds)))
    return GX_EINVAL;
  if (p->lock_readers > 1 || (p->lock_readers && (!p->lock_model || p->n_shards > 1)) || p->lock_defer_slots > 4096)
    return GX_EINVAL;  // gx.h lock_readers: unsharded engines with the lock modelled
  if (p->fd_handoff_shared > 1 || (p->fd_handoff_shared && (!p->fd_enable || !p->lock_model || p->n_shards > 1)))
    return GX_EINVAL;  // gx.h fd_handoff_shared
  if (p->fd_enable) {
    if (p->n_hosts > 65534 || p->fanout > 16) return GX_EINVAL;
    if (p->fd_probe_rounds < 1 || p->fd_indirect_checks > 16 || p->fd_msg_cap < 1 || p->fd_msg_cap > 64) return GX_EINVAL;
    if (p->fd_retransmit_limit < 1 || p->fd_retransmit_limit > GX_FD_MAX_TX || p->fd_suspicion_k > 2) return GX_EINVAL;
    for (uint32_t c = 0; c <= p->fd_suspicion_k; c++)
      if (p->fd_suspicion_rounds[c] > (1u << 30)) return GX_EINVAL;
  }
  return GX_OK;
}

int gx_destroy(gx_engine *e) {
  if (!e) return GX_EINVAL;
  (void)hipSetDevice(e->device);
  // every stream that may still run a kernel over the engine's buffers, before any is freed (the
  // planned exchange's look-ahead k_xplan batch on xplan_stream included: it was synchronized only
  // after the frees before round 6)
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  if (e->side_stream) (void)hipStreamSynchronize(e->side_stream);
  if (e->xplan_stream) (void)hipStreamSynchronize(e->xplan_stream);
  for (auto &t : e->pending_ev) {
    (void)hipEventDestroy(t.a);
    (void)hipEventDestroy(t.b);
  }
  Dev &d = e->d;
  void *ptrs[] = {e->ae_dig, e->ae_mask, e->ae_fmask, e->ae_lt, e->ae_retL, e->ae_bcnt, e->ae_cnt, e->ae_nfol, e->ae_sz, e->ae_off, e->ae_rioff, e->ae_err, d.msg_key, d.in_stamp, e->ob_entries, e->ob_counts, e->ob_total, e->ob_claim, e->ae_pa, e->ae_pb, e->ae_pack_host, e->ae_pack_t, e->ae_pack_other, e->ae_pack_first, e->ae_skip, e->fd_rsnap, e->ae_prow,
                  e->ae_pcount, d.view, d.minexp, d.own_status, d.hs, d.fifo, d.sleep, d.dq, d.arena, d.arena_len, d.msg, d.msg_w0, d.msg_len,
                  d.msg_dst, e->in_cnt_buf, d.scan_list, d.scan_cnt, d.tick,
                  d.sbytes, d.srvt, d.vlc, d.ev_slot, d.ev_log, d.ev_cnt, d.ctr, d.in_hdr, d.in_ovf, d.in_rec, d.work_cnt, d.work, d.mrec, e->pp_dev, e->pp_prow, e->name_rank, e->api_dev, e->conv_bad, e->digest_buf, d.kprof,
                  d.mem, d.fd_dl, d.fdh, d.fdm, d.fd_len, d.fd_peers, d.fd_np, d.fd_snap, d.lkb, d.pexp, d.dpool, d.dpool_host, d.dpool_res, d.dclaim, d.ro_flag, d.ro_list, d.fdq};
  for (void *p : ptrs)
    if (p) (void)hipFree(p);
  codec_free(e);
  if (e->own_stream) (void)hipStreamDestroy(e->own_stream);
  if (e->side_stream) (void)hipStreamDestroy(e->side_stream);
  if (e->side_start) (void)hipEventDestroy(e->side_start);
  if (e->side_done) (void)hipEventDestroy(e->side_done);
  if (e->scan_snap) (void)hipHostFree(e->scan_snap);
  if (e->xplan_dev) (void)hipFree(e->xplan_dev);
  if (e->scan_tmp) (void)hipFree(e->scan_tmp);
  if (e->scan_chunk) (void)hipFree(e->scan_chunk);
  if (e->xplan_host) (void)hipHostFree(e->xplan_host);
  for (int i = 0; i < 2; i++)
    if (e->xplan_ev[i]) (void)hipEventDestroy(e->xplan_ev[i]);
  if (e->xplan_join) (void)hipEventDestroy(e->xplan_join);
  if (e->xplan_stream) (void)hipStreamDestroy(e->xplan_stream);
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
  memset(e->host_bytes, 0, sizeof(e->host_bytes));
  memset(e->host_units, 0, sizeof(e->host_units));
  e->codec = nullptr;
  e->api_dev = nullptr;
  e->api_dev_bytes = 0;
  e->conv_bad = nullptr;
  e->digest_buf = nullptr;
  e->stream = e->own_stream = e->side_stream = nullptr;
  e->in_cnt_buf = nullptr;
  e->side_start = e->side_done = nullptr;
  e->side_pending = false;
  e->scan_heavy = true;  // k_scan placement until the first snapshots say no view gets scanned
  e->scan_snap = e->scan_snap_dev = nullptr;
  e->scan_tag[0] = e->scan_tag[1] = 0xffffffffu;
  e->scan_k = e->scan_last = 0;
  e->async_phases = 0;
  e->ob_entries = nullptr;
  e->ob_counts = nullptr;
  e->n_ob = 0;
  e->ob_async = false;
  e->ob_total = nullptr;
  e->ob_claim = nullptr;
  e->ae_pa = e->ae_pb = e->ae_pack_host = e->ae_pack_t = e->ae_pack_other = nullptr;
  e->ae_pack_first = e->ae_skip = nullptr;
  e->fd_rsnap = nullptr;
  e->ae_prow = nullptr;
  e->ae_pcount = nullptr;
  e->ae_dig = nullptr;
  e->ae_mask = e->ae_fmask = e->ae_cnt = e->ae_nfol = e->ae_err = nullptr;
  e->ae_lt = nullptr;
  e->ae_retL = nullptr;
  e->ae_bcnt = nullptr;
  e->ae_sz = e->ae_off = e->ae_rioff = nullptr;
  e->ae_delta_round = e->ae_ret_round = -1;
  e->delta_total = e->lead_in_total = e->ret_total = 0;
  e->n_plan = e->n_pack = e->n_plan_rows = 0;
  e->ae_planned_round = -1;
  e->ae_local_round = -1;
  e->pp_dev = nullptr;
  e->pp_prow = nullptr;
  e->name_rank = nullptr;
  Dev &d = e->d;
  d.p = *p;
  d.epoch = gx_epoch_of(p->t0_ns);
  d.p.t0_ns -= d.epoch;  // every device time is epoch-relative
  d.H = p->n_hosts;
  d.S = p->n_services;
  d.R = p->n_hosts * p->n_services;
  d.Q = p->queue_cap;
  d.A = p->list_slots;
  d.L = p->packet_cap + p->pending_cap;
  d.K = p->fanout;
  d.NG = p->gossip_messages > 1 ? p->gossip_messages : 1;
  d.KG = d.K * d.NG;
  d.KE = d.KG + (p->probe_piggyback ? 2u : 0u);  // the probe ping and ack entries (gx.h probe_piggyback)
  d.divS = d.S > 1 ? ~0ull / d.S + 1 : 0;
  d.logS = 0;
  while ((1u << d.logS) < d.S) d.logS++;  // used where S divides 64 (a power of two)
  d.G = p->n_shards > 1 ? p->n_shards : 1;
  d.gid = d.G > 1 ? p->shard_id : 0;
  d.lo = (uint32_t)(((uint64_t)d.gid * d.H) / d.G);
  d.Hl = (uint32_t)(((uint64_t)(d.gid + 1) * d.H) / d.G) - d.lo;
  d.n_remote = 0;
  d.SQ = pow2_at_least(64 > d.KE * (p->retransmit_rounds + 1) ? 64 : d.KE * (p->retransmit_rounds + 1));
  d.DQ = pow2_at_least(d.L + p->pending_cap + 64);
  d.round = 0;
  if (hipStreamCreateWithFlags(&e->own_stream, hipStreamNonBlocking) != hipSuccess) {
    delete e;
    return GX_EIO;
  }
  e->stream = e->own_stream;
  e->async_phases = 0;
  if (hipStreamCreateWithFlags(&e->side_stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&e->side_start, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&e->side_done, hipEventDisableTiming) != hipSuccess ||
      hipHostMalloc((void **)&e->scan_snap, 2 * sizeof(uint64_t), hipHostMallocMapped) != hipSuccess ||
      hipHostGetDevicePointer((void **)&e->scan_snap_dev, e->scan_snap, 0) != hipSuccess) {
    (void)hipGetLastError();
    gx_destroy(e);
    return GX_EIO;
  }
  e->scan_snap[0] = e->scan_snap[1] = ~0ull;
  // per-host arrays hold this shard's Hl hosts; the message table also takes the packets received
  // from other shards (at most (H - Hl) * K), so it is sized H * K.
  size_t Hg = d.H, H = d.Hl, K = d.KE ? d.KE : 1;
  ALLOC(d.view, sizeof(uint64_t) * H * d.R);
  ALLOC(d.own_status, H * d.S);
  ALLOC(d.hs, sizeof(gx_host_state) * H);
  ALLOC(d.fifo, sizeof(gx_job) * H * d.Q);
  ALLOC(d.sleep, sizeof(gx_sleeper) * H * d.SQ);
  ALLOC(d.dq, sizeof(grec) * H * d.DQ);
  ALLOC(d.arena, sizeof(grec) * H * d.A * d.L);
  ALLOC(d.arena_len, sizeof(uint32_t) * H * d.A);
  d.AW = (d.A + 31) / 32;
  ALLOC(d.arena_bits, sizeof(uint32_t) * H * d.AW);
  ALLOC(d.msg, sizeof(grec) * Hg * K * p->packet_cap);
  ALLOC(d.msg_w0, sizeof(uint64_t) * Hg * K * p->packet_cap);
  ALLOC(d.msg_len, sizeof(uint32_t) * Hg * K);
  ALLOC(d.msg_dst, sizeof(uint32_t) * Hg * K);
  ALLOC(d.msg_key, sizeof(uint32_t) * Hg * K);
  ALLOC(e->in_cnt_buf, sizeof(uint32_t) * 2 * H);
  d.nblk_ae = (d.R + GX_DIGEST_SLOTS - 1) / GX_DIGEST_SLOTS;
  // default: 64 slots; with GossipMessages > 1 (up to NG packets per sender) GX_DI_MAX, so the
  // wave merge takes the wide inboxes instead of the serial overflow path
  d.DI = p->inbox_slots ? p->inbox_slots : (d.NG > 1 ? GX_DI_MAX : 64);
  d.DR = d.DI < 8 ? d.DI : 8;  // inline packets: 99.6% of Poisson(fanout 3) in-degrees fit 8 slots
  // senders read their local receivers' view slots and drop no-op records; packets from other
  // shards are filtered the same way on arrival (k_inbox_unpack)
  d.sfilt = 1u;
  ALLOC(d.in_hdr, sizeof(uint4) * H * d.DI);
  ALLOC(d.in_ovf, sizeof(uint4) * Hg * K);
  ALLOC(d.in_rec, sizeof(grec) * H * d.DR * p->packet_cap);
  ALLOC(d.work_cnt, sizeof(uint32_t) * GX_WC_N);
  ALLOC(d.work, sizeof(uint32_t) * H);
  if (p->push_pull_mode == GX_PP_INITIATE) {
    ALLOC(e->pp_dev, sizeof(uint32_t) * 2 * Hg);
    ALLOC(e->pp_prow, sizeof(int32_t) * Hg);
    HIPCHK(hipMemset(e->pp_prow, 0xff, sizeof(int32_t) * Hg));
  }
  ALLOC(d.mrec, sizeof(uint32_t) * H);
  HIPCHK(hipMemset(d.mrec, 0, sizeof(uint32_t) * H));
  ALLOC(d.minexp, sizeof(unsigned long long) * H);
  ALLOC(d.scan_list, sizeof(grec) * H * d.L);
  ALLOC(d.scan_cnt, sizeof(uint32_t) * H);
  // worklist scans split rows of at least 64K slots into chunks of >= 32K (S | 128: owners never
  // straddle a chunk; the split path runs without listeners)
  e->scan_nch = 1;
  if (d.R >= 65536 && d.S >= 2 && 128 % d.S == 0) {
    e->scan_nch = d.R / 32768 < 16 ? d.R / 32768 : 16;  // the most chunks a row takes (scan_chunks)
    ALLOC(e->scan_tmp, sizeof(grec) * H * e->scan_nch * d.L);
    ALLOC(e->scan_chunk, sizeof(ScanChunk) * H * e->scan_nch);
  }
  ALLOC(d.tick, H);
  ALLOC(d.sbytes, sizeof(uint16_t) * d.R);
  ALLOC(d.srvt, sizeof(gx_server_times) * H * Hg);
  ALLOC(d.vlc, sizeof(int64_t) * H);
  ALLOC(d.ev_slot, sizeof(int32_t) * H);
  ALLOC(d.ctr, sizeof(DevCtr));
  d.departures = p->depart_round >= 0 && p->depart_ppm;
  if (p->fd_enable) {  // member rows of this shard's hosts
    ALLOC(d.mem, sizeof(gx_member) * H * Hg);
    ALLOC(d.fd_dl, sizeof(int32_t) * H * Hg);
    ALLOC(d.fdh, sizeof(gx_fd_host) * H);
    ALLOC(d.fdm, sizeof(gx_fd_msg) * Hg * K * p->fd_msg_cap);
    ALLOC(d.fd_len, sizeof(uint32_t) * Hg * K);
    ALLOC(d.fd_peers, sizeof(uint32_t) * H * K);
    ALLOC(d.fd_np, sizeof(uint32_t) * H);
    if (p->fd_push_pull_state) ALLOC(d.fd_snap, sizeof(uint64_t) * H * Hg);
  }
  if (p->lock_model) {  // locked hosts' inbound pipelines and waiting ExpireServer calls (gx.h lock_model)
    d.C = p->lock_buffer;
    ALLOC(d.lkb, sizeof(grec) * H * d.C);
    d.PW = (d.H + 31) / 32;
    if (p->storm_round >= 0 || p->fd_enable) {
      ALLOC(d.pexp, sizeof(uint32_t) * H * d.PW);
      HIPCHK(hipMemset(d.pexp, 0, sizeof(uint32_t) * H * d.PW));
    }
    if (p->lock_readers) {  // the waiting push-pull merges' pool (gx.h lock_readers)
      d.P = p->lock_defer_slots ? p->lock_defer_slots : 64;
      ALLOC(d.dpool, sizeof(uint64_t) * d.P * d.R);
      ALLOC(d.dpool_host, sizeof(uint32_t) * d.P);
      ALLOC(d.dpool_res, sizeof(uint32_t) * d.P);
      ALLOC(d.dclaim, sizeof(uint32_t) * d.P);
      ALLOC(d.ro_flag, H);
      ALLOC(d.ro_list, sizeof(uint32_t) * H);
      HIPCHK(hipMemset(d.dpool_host, 0xff, sizeof(uint32_t) * d.P));
      HIPCHK(hipMemset(d.dclaim, 0xff, sizeof(uint32_t) * d.P));
      HIPCHK(hipMemset(d.dpool_res, 0, sizeof(uint32_t) * d.P));
      HIPCHK(hipMemset(d.ro_flag, 0, H));
    }
    if (p->fd_handoff_shared) {  // the handoff queue's places after the 53 the handler's chain holds
      d.HQ = d.C > GX_LOCK_HANDLER_AT ? d.C - GX_LOCK_HANDLER_AT : 0;
      ALLOC(d.fdq, sizeof(gx_fd_msg) * H * (d.HQ ? d.HQ : 1));
    }
  }
  ALLOC(e->conv_bad, sizeof(unsigned long long));
  e->xplan_stream = nullptr;
  e->xplan_dev = e->xplan_host = nullptr;
  e->xplan_start[0] = e->xplan_start[1] = -1;
  e->xplan_waits[0] = e->xplan_waits[1] = 0;
  e->xplan_ev[0] = e->xplan_ev[1] = nullptr;
  e->xplan_join = nullptr;
  e->xbound_round = -1;
  e->xbound_dev = nullptr;
  e->kprof_n = 0;
  if (getenv("GX_KPROF")) {  // diagnostics: phase marks of every k_send wave (gx_kprof_read)
    e->kprof_n = (size_t)nblk(d.Hl, 64) * 4 * 8 + GX_KPROF_MERGE_N + 3ull * d.H;  // + merge counts + push-pull blocks + scans
    ALLOC(d.kprof, sizeof(unsigned long long) * e->kprof_n);
    HIPCHK(hipMemset(d.kprof, 0, sizeof(unsigned long long) * e->kprof_n));
  }
  ALLOC(e->digest_buf, sizeof(uint64_t) * H);
  if (d.G > 1) {
    ALLOC(e->ob_entries, sizeof(uint32_t) * H * K);
    ALLOC(d.in_stamp, sizeof(uint32_t) * Hg * K);
    HIPCHK(hipMemset(d.in_stamp, 0, sizeof(uint32_t) * Hg * K));
    ALLOC(e->ob_total, sizeof(uint32_t));
    ALLOC(e->ob_claim, sizeof(uint32_t) * (XPLAN_GMAX + 1));
    HIPCHK(hipMemset(e->ob_claim, 0, sizeof(uint32_t) * (XPLAN_GMAX + 1)));
    ALLOC(e->ob_counts, sizeof(uint32_t) * p->n_shards * (1 + 2 * ((H * K + 255) / 256)));
    size_t np = Hg / 2 + 1;
    ALLOC(e->ae_pa, sizeof(uint32_t) * np);
    ALLOC(e->ae_pb, sizeof(uint32_t) * np);
    ALLOC(e->ae_prow, sizeof(int32_t) * np);
    ALLOC(e->ae_pcount, np);
    ALLOC(e->ae_pack_host, sizeof(uint32_t) * np);
    ALLOC(e->ae_pack_t, sizeof(uint32_t) * np);
    ALLOC(e->ae_pack_other, sizeof(uint32_t) * np);
    ALLOC(e->ae_pack_first, np);
    ALLOC(e->ae_skip, np);
    if (p->fd_enable && p->fd_push_pull_state) ALLOC(e->fd_rsnap, sizeof(uint64_t) * np * Hg);
    e->nblk = (d.R + GX_DIGEST_SLOTS - 1) / GX_DIGEST_SLOTS;
    e->nmw = (e->nblk + 31) / 32;
    ALLOC(e->ae_dig, sizeof(ulonglong2) * H * e->nblk);
    ALLOC(e->ae_mask, sizeof(uint32_t) * H * e->nmw);
    ALLOC(e->ae_fmask, sizeof(uint32_t) * H * e->nmw);
    ALLOC(e->ae_lt, sizeof(uint16_t) * H * e->nblk);
    ALLOC(e->ae_retL, sizeof(uint16_t) * H * e->nblk);
    ALLOC(e->ae_bcnt, sizeof(uint32_t) * H * e->nblk);
    ALLOC(e->ae_cnt, sizeof(uint32_t) * H);
    ALLOC(e->ae_nfol, sizeof(uint32_t) * H);
    ALLOC(e->ae_sz, sizeof(uint64_t) * 4 * H);
    ALLOC(e->ae_off, sizeof(uint64_t) * 4 * H);
    ALLOC(e->ae_rioff, sizeof(uint64_t) * H);
    ALLOC(e->ae_err, sizeof(uint32_t));
  }
  hipStream_t s = e->stream;
  uint64_t *rec_word = nullptr;
  ALLOC(rec_word, sizeof(uint64_t) * d.R);
  HIPCHK(hipMemsetAsync(d.ctr, 0, sizeof(DevCtr), s));
  HIPCHK(hipMemsetAsync(d.ctr->first_drop, 0xff, sizeof(d.ctr->first_drop), s));  // min: none yet
  HIPCHK(hipMemsetAsync(d.arena_len, 0, sizeof(uint32_t) * H * d.A, s));
  HIPCHK(hipMemsetAsync(d.msg_len, 0, sizeof(uint32_t) * Hg * K, s));
  HIPCHK(hipMemsetAsync(e->in_cnt_buf, 0, sizeof(uint32_t) * 2 * H, s));
  HIPCHK(hipMemsetAsync(d.work_cnt, 0, sizeof(uint32_t) * GX_WC_N, s));
  HIPCHK(hipMemsetAsync(d.tick, 0, H, s));
  HIPCHK(hipMemsetAsync(d.ev_slot, 0xff, sizeof(int32_t) * H, s));  // -1: no listener
  k_fill_u16<<<256, 256, 0, s>>>(d.sbytes, d.R, (uint16_t)GX_STATIC_BYTES_DEFAULT);
  set_round_fields(e);
  k_init_rec<<<nblk(d.R, 256), 256, 0, s>>>(d, rec_word);
  k_init_views<<<2048, 256, 0, s>>>(d, rec_word);
  k_init_times<<<2048, 256, 0, s>>>(d, rec_word);
  k_init_hosts<<<nblk(d.Hl, 256), 256, 0, s>>>(d);
  if (p->fd_enable) {
    k_fd_init<<<2048, 256, 0, s>>>(d);
    HIPCHK(hipMemsetAsync(d.fd_len, 0, sizeof(uint32_t) * Hg * K, s));
  }
  k_minexp_recompute<<<d.Hl, 256, 0, s>>>(d, 0);
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
  if (!e || round < e->d.round || round >= GX_MAX_ROUND) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  if (round != e->d.round) {  // a jump: this round's and the next round's counters start empty
    HIPCHK(hipMemsetAsync(e->in_cnt_buf, 0, sizeof(uint32_t) * 2 * e->d.Hl, e->stream));
    HIPCHK(hipMemsetAsync(e->d.work_cnt, 0, sizeof(uint32_t) * GX_WC_ERR, e->stream));
  }
  e->d.round = round;
  set_round_fields(e);
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
  if (!e || e->d.G > 1 || e->d.round + n_rounds >= GX_MAX_ROUND) return GX_EINVAL;
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
  if (s->host >= e->d.H || s->svc >= e->d.S || s->status > 6) return GX_EINVAL;
  g->w = pack(gx_ts_in(s->updated_ns, e->d.epoch), s->status);
  g->r = s->host * e->d.S + s->svc;
  g->pad = 0;
  return GX_OK;
}
static void to_svc(const gx_engine *e, const grec *g, gx_service *s) {
  s->updated_ns = ts_of(g->w) + e->d.epoch;
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
      if (!own(e, views[i])) return GX_EINVAL;
  size_t vbytes = ((sizeof(uint32_t) * (n + 1)) + 255) & ~(size_t)255;
  grec *drec;
  int rc = stage_recs(e, svcs, n, vbytes + 256, &drec);
  if (rc) return rc;
  uint32_t *dviews = (uint32_t *)e->api_dev;
  uint32_t *dacc = (uint32_t *)((char *)e->api_dev + vbytes);
  if (views && n) HIPCHK(hipMemcpyAsync(dviews, views, sizeof(uint32_t) * n, hipMemcpyHostToDevice, e->stream));
  set_round_fields(e);
  k_api_add<<<1, 64, 0, e->stream>>>(e->d, views ? dviews : nullptr, fixed_view, drec, n, src, dacc);
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
  if (!e || !own(e, host) || (n && !recs)) return GX_EINVAL;
  return api_add(e, nullptr, host, recs, n, SRC_GOSSIP, nullptr);
}

int gx_merge_remote_state(gx_engine *e, uint32_t view, const gx_service *svcs, uint32_t n) {
  if (!e || !own(e, view) || (n && !svcs)) return GX_EINVAL;
  return api_add(e, nullptr, view, svcs, n, SRC_AE, nullptr);
}

int gx_merge(gx_engine *e, uint32_t dst, uint32_t src) {
  if (!e || !own(e, dst) || !own(e, src)) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  set_round_fields(e);
  const bool ev = !e->log_views.empty();
  if (e->d.R % 2 == 0 && !ev) k_merge_views<true, false><<<1, 256, 0, e->stream>>>(e->d, dst, src);
  else if (e->d.R % 2 == 0) k_merge_views<true, true><<<1, 256, 0, e->stream>>>(e->d, dst, src);
  else if (!ev) k_merge_views<false, false><<<1, 256, 0, e->stream>>>(e->d, dst, src);
  else k_merge_views<false, true><<<1, 256, 0, e->stream>>>(e->d, dst, src);
  return sync_check(e);
}

int gx_tombstone_others(gx_engine *e, uint32_t view, gx_service *out, uint32_t cap, uint32_t *n_out) {
  if (!e || !own(e, view) || (cap && !out)) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  int rc = ensure_api(e, 256 + sizeof(grec) * (cap + 1));
  if (rc) return rc;
  uint32_t *dcnt = (uint32_t *)e->api_dev;
  grec *dlist = (grec *)((char *)e->api_dev + 256);
  set_round_fields(e);
  (e->d.R % 2 == 0 ? k_scan<true, true> : k_scan<false, true>)<<<1, 256, 0, e->stream>>>(e->d, dlist, 0, cap, dcnt,
                                                                                        (int)view);
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
  if (!e || !own(e, host) || (n_running && !running) || (cap && !out)) return GX_EINVAL;
  uint64_t mask = 0;
  for (uint32_t i = 0; i < n_running; i++) {
    if (running[i] >= e->d.S) return GX_EINVAL;
    mask |= 1ull << running[i];
  }
  HIPCHK(hipSetDevice(e->device));
  int rc = ensure_api(e, 64);
  if (rc) return rc;
  set_round_fields(e);
  k_api_tomb<<<1, 64, 0, e->stream>>>(e->d, host, mask, (uint64_t *)e->api_dev);
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
  if (!e || !own(e, view) || owner >= e->d.H) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  int rc = ensure_api(e, 64);
  if (rc) return rc;
  set_round_fields(e);
  k_api_expire<<<1, 64, 0, e->stream>>>(e->d, view, owner, (uint32_t *)e->api_dev);
  uint32_t x = 0;
  HIPCHK(hipMemcpyAsync(&x, e->api_dev, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  rc = sync_check(e);
  if (rc) return rc;
  if (expired) *expired = (int)x;
  return GX_OK;
}

int gx_notify_leave(gx_engine *e, uint32_t view, uint32_t node) { return gx_expire_server(e, view, node, nullptr); }

int gx_send_services(gx_engine *e, uint32_t host, const gx_service *svcs, uint32_t n, uint32_t n_passes) {
  if (!e || !own(e, host) || (n && !svcs) || n_passes < 1 || n_passes > GX_JOB_MAX_PASSES) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  grec *drec;
  int rc = stage_recs(e, svcs, n, 0, &drec);
  if (rc) return rc;
  set_round_fields(e);
  k_api_send<<<1, 64, 0, e->stream>>>(e->d, host, drec, n, n_passes);
  return sync_check(e);
}

int gx_broadcast_services(gx_engine *e, uint32_t host, const gx_service *list, uint32_t n) {
  if (!e || !own(e, host) || (n && !list) || n > 64) return GX_EINVAL;
  for (uint32_t i = 0; i < n; i++)
    if (list[i].host != host) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  grec *drec;
  int rc = stage_recs(e, list, n, 0, &drec);
  if (rc) return rc;
  set_round_fields(e);
  k_api_bs<<<1, 64, 0, e->stream>>>(e->d, host, drec, n);
  return sync_check(e);
}

int gx_broadcast_tombstones(gx_engine *e, uint32_t host, const gx_service *list, uint32_t n) {
  if (!e || !own(e, host) || (n && !list)) return GX_EINVAL;
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
  (e->d.R % 2 == 0 ? k_scan<true, true> : k_scan<false, true>)<<<1, 256, 0, e->stream>>>(e->d, dlist, 0, e->d.L, dcnt,
                                                                                        (int)host);
  k_api_bt<<<1, 64, 0, e->stream>>>(e->d, host, mask, dlist, dcnt);
  return sync_check(e);
}

int gx_owner_slots_in_use(gx_engine *e, uint32_t owner, uint64_t *mask) {
  if (!e || !mask || owner >= e->d.H) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  int rc = ensure_api(e, 64);
  if (rc) return rc;
  HIPCHK(hipMemsetAsync(e->api_dev, 0, sizeof(uint64_t), e->stream));
  k_slots_in_use<<<nblk(e->d.Hl, 256), 256, 0, e->stream>>>(e->d, owner, (unsigned long long *)e->api_dev);
  HIPCHK(hipMemcpyAsync(mask, e->api_dev, sizeof(uint64_t), hipMemcpyDeviceToHost, e->stream));
  return sync_check(e);
}

int gx_is_new_service(gx_engine *e, uint32_t view, const gx_service *svc, int *out) {
  grec g;
  if (!e || !svc || !out || !own(e, view) || to_grec(e, svc, &g)) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  int rc = ensure_api(e, 64);
  if (rc) return rc;
  k_api_is_new<<<1, 64, 0, e->stream>>>(e->d, view, g.w, g.r, (uint32_t *)e->api_dev);
  uint32_t x = 0;
  HIPCHK(hipMemcpyAsync(&x, e->api_dev, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  rc = sync_check(e);
  if (rc) return rc;
  *out = (int)x;
  return GX_OK;
}

static int getb_impl(gx_engine *e, uint32_t host, uint32_t limit, uint32_t limit_bytes, uint32_t overhead,
                     gx_service *out, uint32_t *n_out) {
  HIPCHK(hipSetDevice(e->device));
  int rc = ensure_api(e, 256 + sizeof(grec) * (limit + 1));
  if (rc) return rc;
  uint32_t *dn = (uint32_t *)e->api_dev;
  grec *dpk = (grec *)((char *)e->api_dev + 256);
  set_round_fields(e);
  k_api_getb<<<1, 64, 0, e->stream>>>(e->d, host, limit, dpk, dn, limit_bytes, overhead);
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

int gx_get_broadcasts(gx_engine *e, uint32_t host, uint32_t limit, gx_service *out, uint32_t cap, uint32_t *n_out) {
  if (limit == GX_LIMIT_DEFAULT) limit = e ? e->d.p.packet_cap : 0;
  if (!e || !own(e, host) || !n_out || limit > 256 || cap < limit || (limit && !out)) return GX_EINVAL;
  return getb_impl(e, host, limit, 0, 0, out, n_out);
}

int gx_get_broadcasts_bytes(gx_engine *e, uint32_t host, uint32_t overhead, uint32_t limit, gx_service *out,
                            uint32_t cap, uint32_t *n_out) {
  if (!e || !own(e, host) || !n_out || (cap && !out) || cap > (1u << 20)) return GX_EINVAL;
  if (limit == 0 || cap == 0) {  // nothing can fit: the batch still moves to pending
    return getb_impl(e, host, 0, 0, 0, out, n_out);
  }
  return getb_impl(e, host, cap, limit, overhead, out, n_out);
}

int gx_set_static_bytes(gx_engine *e, uint32_t owner_lo, uint32_t owner_hi, const uint16_t *bytes) {
  if (!e || owner_lo > owner_hi || owner_hi > e->d.H || (owner_hi > owner_lo && !bytes)) return GX_EINVAL;
  if (owner_hi == owner_lo) return GX_OK;
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipStreamSynchronize(e->stream));
  size_t n = (size_t)(owner_hi - owner_lo) * e->d.S;
  HIPCHK(hipMemcpy(&e->d.sbytes[(size_t)owner_lo * e->d.S], bytes, sizeof(uint16_t) * n, hipMemcpyHostToDevice));
  return GX_OK;
}

int gx_message_bytes(gx_engine *e, const gx_service *recs, uint32_t n, uint32_t *out_bytes) {
  if (!e || (n && (!recs || !out_bytes))) return GX_EINVAL;
  if (!n) return GX_OK;
  std::vector<grec> g(n);
  for (uint32_t i = 0; i < n; i++)
    if (to_grec(e, &recs[i], &g[i])) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  int rc = ensure_api(e, 256 + (sizeof(grec) + sizeof(uint32_t)) * (size_t)n);
  if (rc) return rc;
  grec *dg = (grec *)((char *)e->api_dev + 256);
  uint32_t *dout = (uint32_t *)(dg + n);
  HIPCHK(hipMemcpyAsync(dg, g.data(), sizeof(grec) * n, hipMemcpyHostToDevice, e->stream));
  k_api_msg_bytes<<<nblk(n, 256), 256, 0, e->stream>>>(e->d, dg, n, dout);
  HIPCHK(hipMemcpyAsync(out_bytes, dout, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, e->stream));
  return sync_check(e);
}

int gx_local_state(gx_engine *e, uint32_t view, gx_service *out, uint32_t cap, uint32_t *n_out) {
  if (!e || !own(e, view) || (cap && !out)) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipStreamSynchronize(e->stream));
  std::vector<uint64_t> row(e->d.R);
  HIPCHK(hipMemcpy(row.data(), &e->d.view[(size_t)(view - e->d.lo) * e->d.R], sizeof(uint64_t) * e->d.R,
                   hipMemcpyDeviceToHost));
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

extern "C" int gx_sort_u64_pairs(void *tmp, size_t *tmp_bytes, uint64_t *keys_in, uint64_t *keys_out,
                                 uint32_t *vals_in, uint32_t *vals_out, uint32_t n, int end_bit, hipStream_t s);
extern "C" int gx_sort_u32_pairs(void *tmp, size_t *tmp_bytes, uint32_t *keys_in, uint32_t *keys_out,
                                 uint32_t *vals_in, uint32_t *vals_out, uint32_t n, int end_bit, hipStream_t s);

// EachServiceSorted / SortedServices / ByService on the device: the view's present records
// compacted in key order, stable radix sort by Updated (ties stay in key order), for ByService a
// second stable sort by the Name rank, then written out as gx_service.
static int sorted_view(gx_engine *e, uint32_t view, uint32_t owner, bool by_name, gx_service *out, uint32_t *group_out,
                       uint32_t cap, uint32_t *n_out) {
  Dev &d = e->d;
  HIPCHK(hipSetDevice(e->device));
  hipStream_t s = e->stream;
  const uint32_t vi = view - d.lo, nb = (d.R + VC_CHUNK - 1) / VC_CHUNK;
  uint32_t *cnt = nullptr, *v0 = nullptr, *v1 = nullptr, *k32a = nullptr, *k32b = nullptr;
  uint64_t *k0 = nullptr, *k1 = nullptr;
  gx_service *dout = nullptr;
  void *tmp = nullptr;
  int rc = GX_OK;
  uint32_t n = 0;
  auto fail = [&](hipError_t err) { return err == hipSuccess ? GX_OK : (err == hipErrorOutOfMemory ? GX_ENOMEM : GX_EIO); };
#define VCK(x)                    \
  do {                            \
    rc = fail(x);                 \
    if (rc) goto done;            \
  } while (0)
  VCK(hipMalloc(&cnt, sizeof(uint32_t) * (nb + 1)));
  k_vc_count<<<nb, 256, 0, s>>>(d, vi, owner, cnt);
  k_vc_scan<<<1, 1024, 0, s>>>(cnt, nb);
  VCK(hipMemcpyAsync(&n, &cnt[nb], sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  VCK(hipStreamSynchronize(s));
  if (n) {
    VCK(hipMalloc(&k0, sizeof(uint64_t) * n));
    VCK(hipMalloc(&k1, sizeof(uint64_t) * n));
    VCK(hipMalloc(&v0, sizeof(uint32_t) * n));
    VCK(hipMalloc(&v1, sizeof(uint32_t) * n));
    VCK(hipMalloc(&dout, sizeof(gx_service) * n));
    k_vc_write<<<nb, 256, 0, s>>>(d, vi, owner, cnt, k0, v0);
    size_t tb = 0, tb2 = 0;
    if (gx_sort_u64_pairs(nullptr, &tb, k0, k1, v0, v1, n, 64 - GX_TS_SHIFT, s)) VCK(hipErrorUnknown);
    if (by_name) {
      VCK(hipMalloc(&k32a, sizeof(uint32_t) * n));
      VCK(hipMalloc(&k32b, sizeof(uint32_t) * n));
      if (gx_sort_u32_pairs(nullptr, &tb2, k32a, k32b, v1, v0, n, 32, s)) VCK(hipErrorUnknown);
    }
    VCK(hipMalloc(&tmp, std::max<size_t>(std::max(tb, tb2), 1)));
    if (gx_sort_u64_pairs(tmp, &tb, k0, k1, v0, v1, n, 64 - GX_TS_SHIFT, s)) VCK(hipErrorUnknown);
    uint32_t *order = v1;
    if (by_name) {
      k_vc_rank<<<nblk(n, 256), 256, 0, s>>>(e->name_rank, v1, k32a, n);
      if (gx_sort_u32_pairs(tmp, &tb2, k32a, k32b, v1, v0, n, 32, s)) VCK(hipErrorUnknown);
      order = v0;
    }
    k_vc_out<<<nblk(n, 256), 256, 0, s>>>(d, vi, order, n, dout);
    const uint32_t m = n < cap ? n : cap;
    if (m) {
      VCK(hipMemcpyAsync(out, dout, sizeof(gx_service) * m, hipMemcpyDeviceToHost, s));
      if (by_name && group_out) VCK(hipMemcpyAsync(group_out, k32b, sizeof(uint32_t) * m, hipMemcpyDeviceToHost, s));
    }
    VCK(hipStreamSynchronize(s));
    VCK(hipGetLastError());
  }
  if (n_out) *n_out = n;
done:
#undef VCK
  for (void *p : {(void *)cnt, (void *)k0, (void *)k1, (void *)v0, (void *)v1, (void *)k32a, (void *)k32b, (void *)dout, tmp})
    if (p) (void)hipFree(p);
  return rc;
}

int gx_each_service_sorted(gx_engine *e, uint32_t view, uint32_t owner, gx_service *out, uint32_t cap,
                           uint32_t *n_out) {
  if (!e || !own(e, view) || (owner != GX_ALL_OWNERS && owner >= e->d.H) || (cap && !out)) return GX_EINVAL;
  return sorted_view(e, view, owner, false, out, nullptr, cap, n_out);
}

int gx_set_service_names(gx_engine *e, const char *names, const uint64_t *off) {
  if (!e || !off) return GX_EINVAL;
  const uint32_t R = e->d.R;
  if (off[0] != 0) return GX_EINVAL;
  for (uint32_t r = 0; r < R; r++)
    if (off[r + 1] < off[r]) return GX_EINVAL;
  if (off[R] && !names) return GX_EINVAL;
  // rank = index of the record's Name among the distinct names in bytewise order
  std::vector<uint32_t> idx(R), rank(R);
  for (uint32_t r = 0; r < R; r++) idx[r] = r;
  auto name = [&](uint32_t r) { return std::string(names ? names + off[r] : "", (size_t)(off[r + 1] - off[r])); };
  std::vector<std::string> nm(R);
  for (uint32_t r = 0; r < R; r++) nm[r] = name(r);
  std::stable_sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return nm[a] < nm[b]; });
  uint32_t g = 0;
  for (uint32_t k = 0; k < R; k++) {
    if (k && nm[idx[k]] != nm[idx[k - 1]]) g++;
    rank[idx[k]] = g;
  }
  HIPCHK(hipSetDevice(e->device));
  if (!e->name_rank) {
    if (hipMalloc(&e->name_rank, sizeof(uint32_t) * R) != hipSuccess) {
      (void)hipGetLastError();
      e->name_rank = nullptr;
      return GX_ENOMEM;
    }
  }
  HIPCHK(hipMemcpy(e->name_rank, rank.data(), sizeof(uint32_t) * R, hipMemcpyHostToDevice));
  return GX_OK;
}

int gx_by_service(gx_engine *e, uint32_t view, gx_service *out, uint32_t *group_out, uint32_t cap, uint32_t *n_out) {
  if (!e || !own(e, view) || (cap && !out)) return GX_EINVAL;
  if (!e->name_rank) return GX_ENOENT;
  return sorted_view(e, view, GX_ALL_OWNERS, true, out, group_out, cap, n_out);
}

int gx_epoch(gx_engine *e, int64_t *epoch_ns) {
  if (!e || !epoch_ns) return GX_EINVAL;
  *epoch_ns = e->d.epoch;
  return GX_OK;
}

int gx_read_server_times(gx_engine *e, uint32_t view, uint32_t lo, uint32_t hi, gx_server_times *out) {
  if (!e || !own(e, view) || lo > hi || hi > e->d.H || (hi > lo && !out)) return GX_EINVAL;
  if (hi == lo) return GX_OK;
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipStreamSynchronize(e->stream));
  HIPCHK(hipMemcpy(out, &e->d.srvt[(size_t)(view - e->d.lo) * e->d.H + lo], sizeof(gx_server_times) * (hi - lo),
                   hipMemcpyDeviceToHost));
  for (uint32_t o = 0; o < hi - lo; o++) {
    out[o].last_updated_ns = abs_tm(e, out[o].last_updated_ns);
    out[o].last_changed_ns = abs_tm(e, out[o].last_changed_ns);
  }
  return GX_OK;
}

int gx_read_last_changed(gx_engine *e, uint32_t lo, uint32_t hi, int64_t *out) {
  if (!e || lo > hi || (hi > lo && (!out || !own(e, lo) || !own(e, hi - 1)))) return GX_EINVAL;
  if (hi == lo) return GX_OK;
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipStreamSynchronize(e->stream));
  HIPCHK(hipMemcpy(out, &e->d.vlc[lo - e->d.lo], sizeof(int64_t) * (hi - lo), hipMemcpyDeviceToHost));
  for (uint32_t v = 0; v < hi - lo; v++) out[v] = abs_tm(e, out[v]);
  return GX_OK;
}

// Device event logs: one per listening view, sized for the largest channel capacity.
static int rebuild_logs(gx_engine *e) {
  Dev &d = e->d;
  std::vector<uint32_t> views;
  uint32_t cap = 0;
  for (auto &l : e->listeners) {
    bool seen = false;
    for (uint32_t v : views) seen |= v == l.view;
    if (!seen) views.push_back(l.view);
    cap = l.cap > cap ? l.cap : cap;
  }
  HIPCHK(hipStreamSynchronize(e->stream));
  if (d.ev_log) (void)hipFree(d.ev_log);
  if (d.ev_cnt) (void)hipFree(d.ev_cnt);
  d.ev_log = nullptr;
  d.ev_cnt = nullptr;
  d.ev_cap = 0;
  HIPCHK(hipMemset(d.ev_slot, 0xff, sizeof(int32_t) * d.Hl));
  e->log_views = views;
  if (views.empty()) return GX_OK;
  if (hipMalloc((void **)&d.ev_log, sizeof(gx_change_event) * cap * views.size()) != hipSuccess ||
      hipMalloc((void **)&d.ev_cnt, sizeof(uint32_t) * views.size()) != hipSuccess) {
    (void)hipGetLastError();
    e->listeners.clear();
    e->log_views.clear();
    return GX_ENOMEM;
  }
  d.ev_cap = cap;
  HIPCHK(hipMemset(d.ev_cnt, 0, sizeof(uint32_t) * views.size()));
  for (size_t k = 0; k < views.size(); k++) {
    int32_t slot = (int32_t)k;
    HIPCHK(hipMemcpy(&d.ev_slot[views[k] - d.lo], &slot, sizeof(int32_t), hipMemcpyHostToDevice));
  }
  return GX_OK;
}

int gx_add_listener(gx_engine *e, uint32_t view, uint32_t id, uint32_t capacity) {
  if (!e || !own(e, view) || capacity < 1 || capacity > GX_LISTENER_MAX_CAPACITY) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  bool found = false;
  for (auto &l : e->listeners)
    if (l.view == view && l.id == id) {
      l.cap = capacity;
      l.ring.clear();
      found = true;
    }
  if (!found) {
    if (e->listeners.size() >= GX_MAX_LISTENERS) return GX_ENOMEM;
    e->listeners.push_back({view, id, capacity, {}});
  }
  return rebuild_logs(e);
}

int gx_remove_listener(gx_engine *e, uint32_t view, uint32_t id) {
  if (!e) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  for (size_t i = 0; i < e->listeners.size(); i++)
    if (e->listeners[i].view == view && e->listeners[i].id == id) {
      e->listeners.erase(e->listeners.begin() + (long)i);
      return rebuild_logs(e);
    }
  return GX_ENOENT;
}

int gx_listener_drain(gx_engine *e, uint32_t view, uint32_t id, gx_change_event *out, uint32_t cap,
                      uint32_t *n_out) {
  if (!e || !n_out || (cap && !out)) return GX_EINVAL;
  for (auto &l : e->listeners)
    if (l.view == view && l.id == id) {
      uint32_t n = (uint32_t)l.ring.size() < cap ? (uint32_t)l.ring.size() : cap;
      for (uint32_t i = 0; i < n; i++) {
        out[i] = l.ring.front();
        l.ring.pop_front();
      }
      *n_out = n;
      return GX_OK;
    }
  return GX_ENOENT;
}

int gx_read_views(gx_engine *e, uint32_t lo, uint32_t hi, uint64_t *out) {
  if (!e || lo > hi || lo < e->d.lo || hi > e->d.lo + e->d.Hl || (hi > lo && !out)) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipStreamSynchronize(e->stream));
  if (hi > lo)
    HIPCHK(hipMemcpy(out, &e->d.view[(size_t)(lo - e->d.lo) * e->d.R], sizeof(uint64_t) * (size_t)(hi - lo) * e->d.R,
                     hipMemcpyDeviceToHost));
  return GX_OK;
}

int gx_notify_msgs(gx_engine *e, const uint32_t *hosts, const gx_service *recs, uint32_t n) {
  if (!e || (n && (!hosts || !recs))) return GX_EINVAL;
  for (uint32_t i = 0; i < n;) {
    uint32_t j = i + 1;
    while (j < n && hosts[j] == hosts[i]) j++;
    int rc = gx_notify_msg(e, hosts[i], recs + i, j - i);
    if (rc) return rc;
    i = j;
  }
  return GX_OK;
}

int gx_read_view(gx_engine *e, uint32_t view, int64_t *ts_ns, uint8_t *status) {
  if (!e || !ts_ns || !status) return GX_EINVAL;
  size_t R = (size_t)e->d.R;
  uint64_t *w = (uint64_t *)malloc(8 * R);
  if (!w) return GX_ENOMEM;
  int rc = gx_read_views(e, view, view + 1, w);
  for (size_t r = 0; rc == GX_OK && r < R; r++) {
    status[r] = (uint8_t)(w[r] & 7u);
    ts_ns[r] = status[r] == GX_ABSENT ? INT64_MIN : (int64_t)(w[r] >> 3) + e->d.epoch;
  }
  free(w);
  return rc;
}

int gx_write_views(gx_engine *e, uint32_t lo, uint32_t hi, const uint64_t *in) {
  if (!e || lo > hi || lo < e->d.lo || hi > e->d.lo + e->d.Hl || (hi > lo && !in)) return GX_EINVAL;
  size_t n = (size_t)(hi - lo) * e->d.R;
  for (size_t i = 0; i < n; i++)
    if (st_of(in[i]) == 7 && in[i] != GX_SLOT_ABSENT) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipStreamSynchronize(e->stream));
  if (n) HIPCHK(hipMemcpy(&e->d.view[(size_t)(lo - e->d.lo) * e->d.R], in, sizeof(uint64_t) * n, hipMemcpyHostToDevice));
  set_round_fields(e);
  k_api_mark<<<1, 64, 0, e->stream>>>(e->d);
  if (hi > lo) k_minexp_recompute<<<hi - lo, 256, 0, e->stream>>>(e->d, lo - e->d.lo);
  return sync_check(e);
}

int gx_write_slot(gx_engine *e, uint32_t view, const gx_service *svc) {
  if (!e || !svc || !own(e, view)) return GX_EINVAL;
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
  k_api_set_slot<<<1, 64, 0, e->stream>>>(e->d, view, r, w);
  return sync_check(e);
}

int gx_read_hosts(gx_engine *e, uint32_t lo, uint32_t hi, gx_host_state *out) {
  if (!e || lo > hi || lo < e->d.lo || hi > e->d.lo + e->d.Hl || (hi > lo && !out)) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipStreamSynchronize(e->stream));
  if (hi > lo) HIPCHK(hipMemcpy(out, &e->d.hs[lo - e->d.lo], sizeof(gx_host_state) * (hi - lo), hipMemcpyDeviceToHost));
  return GX_OK;
}

#define GX_READ_RING(J)                                                                                     \
  static int read_ring(gx_engine *e, const J *base, uint32_t ring, uint32_t head, uint32_t n, J *out, uint32_t cap) { \
    uint32_t m = n < cap ? n : cap;                                                                         \
    for (uint32_t i = 0; i < m;) {                                                                          \
      uint32_t idx = (head + i) % ring;                                                                     \
      uint32_t run = ring - idx;                                                                            \
      if (run > m - i) run = m - i;                                                                         \
      HIPCHK(hipMemcpy(&out[i], &base[idx], sizeof(J) * run, hipMemcpyDeviceToHost));                      \
      i += run;                                                                                             \
    }                                                                                                       \
    return GX_OK;                                                                                           \
  }
GX_READ_RING(gx_job)
GX_READ_RING(gx_sleeper)
#undef GX_READ_RING
int gx_read_queue(gx_engine *e, uint32_t host, gx_job *out, uint32_t cap, uint32_t *n_out) {
  if (!e || !own(e, host) || (cap && !out)) return GX_EINVAL;
  gx_host_state h;
  int rc = gx_read_hosts(e, host, host + 1, &h);
  if (rc) return rc;
  uint32_t n = h.fifo_stored - h.fifo_head;  // the stored jobs (gx.h)
  rc = read_ring(e, &e->d.fifo[(size_t)(host - e->d.lo) * e->d.Q], e->d.Q, h.fifo_head % e->d.Q, n, out, cap);
  if (rc) return rc;
  if (n_out) *n_out = n;
  return GX_OK;
}

int gx_read_sleepers(gx_engine *e, uint32_t host, gx_sleeper *out, uint32_t cap, uint32_t *n_out) {
  if (!e || !own(e, host) || (cap && !out)) return GX_EINVAL;
  gx_host_state h;
  int rc = gx_read_hosts(e, host, host + 1, &h);
  if (rc) return rc;
  uint32_t n = h.sleep_tail - h.sleep_head;
  rc = read_ring(e, &e->d.sleep[(size_t)(host - e->d.lo) * e->d.SQ], e->d.SQ, h.sleep_head % e->d.SQ, n, out, cap);
  if (rc) return rc;
  if (n_out) *n_out = n;
  return GX_OK;
}

int gx_read_pending(gx_engine *e, uint32_t host, gx_service *out, uint32_t cap, uint32_t *n_out) {
  if (!e || !own(e, host) || (cap && !out)) return GX_EINVAL;
  gx_host_state h;
  int rc = gx_read_hosts(e, host, host + 1, &h);
  if (rc) return rc;
  std::vector<grec> dq(e->d.DQ);
  HIPCHK(hipMemcpy(dq.data(), &e->d.dq[(size_t)(host - e->d.lo) * e->d.DQ], sizeof(grec) * e->d.DQ, hipMemcpyDeviceToHost));
  for (uint32_t i = 0; i < h.dq_len && i < cap; i++) to_svc(e, &dq[(h.dq_head + i) & (e->d.DQ - 1)], &out[i]);
  if (n_out) *n_out = h.dq_len;
  return GX_OK;
}

int gx_read_list(gx_engine *e, uint32_t host, uint32_t slot, gx_service *out, uint32_t cap, uint32_t *n_out) {
  if (!e || !own(e, host) || slot >= e->d.A || (cap && !out)) return GX_EINVAL;
  gx_host_state h;
  int rc = gx_read_hosts(e, host, host + 1, &h);
  if (rc) return rc;
  uint32_t n = 0, bits = 0;
  HIPCHK(hipMemcpy(&bits, &e->d.arena_bits[(size_t)(host - e->d.lo) * e->d.AW + slot / 32], sizeof(uint32_t),
                   hipMemcpyDeviceToHost));
  if ((bits >> (slot % 32)) & 1u)
    HIPCHK(hipMemcpy(&n, &e->d.arena_len[(size_t)(host - e->d.lo) * e->d.A + slot], sizeof(uint32_t), hipMemcpyDeviceToHost));
  uint32_t m = n < cap ? n : cap;
  if (m) {
    std::vector<grec> tmp(m);
    HIPCHK(hipMemcpy(tmp.data(), &e->d.arena[((size_t)(host - e->d.lo) * e->d.A + slot) * e->d.L], sizeof(grec) * m,
                     hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < m; i++) to_svc(e, &tmp[i], &out[i]);
  }
  if (n_out) *n_out = n;
  return GX_OK;
}

int gx_host_digests(gx_engine *e, uint64_t *out) {
  if (!e || !out) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  k_digest<<<nblk(e->d.Hl, 256), 256, 0, e->stream>>>(e->d, e->digest_buf);
  HIPCHK(hipMemcpyAsync(out, e->digest_buf, sizeof(uint64_t) * e->d.Hl, hipMemcpyDeviceToHost, e->stream));
  return sync_check(e);
}

// ------------------------------------------------------------------------- sharded rounds --
static uint32_t shard_of(const Dev &d, uint32_t v) {  // shard g owns [floor(g H / G), floor((g + 1) H / G))
  uint32_t g = (uint32_t)(((uint64_t)v * d.G) / d.H);
  while (g > 0 && (uint32_t)(((uint64_t)g * d.H) / d.G) > v) g--;
  while (g + 1 < d.G && (uint32_t)(((uint64_t)(g + 1) * d.H) / d.G) <= v) g++;
  return g;
}
// packet slot (gx.h wire format): header, packet_cap records, then fd_msg_cap memberlist messages
// when the failure detector is on
static size_t slot_bytes(const Dev &d) {
  return 16 + 16ull * d.p.packet_cap + (d.p.fd_enable ? 16ull * d.p.fd_msg_cap : 0);
}
static size_t dig_bytes(const gx_engine *e) { return dig_stride(e->d, e->nblk); }

int gx_round_send(gx_engine *e) {
  if (!e) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  int rc = round_send_impl(e);
  return rc ? rc : phase_done(e);
}

// Entries of this shard's packets bound for other shards, grouped by destination shard in key
// order; sizes in bytes per shard.
int gx_outbox_bytes(gx_engine *e, uint64_t *bytes) {
  if (!e || !bytes) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  Dev &d = e->d;
  for (uint32_t g = 0; g < d.G; g++) bytes[g] = 0;
  e->n_ob = 0;
  e->ob_async = false;
  if (d.G < 2 || !d.K) return GX_OK;
  set_round_fields(e);
  const size_t ne = (size_t)d.Hl * d.KE;
  const uint32_t nchunk = (uint32_t)((ne + 255) / 256);
  uint32_t *ccnt = e->ob_counts + d.G, *off = ccnt + (size_t)nchunk * d.G;
  const size_t lds = sizeof(uint32_t) * 4 * d.G;
  k_ob_count<<<nchunk, 256, lds, e->stream>>>(d, ccnt);
  k_ob_scan<<<1, 256, 0, e->stream>>>(d, ccnt, nchunk, off, e->ob_counts);
  k_ob_fill<<<nchunk, 256, lds, e->stream>>>(d, off, e->ob_entries);
  std::vector<uint32_t> cnt(d.G);
  HIPCHK(hipMemcpyAsync(cnt.data(), e->ob_counts, sizeof(uint32_t) * d.G, hipMemcpyDeviceToHost, e->stream));
  int rc = sync_check(e);
  if (rc) return rc;
  uint64_t n = 0;
  for (uint32_t g = 0; g < d.G; g++) {
    bytes[g] = cnt[g] * slot_bytes(d);
    n += cnt[g];
  }
  e->n_ob = (uint32_t)n;
  return GX_OK;
}

int gx_outbox_sizes_async(gx_engine *e, uint64_t *bytes) {
  if (!e || !bytes) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  Dev &d = e->d;
  e->n_ob = 0;
  e->ob_async = false;
  if (d.G < 2 || !d.K) {
    HIPCHK(hipMemsetAsync(bytes, 0, sizeof(uint64_t) * d.G, e->stream));
    return phase_done(e);
  }
  set_round_fields(e);
  const size_t ne = (size_t)d.Hl * d.KE;
  const uint32_t nchunk = (uint32_t)((ne + 255) / 256);
  uint32_t *ccnt = e->ob_counts + d.G, *off = ccnt + (size_t)nchunk * d.G;
  const size_t lds = sizeof(uint32_t) * 4 * d.G;
  k_ob_count<<<nchunk, 256, lds, e->stream>>>(d, ccnt);
  k_ob_scan<<<1, 256, 0, e->stream>>>(d, ccnt, nchunk, off, e->ob_counts);
  k_ob_fill<<<nchunk, 256, lds, e->stream>>>(d, off, e->ob_entries);
  k_ob_bytes<<<1, 64, 0, e->stream>>>(d, e->ob_counts, (unsigned long long *)bytes, e->ob_total);
  e->ob_async = true;
  return phase_done(e);
}

int gx_outbox_pack(gx_engine *e, void *buf, uint64_t cap) {
  if (!e || (cap && !buf)) return GX_EINVAL;
  if (e->ob_async) {  // the slot count is on the device: a grid of the largest possible count
    HIPCHK(hipSetDevice(e->device));
    e->ob_async = false;
    const uint32_t cap_slots = (uint32_t)(cap / slot_bytes(e->d));
    const uint32_t nmax = e->d.Hl * e->d.KE;
    if (nmax) k_outbox_pack<<<nmax, 64, 0, e->stream>>>(e->d, e->ob_entries, 0, (uint8_t *)buf, e->ob_total, cap_slots);
    return phase_done(e);
  }
  if (!e->n_ob) return GX_OK;
  if (cap < e->n_ob * slot_bytes(e->d)) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  k_outbox_pack<<<e->n_ob, 64, 0, e->stream>>>(e->d, e->ob_entries, e->n_ob, (uint8_t *)buf);
  return phase_done(e);
}

static bool send_packs(const Dev &d);
// Batch `start` of slot bounds into host slot k (asynchronous, on xplan_stream).
static int xplan_launch(gx_engine *e, int k, int64_t start) {
  Dev &d = e->d;
  const size_t n = (size_t)XPLAN_BATCH * d.G * d.G;
  uint32_t *dev = e->xplan_dev + (size_t)k * n;
  // the rounds queued so far may read this half (a packing k_send, Dev::ob_cnt): the rewrite waits
  // for them; without packing sends only the host half is read, so the look-ahead runs at once
  if (send_packs(d)) {
    HIPCHK(hipEventRecord(e->xplan_join, e->stream));
    HIPCHK(hipStreamWaitEvent(e->xplan_stream, e->xplan_join, 0));
  }
  HIPCHK(hipMemsetAsync(dev, 0, sizeof(uint32_t) * n, e->xplan_stream));
  k_xplan<<<dim3(nblk(d.H, 256), XPLAN_BATCH), 256, 0, e->xplan_stream>>>(d, start, dev);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(e->xplan_host + (size_t)k * n, dev, sizeof(uint32_t) * n, hipMemcpyDeviceToHost,
                        e->xplan_stream));
  HIPCHK(hipEventRecord(e->xplan_ev[k], e->xplan_stream));
  e->xplan_start[k] = start;
  return GX_OK;
}
// The counts of the current round: its batch (computed XPLAN_BATCH rounds ahead, so the wait below
// finds it done except for the first batch) and the next batch queued behind it.
static int xplan_counts(gx_engine *e, const uint32_t **out) {
  Dev &d = e->d;
  if (!e->xplan_dev) {
    if (hipStreamCreateWithFlags(&e->xplan_stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&e->xplan_ev[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->xplan_ev[1], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->xplan_join, hipEventDisableTiming) != hipSuccess ||
        hipMalloc((void **)&e->xplan_dev, sizeof(uint32_t) * 2 * XPLAN_BATCH * d.G * d.G) != hipSuccess ||
        hipHostMalloc((void **)&e->xplan_host, sizeof(uint32_t) * 2 * XPLAN_BATCH * d.G * d.G) != hipSuccess) {
      (void)hipGetLastError();
      return GX_ENOMEM;
    }
  }
  const int64_t start = d.round - d.round % XPLAN_BATCH;
  const int k = (int)((start / XPLAN_BATCH) & 1);
  int rc = GX_OK;
  if (e->xplan_start[k] != start) rc = xplan_launch(e, k, start);
  if (!rc && e->xplan_start[k ^ 1] != start + XPLAN_BATCH) rc = xplan_launch(e, k ^ 1, start + XPLAN_BATCH);
  if (rc) return rc;
  e->xplan_waits[1]++;
  const hipError_t q = hipEventQuery(e->xplan_ev[k]);
  if (q == hipErrorNotReady) {
    e->xplan_waits[0]++;  // this call blocks the host
    HIPCHK(hipEventSynchronize(e->xplan_ev[k]));
  } else {
    HIPCHK(q);
  }
  const size_t row = ((size_t)k * XPLAN_BATCH + (size_t)(d.round - start)) * d.G * d.G;
  *out = e->xplan_host + row;
  e->xbound_dev = e->xplan_dev + row + (size_t)d.gid * d.G;
  return GX_OK;
}

int gx_exchange_plan(gx_engine *e, uint64_t *sizes) {
  if (!e || !sizes) return GX_EINVAL;
  Dev &d = e->d;
  if (d.p.fd_enable) return GX_ENOSYS;
  if (d.G > XPLAN_GMAX) return GX_EINVAL;
  for (uint32_t i = 0; i < d.G * d.G; i++) sizes[i] = 0;
  if (d.G < 2 || !d.K) return GX_OK;
  HIPCHK(hipSetDevice(e->device));
  const uint32_t *c = nullptr;
  int rc = xplan_counts(e, &c);
  if (rc) return rc;
  for (uint32_t i = 0; i < d.G * d.G; i++) sizes[i] = (uint64_t)c[i] * slot_bytes(d);
  for (uint32_t g = 0; g < XPLAN_GMAX; g++) e->xbound.n[g] = g < d.G ? c[d.gid * d.G + g] : 0u;
  e->xbound_round = d.round;
  return GX_OK;
}

int gx_outbox_pack_planned(gx_engine *e, void *buf, uint64_t cap) {
  if (!e || (cap && !buf)) return GX_EINVAL;
  Dev &d = e->d;
  if (d.p.fd_enable) return GX_ENOSYS;
  if (d.G < 2 || !d.K) return GX_OK;
  if (e->xbound_round != d.round) {  // the plan of this round, if the caller did not ask for it
    std::vector<uint64_t> tmp((size_t)d.G * d.G);
    int rc = gx_exchange_plan(e, tmp.data());
    if (rc) return rc;
  }
  uint64_t slots = 0;
  for (uint32_t g = 0; g < d.G; g++) slots += e->xbound.n[g];
  if (cap < slots * slot_bytes(d)) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  set_round_fields(e);
  const size_t ne = (size_t)d.Hl * d.KE;
  const uint32_t nchunk = (uint32_t)((ne + 255) / 256);
  uint32_t *ccnt = e->ob_counts + d.G, *off = ccnt + (size_t)nchunk * d.G;
  const size_t lds = sizeof(uint32_t) * 4 * d.G;
  k_ob_count<<<nchunk, 256, lds, e->stream>>>(d, ccnt);
  k_ob_scan<<<1, 256, 0, e->stream>>>(d, ccnt, nchunk, off, e->ob_counts);
  k_ob_fill<<<nchunk, 256, lds, e->stream>>>(d, off, e->ob_entries);
  // one block at least: block 0 checks every destination's packets against its plan bound
  k_outbox_pack_planned<<<(unsigned)(slots ? slots : 1), 64, 0, e->stream>>>(d, e->ob_entries, e->ob_counts, e->xbound, (uint8_t *)buf);
  e->n_ob = 0;
  e->ob_async = false;
  return phase_done(e);
}

int gx_inbox_unpack(gx_engine *e, const void *buf, uint64_t bytes) {
  if (!e || (bytes && !buf) || bytes % slot_bytes(e->d)) return GX_EINVAL;
  uint64_t n = bytes / slot_bytes(e->d);
  if (n > (uint64_t)(e->d.H - e->d.Hl) * e->d.KE) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  if (n) k_inbox_unpack<<<(unsigned)n, 64, 0, e->stream>>>(e->d, (const uint8_t *)buf, (uint32_t)n);
  e->d.n_remote = (uint32_t)n;
  return phase_done(e);
}

int gx_round_merge(gx_engine *e) {
  if (!e) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  int rc = round_merge_impl(e);
  return rc ? rc : phase_done(e);
}

// Push-pull plan of this round (host side): global pairs t -> (a, b); local pairs, rows to send
// (grouped by destination shard, ascending t) and rows to receive (by source shard, ascending t).
static int ae_plan(gx_engine *e, uint64_t *bytes) {
  Dev &d = e->d;
  set_round_fields(e);
  std::vector<uint32_t> pa, pb;
  uint32_t groups[2][2];
  int ng;
  if (d.pair_split) {
    groups[0][0] = 0; groups[0][1] = d.H / 2;
    groups[1][0] = d.H / 2; groups[1][1] = d.H - d.H / 2;
    ng = 2;
  } else {
    groups[0][0] = 0; groups[0][1] = d.H;
    ng = 1;
  }
  // the pair schedule (Feistel permutations, as k_ae draws it) on the device, read back once
  uint32_t n0 = groups[0][1] / 2, n1 = ng > 1 ? groups[1][1] / 2 : 0, np = n0 + n1;
  uint64_t key0 = rng4(d.p.seed, ST_AE, (uint64_t)d.round, groups[0][0], 0);
  uint64_t key1 = ng > 1 ? rng4(d.p.seed, ST_AE, (uint64_t)d.round, groups[1][0], 0) : 0;
  pa.resize(np);
  pb.resize(np);
  if (np) {
    k_ae_pairs<<<(np + 255) / 256, 256, 0, e->stream>>>(groups[0][0], groups[0][1], key0, groups[1][0],
                                                         ng > 1 ? groups[1][1] : 0, key1, n0, np, e->ae_pa, e->ae_pb);
    HIPCHK(hipMemcpyAsync(pa.data(), e->ae_pa, 4ull * np, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(pb.data(), e->ae_pb, 4ull * np, hipMemcpyDeviceToHost, e->stream));
    int rc = sync_check(e);
    if (rc) return rc;
  }
  // a pair with a crashed member does not run (both shards skip it alike; pair indices unchanged)
  std::vector<uint8_t> runs(pa.size(), 1);
  if (d.departures)
    for (size_t t = 0; t < pa.size(); t++)
      runs[t] = !departed_at(d.p, d.round, pa[t]) && !departed_at(d.p, d.round, pb[t]);
  // one pass over the pairs: cross pairs bucketed by the partner's shard (messages go out and
  // come in grouped by shard, ascending t, so cross pair k has the same index both ways), then
  // the pairs with both hosts here
  std::vector<std::vector<uint32_t>> by_g(d.G);
  std::vector<uint32_t> local_t;
  for (size_t t = 0; t < pa.size(); t++) {
    if (!runs[t]) continue;
    bool la = own(e, pa[t]), lb = own(e, pb[t]);
    if (la && lb) local_t.push_back((uint32_t)t);
    else if (la != lb) by_g[shard_of(d, la ? pb[t] : pa[t])].push_back((uint32_t)t);
  }
  std::vector<uint32_t> plan_a, plan_b, pack_host, pack_t, pack_other;
  std::vector<uint8_t> pack_first;
  std::vector<int32_t> plan_row;
  std::vector<uint8_t> plan_cnt;
  for (uint32_t g = 0; g < d.G; g++) bytes[g] = 0;
  e->pack_gstart.assign(d.G + 1, 0);
  int32_t row = 0;
  for (uint32_t g = 0; g < d.G; g++) {
    e->pack_gstart[g] = (uint32_t)pack_host.size();
    for (uint32_t t : by_g[g]) {
      bool la = own(e, pa[t]);
      uint32_t mine = la ? pa[t] : pb[t], other = la ? pb[t] : pa[t];
      pack_host.push_back(mine);
      pack_t.push_back(t);
      pack_other.push_back(other);
      pack_first.push_back(la ? 1 : 0);
      bytes[g] += dig_bytes(e);
      plan_a.push_back(mine);
      plan_b.push_back(other);
      plan_row.push_back(row++);
      plan_cnt.push_back(la ? 1 : 0);
    }
  }
  e->pack_gstart[d.G] = (uint32_t)pack_host.size();
  for (uint32_t t : local_t) {
    plan_a.push_back(pa[t]);
    plan_b.push_back(pb[t]);
    plan_row.push_back(-1);
    plan_cnt.push_back(0);
  }
  e->n_plan = (uint32_t)plan_a.size();
  e->n_plan_rows = (uint32_t)row;
  e->n_pack = (uint32_t)pack_host.size();
  if (e->n_plan) {
    HIPCHK(hipMemcpy(e->ae_pa, plan_a.data(), 4 * e->n_plan, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->ae_pb, plan_b.data(), 4 * e->n_plan, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->ae_prow, plan_row.data(), 4 * e->n_plan, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->ae_pcount, plan_cnt.data(), e->n_plan, hipMemcpyHostToDevice));
  }
  if (e->n_pack) {
    HIPCHK(hipMemcpy(e->ae_pack_host, pack_host.data(), 4 * e->n_pack, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->ae_pack_t, pack_t.data(), 4 * e->n_pack, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->ae_pack_other, pack_other.data(), 4 * e->n_pack, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->ae_pack_first, pack_first.data(), e->n_pack, hipMemcpyHostToDevice));
    HIPCHK(hipMemsetAsync(e->ae_skip, 0, e->n_pack, e->stream));
  }
  if (pp_state(d)) k_fd_snap<<<2048, 256, 0, e->stream>>>(d);  // round-start member lists (pushPull)
  e->ae_planned_round = (int)d.round;
  return GX_OK;
}

int gx_ae_bytes(gx_engine *e, uint64_t *bytes) {
  if (!e || !bytes) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  for (uint32_t g = 0; g < e->d.G; g++) bytes[g] = 0;
  e->n_plan = e->n_pack = e->n_plan_rows = 0;
  e->ae_planned_round = -1;
  if (e->d.G < 2 || !ae_round(e)) return GX_OK;
  return ae_plan(e, bytes);
}

int gx_ae_pack(gx_engine *e, void *buf, uint64_t cap) {
  if (!e || (cap && !buf)) return GX_EINVAL;
  if (!e->n_pack) return GX_OK;
  if (e->ae_planned_round != (int)e->d.round || cap < e->n_pack * dig_bytes(e)) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  if (e->d.R % 2 == 0)
    k_ae_digest<true><<<e->n_pack, 256, 0, e->stream>>>(e->d, e->ae_pack_host, e->ae_pack_t, e->ae_pack_other,
                                                         e->ae_pack_first, (uint8_t *)buf,
                                                         e->ae_dig, e->nblk, e->ae_bcnt);
  else
    k_ae_digest<false><<<e->n_pack, 256, 0, e->stream>>>(e->d, e->ae_pack_host, e->ae_pack_t, e->ae_pack_other,
                                                          e->ae_pack_first, (uint8_t *)buf,
                                                          e->ae_dig, e->nblk, e->ae_bcnt);
  return phase_done(e);
}

// Received digests -> differing blocks and who leads each; lead message sizes per shard, and the
// offsets of this side's lead messages and of the partner's in the lead inbox.
int gx_ae_delta_bytes(gx_engine *e, const void *digests, uint64_t bytes, uint64_t *out) {
  if (!e || !out || (bytes && !digests)) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  Dev &d = e->d;
  for (uint32_t g = 0; g < d.G; g++) out[g] = 0;
  e->ae_delta_round = e->ae_ret_round = -1;
  e->delta_total = e->lead_in_total = 0;
  if (d.G < 2 || !ae_round(e)) return bytes ? GX_EINVAL : GX_OK;
  if (e->ae_planned_round != (int)d.round || bytes != e->n_pack * dig_bytes(e)) return GX_EINVAL;
  const uint32_t np = e->n_pack;
  std::vector<uint64_t> sz(2 * (size_t)np);
  if (np) {
    HIPCHK(hipMemsetAsync(e->ae_err, 0, sizeof(uint32_t), e->stream));
    k_ae_mask<<<np, 256, 0, e->stream>>>(d, (const uint8_t *)digests, e->ae_dig, e->ae_pack_t, e->ae_pack_host,
                                         e->ae_pack_other, e->ae_pack_first, e->nblk, e->nmw, e->ae_mask,
                                         e->ae_fmask, e->ae_lt, e->ae_cnt, e->ae_nfol, e->ae_sz, e->ae_sz + np,
                                         e->ae_err, e->ae_skip);
    if (pp_state(d))  // the partners' member lists ride with their digests
      k_fd_rsnap<<<1024, 256, 0, e->stream>>>(d, (const uint8_t *)digests, dig_bytes(e), e->nblk, np, e->fd_rsnap);
    uint32_t err = 0;
    HIPCHK(hipMemcpyAsync(&err, e->ae_err, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(sz.data(), e->ae_sz, sizeof(uint64_t) * 2 * np, hipMemcpyDeviceToHost, e->stream));
    int rc = sync_main(e);
    if (rc) return rc;
    if (err) return GX_EINVAL;  // digests of another pair or another row size
  }
  e->delta_off_h.assign(2 * (size_t)np, 0);
  uint64_t o = 0, oi = 0;
  for (uint32_t g = 0; g < d.G; g++)
    for (uint32_t k = e->pack_gstart[g]; k < e->pack_gstart[g + 1]; k++) {
      e->delta_off_h[k] = o;
      e->delta_off_h[np + k] = oi;
      out[g] += sz[k];
      o += sz[k];
      oi += sz[np + k];
    }
  e->delta_total = o;
  e->lead_in_total = oi;
  if (np) HIPCHK(hipMemcpy(e->ae_off, e->delta_off_h.data(), sizeof(uint64_t) * 2 * np, hipMemcpyHostToDevice));
  e->ae_delta_round = (int)d.round;
  return GX_OK;
}

int gx_ae_delta_pack(gx_engine *e, void *buf, uint64_t cap) {
  if (!e || (cap && !buf)) return GX_EINVAL;
  if (!e->n_pack) return GX_OK;
  if (e->ae_delta_round != (int)e->d.round || cap < e->delta_total) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  if (e->nblk <= XS_MAXB)  // offsets up front, a wave per block (profiles/ab_shard_ae.sh)
    k_ae_lead_pack_w<<<e->n_pack, 256, 0, e->stream>>>(e->d, e->ae_pack_host, e->ae_pack_t, e->ae_mask, e->ae_cnt,
                                                        e->ae_off, e->nmw, (const ulonglong2 *)e->ae_dig, e->nblk,
                                                        (uint8_t *)buf);
  else
    k_ae_lead_pack<<<e->n_pack, 256, 0, e->stream>>>(e->d, e->ae_pack_host, e->ae_pack_t, e->ae_mask, e->ae_cnt,
                                                      e->ae_off, e->nmw, (uint8_t *)buf);
  return phase_done(e);
}

// Received lead blocks -> return message sizes: per destination shard a u64 size table, then the
// messages (gx.h "return").
int gx_ae_return_bytes(gx_engine *e, const void *lead, uint64_t lead_bytes, uint64_t *out) {
  if (!e || !out || (lead_bytes && !lead)) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  Dev &d = e->d;
  for (uint32_t g = 0; g < d.G; g++) out[g] = 0;
  e->ae_ret_round = -1;
  e->ret_total = 0;
  const uint32_t np = e->n_pack;
  if (d.G < 2 || !ae_round(e) || !np) return lead_bytes ? GX_EINVAL : GX_OK;
  if (e->ae_delta_round != (int)d.round || lead_bytes != e->lead_in_total) return GX_EINVAL;
  if (e->nblk <= XS_MAXB)
    k_ae_ret_w<true><<<np, 256, 0, e->stream>>>(d, e->ae_pack_host, e->ae_pack_t, e->ae_fmask, e->ae_nfol, e->ae_lt,
                                                (const uint8_t *)lead, e->ae_off + np, e->nblk, e->nmw,
                                                e->ae_sz + 2 * np, nullptr, nullptr, nullptr, e->ae_retL);
  else
    k_ae_ret<true><<<np, 256, 0, e->stream>>>(d, e->ae_pack_host, e->ae_pack_t, e->ae_fmask, e->ae_nfol, e->ae_lt,
                                              (const uint8_t *)lead, e->ae_off + np, e->nblk, e->nmw,
                                              e->ae_sz + 2 * np, nullptr, nullptr, nullptr);
  std::vector<uint64_t> rsz(np);
  HIPCHK(hipMemcpyAsync(rsz.data(), e->ae_sz + 2 * np, sizeof(uint64_t) * np, hipMemcpyDeviceToHost, e->stream));
  int rc = sync_main(e);
  if (rc) return rc;
  std::vector<uint64_t> off(2 * (size_t)np);  // message offsets, size-table entry offsets
  uint64_t o = 0;
  for (uint32_t g = 0; g < d.G; g++) {
    uint32_t k0 = e->pack_gstart[g], k1 = e->pack_gstart[g + 1];
    uint64_t seg = o;
    o += 8ull * (k1 - k0);
    for (uint32_t k = k0; k < k1; k++) {
      off[np + k] = seg + 8ull * (k - k0);
      off[k] = o;
      o += rsz[k];
    }
    out[g] = o - seg;
  }
  e->ret_total = o;
  HIPCHK(hipMemcpy(e->ae_off + 2 * np, off.data(), sizeof(uint64_t) * 2 * np, hipMemcpyHostToDevice));
  e->ae_ret_round = (int)d.round;
  return GX_OK;
}

int gx_ae_return_pack(gx_engine *e, const void *lead, uint64_t lead_bytes, void *buf, uint64_t cap) {
  if (!e || (cap && !buf) || (lead_bytes && !lead)) return GX_EINVAL;
  const uint32_t np = e->n_pack;
  if (!np) return GX_OK;
  if (e->ae_ret_round != (int)e->d.round || cap < e->ret_total || lead_bytes != e->lead_in_total) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  if (e->nblk <= XS_MAXB)
    k_ae_ret_w<false><<<np, 256, 0, e->stream>>>(e->d, e->ae_pack_host, e->ae_pack_t, e->ae_fmask, e->ae_nfol,
                                                 e->ae_lt, (const uint8_t *)lead, e->ae_off + np, e->nblk, e->nmw,
                                                 e->ae_sz + 2 * np, e->ae_off + 2 * np, e->ae_off + 3 * np,
                                                 (uint8_t *)buf, e->ae_retL);
  else
    k_ae_ret<false><<<np, 256, 0, e->stream>>>(e->d, e->ae_pack_host, e->ae_pack_t, e->ae_fmask, e->ae_nfol, e->ae_lt,
                                               (const uint8_t *)lead, e->ae_off + np, e->nblk, e->nmw,
                                               e->ae_sz + 2 * np, e->ae_off + 2 * np, e->ae_off + 3 * np,
                                               (uint8_t *)buf);
  return phase_done(e);
}

// Launch the planned pairs [lo, hi) (received-row pairs first, then shard-local pairs).
static void ae_plan_launch(gx_engine *e, uint32_t lo, uint32_t hi, const void *lead, const void *ret,
                           hipStream_t st = nullptr) {
  if (hi <= lo) return;
  if (!st) st = e->stream;
  set_round_fields(e);
  LaunchTimer t(e, GX_K_AE, st);
  const uint32_t np = e->n_pack;
  AeIn in;
  in.lead = (const uint8_t *)lead;
  in.ret = (const uint8_t *)ret;
  in.ioff = e->ae_off + np;
  in.rioff = e->ae_rioff;
  in.lmask = e->ae_mask;
  in.fmask = e->ae_fmask;
  in.lt = e->ae_lt;
  in.nlead = e->ae_cnt;
  in.bcnt = e->ae_bcnt;
  in.nmw = e->nmw;
  in.nblk = e->nblk;
  // fewer than 4 pairs per CU: per-block bandwidth decides (2 tiles in flight measured slower for
  // the cross pairs of a post-heal round: 8.2 -> 9.3 ms at G = 2, H = 16384)
  const bool small = hi - lo < 1024;
#define GX_AE_PLAN(V, E)                                                                                     \
  (E ? k_ae_plan_ev<V> : small ? k_ae_plan_pf2<V> : k_ae_plan<V>)<<<hi - lo, 256, 0, st>>>(                    \
      e->d, e->ae_pa + lo, e->ae_pb + lo, e->ae_prow + lo, e->ae_pcount + lo, in, e->ae_skip)
  const bool ev = !e->log_views.empty();
  if (e->d.R % 2 == 0 && !ev) GX_AE_PLAN(true, false);
  else if (e->d.R % 2 == 0) GX_AE_PLAN(true, true);
  else if (!ev) GX_AE_PLAN(false, false);
  else GX_AE_PLAN(false, true);
#undef GX_AE_PLAN
}

int gx_ae_merge_local(gx_engine *e) {
  if (!e) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  if (!ae_round(e) || e->d.G < 2 || e->ae_local_round == e->d.round) return GX_OK;
  if (e->ae_planned_round != (int)e->d.round) return GX_EINVAL;
  // on the side stream, after the rows are packed: the exchange layer's collectives (ordered
  // behind `stream`) run while these merges do; gx_ae_merge joins them back
  HIPCHK(hipEventRecord(e->side_start, e->stream));
  HIPCHK(hipStreamWaitEvent(e->side_stream, e->side_start, 0));
  ae_plan_launch(e, e->n_plan_rows, e->n_plan, nullptr, nullptr, e->side_stream);
  HIPCHK(hipEventRecord(e->side_done, e->side_stream));
  e->side_pending = true;
  HIPCHK(hipGetLastError());
  e->ae_local_round = e->d.round;
  return GX_OK;
}

int gx_ae_merge(gx_engine *e, const void *lead, uint64_t lead_bytes, const void *ret, uint64_t ret_bytes) {
  if (!e || (lead_bytes && !lead) || (ret_bytes && !ret)) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  if (!ae_round(e)) return GX_OK;
  if (e->d.G < 2) {
    int rc = ae_whole_impl(e);
    return rc ? rc : sync_check(e);
  }
  if (e->ae_planned_round != (int)e->d.round) return GX_EINVAL;
  const uint32_t np = e->n_pack;
  if (np) {
    if (e->ae_ret_round != (int)e->d.round || lead_bytes != e->lead_in_total) return GX_EINVAL;
    // the return inbox: per source shard a size table, then that shard's messages
    std::vector<uint64_t> rio(np), tab;
    uint64_t o = 0;
    for (uint32_t g = 0; g < e->d.G; g++) {
      uint32_t k0 = e->pack_gstart[g], k1 = e->pack_gstart[g + 1];
      if (k1 == k0) continue;
      if (o + 8ull * (k1 - k0) > ret_bytes) return GX_EINVAL;
      tab.resize(k1 - k0);
      HIPCHK(hipMemcpyAsync(tab.data(), (const uint8_t *)ret + o, 8ull * (k1 - k0), hipMemcpyDeviceToHost, e->stream));
      HIPCHK(hipStreamSynchronize(e->stream));
      o += 8ull * (k1 - k0);
      for (uint32_t k = k0; k < k1; k++) {
        rio[k] = o;
        o += tab[k - k0];
      }
    }
    if (o != ret_bytes) return GX_EINVAL;
    HIPCHK(hipMemcpy(e->ae_rioff, rio.data(), sizeof(uint64_t) * np, hipMemcpyHostToDevice));
  }
  bool local_done = e->ae_local_round == e->d.round;
  ae_plan_launch(e, 0, local_done ? e->n_plan_rows : e->n_plan, lead, ret);
  if (pp_state(e->d) && e->n_plan) {  // pushPull's membership half, every planned pair
    LaunchTimer t(e, GX_K_FD);
    k_fd_pushpull_plan<<<2 * e->n_plan, 64, 0, e->stream>>>(e->d, e->ae_pa, e->ae_pb, e->ae_prow, e->ae_skip,
                                                             e->fd_rsnap);
  }
  int jr = join_side(e);  // the next round's phases see the local pairs merged
  if (jr) return jr;
  return phase_done(e);
}

int gx_lock_census(gx_engine *e, uint32_t *unlocked) {
  if (!e || !unlocked) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  int rc = ensure_api(e, sizeof(uint32_t));
  if (rc) return rc;
  set_round_fields(e);
  uint32_t *dv = (uint32_t *)e->api_dev;
  HIPCHK(hipMemsetAsync(dv, 0, sizeof(uint32_t), e->stream));
  if (e->d.Hl) k_lock_census<<<nblk(e->d.Hl, 256), 256, 0, e->stream>>>(e->d, dv);
  HIPCHK(hipMemcpyAsync(unlocked, dv, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  return sync_check(e);
}

// A push-pull round in which every host of the cluster holds the lock (the caller's collective
// census): every pair fails, so the round is only its counts, as the full exchange would make them
// (gx_ae_bytes .. gx_ae_merge): ae_locked once per pair, by the shard of its first host.
int gx_ae_skip_locked(gx_engine *e) {
  if (!e) return GX_EINVAL;
  Dev &d = e->d;
  if (!ae_round(e)) return GX_OK;
  // sharded engines only (one engine runs its push-pull itself; the pair buffers exist when G > 1)
  if (d.G < 2 || !e->ae_pa || !d.p.lock_model || d.departures || d.p.fd_enable) return GX_EINVAL;
  uint32_t unlocked = 0;
  int rc = gx_lock_census(e, &unlocked);
  if (rc) return rc;
  if (unlocked) return GX_EINVAL;  // a host here is free: the pairs must run the exchange
  set_round_fields(e);
  uint32_t base[2] = {0, d.H / 2}, len[2] = {d.H, 0};
  int ng = 1;
  if (d.pair_split) {
    len[0] = d.H / 2;
    len[1] = d.H - d.H / 2;
    ng = 2;
  }
  const uint32_t n0 = len[0] / 2, n1 = ng > 1 ? len[1] / 2 : 0, np = n0 + n1;
  if (!np) return GX_OK;
  const uint64_t key0 = rng4(d.p.seed, ST_AE, (uint64_t)d.round, base[0], 0);
  const uint64_t key1 = ng > 1 ? rng4(d.p.seed, ST_AE, (uint64_t)d.round, base[1], 0) : 0;
  std::vector<uint32_t> pa(np), pb(np);
  k_ae_pairs<<<(np + 255) / 256, 256, 0, e->stream>>>(base[0], len[0], key0, base[1], ng > 1 ? len[1] : 0, key1, n0,
                                                       np, e->ae_pa, e->ae_pb);
  HIPCHK(hipMemcpyAsync(pa.data(), e->ae_pa, 4ull * np, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(pb.data(), e->ae_pb, 4ull * np, hipMemcpyDeviceToHost, e->stream));
  rc = sync_check(e);
  if (rc) return rc;
  uint32_t n_first = 0, any = 0;
  for (uint32_t t = 0; t < np; t++) {
    const bool la = own(e, pa[t]), lb = own(e, pb[t]);
    n_first += la ? 1u : 0u;
    any |= (la || lb) ? 1u : 0u;
  }
  k_ae_locked_note<<<1, 64, 0, e->stream>>>(d, n_first, any);
  return phase_done(e);
}

int gx_round_end(gx_engine *e) {
  if (!e || e->d.round + 1 >= GX_MAX_ROUND) return GX_EINVAL;  // rounds are 32-bit in jobs and sleepers
  HIPCHK(hipSetDevice(e->device));
  int rc = join_side(e);
  if (rc) return rc;
  e->d.round++;
  rc = wake_all(e);
  return rc ? rc : phase_done(e);
}

// A round whose k_send packs the planned exchange itself (Dev::ob_buf): send_planned's rounds
// (round_send_impl's `plan`) with one message per target.
static bool send_packs(const Dev &d) {
  return d.G >= 2 && d.K && d.NG == 1 && !d.p.limit_bytes && d.p.retransmit_rounds > 0 && !d.departures &&
         !d.p.fd_enable;
}

int gx_round_gossip_begin(gx_engine *e, uint64_t *plan, void *buf, uint64_t cap) {
  if (!e || !plan || (cap && !buf)) return GX_EINVAL;
  Dev &d = e->d;
  if (!send_packs(d)) {
    int rc = gx_round_send(e);
    if (!rc) rc = gx_exchange_plan(e, plan);
    if (!rc) rc = gx_outbox_pack_planned(e, buf, cap);
    return rc;
  }
  // the plan first (its batch is on the device since the host saw it done), then one launch that
  // sends and writes every slot of the buffer
  int rc = gx_exchange_plan(e, plan);
  if (rc) return rc;
  uint64_t slots = 0;
  for (uint32_t g = 0; g < d.G; g++) slots += e->xbound.n[g];
  if (cap < slots * slot_bytes(d)) return GX_EINVAL;
  d.ob_buf = (uint8_t *)buf;
  d.ob_cnt = e->xbound_dev;
  d.ob_claim = e->ob_claim;
  rc = gx_round_send(e);
  d.ob_buf = nullptr;
  d.ob_cnt = nullptr;
  d.ob_claim = nullptr;
  e->n_ob = 0;
  e->ob_async = false;
  return rc;
}

int gx_round_gossip_end(gx_engine *e, const void *buf, uint64_t bytes, int *ae) {
  if (!e || !ae) return GX_EINVAL;
  int rc = gx_inbox_unpack(e, buf, bytes);
  if (!rc) rc = gx_round_merge(e);
  if (rc) return rc;
  *ae = ae_round(e) ? 1 : 0;
  return *ae ? GX_OK : gx_round_end(e);
}

int gx_owner_words(gx_engine *e, uint64_t *out) {
  if (!e || !out) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  k_owner_words<<<nblk(e->d.R, 256), 256, 0, e->stream>>>(e->d, out);
  return sync_check(e);
}

int gx_view_minmax(gx_engine *e, uint64_t *mn, uint64_t *mx) {
  if (!e || !mn || !mx) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  k_view_minmax<<<nblk(e->d.R, 256), 256, 0, e->stream>>>(e->d, mn, mx);
  return sync_check(e);
}

static int read_ctr(gx_engine *e, unsigned long long *c, unsigned long long *last_p1, unsigned long long *bytes,
                    unsigned long long *units, unsigned long long *first_drop = nullptr,
                    unsigned long long *first_locked = nullptr) {
  std::vector<DevCtr> tmp(1);
  HIPCHK(hipMemcpyAsync(tmp.data(), e->d.ctr, sizeof(DevCtr), hipMemcpyDeviceToHost, e->stream));
  int rc = sync_check(e);
  if (rc) return rc;
  const DevCtr &x = tmp[0];
  for (int i = 0; i < GX_NCTR_SLOTS; i++) c[i] = 0;
  for (int i = 0; i < 16; i++) bytes[i] = units[i] = 0;
  *last_p1 = 0;
  if (first_drop) *first_drop = ~0ull;
  if (first_locked) *first_locked = ~0ull;
  for (int s = 0; s < GX_SHARDS; s++) {
    if (first_drop && x.first_drop[s][0] < *first_drop) *first_drop = x.first_drop[s][0];
    if (first_locked && x.first_drop[s][1] < *first_locked) *first_locked = x.first_drop[s][1];
    for (int i = 0; i < GX_NCTR_SLOTS; i++) c[i] += x.c[s][i];
    for (int i = 0; i < 16; i++) {
      bytes[i] += x.bytes[s][i];
      units[i] += x.units[s][i];
    }
    if (x.last_change_p1[s][0] > *last_p1) *last_p1 = x.last_change_p1[s][0];
  }
  return GX_OK;
}

int gx_stats_get(gx_engine *e, gx_stats *out) {
  if (!e || !out) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  unsigned long long c[GX_NCTR_SLOTS], lp1, bytes[16], units[16], fdr, flr;
  int rc = read_ctr(e, c, &lp1, bytes, units, &fdr, &flr);
  if (rc) return rc;
  memset(out, 0, sizeof(*out));
  out->queue_deferred = c[C_QDEFER];
  out->locked_merges = c[C_LOCKED_MERGES];
  out->first_locked_round = flr == ~0ull ? -1 : (int64_t)flr;
  out->lock_buffered = c[C_LOCK_BUF];
  out->lock_drops = c[C_LOCK_DROP];
  out->lock_drained = c[C_LOCK_DRAIN];
  out->ae_locked = c[C_AE_LOCKED];
  out->expire_deferred = c[C_EXP_DEFER];
  out->ae_deferred = c[C_AE_DEFER];
  out->ae_defer_lost = c[C_AE_DEFER_LOST];
  out->fd_handoff_queued = c[C_FD_HQ];
  out->fd_handoff_drops = c[C_FD_HQ_DROP];
  out->false_expiries = c[C_FEXP];
  out->first_drop_round = fdr == ~0ull ? -1 : (int64_t)fdr;
  out->lost_packets = c[C_LOST];
  out->fd_probes = c[C_FD_PROBES];
  out->fd_probe_failures = c[C_FD_PROBE_FAIL];
  out->fd_suspicions = c[C_FD_SUSPECT];
  out->fd_confirmations = c[C_FD_CONFIRM];
  out->fd_deaths = c[C_FD_DEATH];
  out->fd_refutes = c[C_FD_REFUTE];
  out->fd_alive_updates = c[C_FD_ALIVE];
  out->fd_msgs_sent = c[C_FD_SENT];
  out->fd_msgs_received = c[C_FD_RECV];
  out->fd_state_merges = c[C_FD_STATE_MERGE];
  out->round = e->d.round;
  out->gossip_merges = c[C_GOSSIP_MERGES];
  out->ae_merges = c[C_AE_MERGES];
  out->local_merges = c[C_LOCAL_MERGES];
  out->gossip_accepts = c[C_GOSSIP_ACC];
  out->ae_accepts = c[C_AE_ACC];
  out->local_accepts = c[C_LOCAL_ACC];
  out->stale_drops = c[C_STALE];
  out->retransmits = c[C_RETX];
  out->queue_drops = c[C_QDROP];
  out->list_drops = c[C_LDROP];
  out->sleep_drops = c[C_SDROP];
  out->pending_drops = c[C_PDROP];
  out->dequeues = c[C_DEQ];
  out->nil_batches = c[C_NIL];
  out->packets = c[C_PACKETS];
  out->records_sent = c[C_RECSENT];
  out->expired = c[C_EXPIRED];
  out->gc = c[C_GC];
  out->own_tombstones = c[C_OWNTOMB];
  out->expire_server = c[C_EXPSRV];
  out->send_jobs = c[C_SENDJOBS];
  out->ae_exchanges = c[C_AEX];
  out->churn_events = c[C_CHURN];
  out->change_events = c[C_CHG];
  out->listener_drops = e->listener_drops;
  out->bytes_sent = c[C_BYTESENT];
  out->cap_cuts = c[C_CAPCUT];
  out->scan_slots = c[C_SCANSLOTS];
  out->ae_slots = c[C_AESLOTS];
  out->last_change_round = (int64_t)lp1 - 1;
  return GX_OK;
}

int gx_timing_get(gx_engine *e, gx_timing *out) {
  if (!e || !out) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  int rc = drain_timing(e);
  if (rc) return rc;
  unsigned long long c[GX_NCTR_SLOTS], lp1, bytes[16], units[16];
  rc = read_ctr(e, c, &lp1, bytes, units);
  if (rc) return rc;
  memset(out, 0, sizeof(*out));
  for (int i = 0; i < GX_K_COUNT; i++) {
    out->ms[i] = e->ms[i];
    out->launches[i] = e->launches[i];
    const bool host = i == GX_K_ENCODE || i == GX_K_DECODE;  // codec classes: accounted on the host
    out->bytes[i] = host ? e->host_bytes[i] : bytes[i];
    out->units[i] = host ? e->host_units[i] : units[i];
  }
  return GX_OK;
}

// ------------------------------------------------------- memberlist failure detection ----
static bool fd_ok(const gx_engine *e, uint32_t host) { return e && e->d.p.fd_enable && own(e, host); }

int gx_fd_read_members(gx_engine *e, uint32_t host, uint32_t lo, uint32_t hi, gx_member *out) {
  if (!fd_ok(e, host) || lo > hi || hi > e->d.H || (!out && hi > lo)) return GX_EINVAL;
  if (hi == lo) return GX_OK;
  HIPCHK(hipSetDevice(e->device));
  const Dev &d = e->d;
  std::vector<int32_t> dl(hi - lo);
  HIPCHK(hipMemcpyAsync(out, &d.mem[(size_t)(host - d.lo) * d.H + lo], sizeof(gx_member) * (hi - lo),
                        hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(dl.data(), &d.fd_dl[(size_t)(host - d.lo) * d.H + lo], sizeof(int32_t) * (hi - lo),
                        hipMemcpyDeviceToHost, e->stream));
  int rc = sync_check(e);
  if (rc) return rc;
  for (uint32_t i = 0; i < hi - lo; i++) out[i].deadline = dl[i];
  return GX_OK;
}

int gx_fd_read_hosts(gx_engine *e, uint32_t lo, uint32_t hi, gx_fd_host *out) {
  if (!e || !e->d.p.fd_enable || lo > hi || (hi > lo && (!own(e, lo) || !own(e, hi - 1))) || (!out && hi > lo))
    return GX_EINVAL;
  if (hi == lo) return GX_OK;
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipMemcpyAsync(out, &e->d.fdh[lo - e->d.lo], sizeof(gx_fd_host) * (hi - lo), hipMemcpyDeviceToHost,
                        e->stream));
  int rc = sync_check(e);
  if (rc) return rc;
  for (uint32_t v = lo; v < hi; v++) out[v - lo].departed = departed_at(e->d.p, e->d.round, v) ? 1u : 0u;
  return GX_OK;
}

int gx_fd_read_queue(gx_engine *e, uint32_t host, gx_fd_msg *out, uint8_t *transmits, uint32_t cap,
                     uint32_t *n_out) {
  if (!fd_ok(e, host) || !n_out) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  const Dev &d = e->d;
  std::vector<gx_member> row(d.H);
  gx_fd_host h;
  HIPCHK(hipMemcpyAsync(row.data(), &d.mem[(size_t)(host - d.lo) * d.H], sizeof(gx_member) * d.H,
                        hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(&h, &d.fdh[host - d.lo], sizeof(gx_fd_host), hipMemcpyDeviceToHost, e->stream));
  int rc = sync_check(e);
  if (rc) return rc;
  uint32_t n = 0;
  for (uint32_t b = 0; b < d.p.fd_retransmit_limit; b++)
    for (uint32_t m = h.q_head[b]; m != GX_FD_NONE && n <= d.H; m = row[m].q_next) {
      if (n < cap) {
        if (out) {
          gx_fd_msg g = {};
          g.incarnation = row[m].msg_incarnation;
          g.node = (uint16_t)m;
          g.from = row[m].msg_from;
          g.kind = row[m].msg_kind;
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
  if (!fd_ok(e, host) || (!msgs && n)) return GX_EINVAL;
  for (uint32_t i = 0; i < n; i++)
    if (msgs[i].node >= e->d.H || msgs[i].kind > GX_M_DEAD) return GX_EINVAL;
  if (!n) return GX_OK;
  HIPCHK(hipSetDevice(e->device));
  int rc = ensure_api(e, sizeof(gx_fd_msg) * n);
  if (rc) return rc;
  set_round_fields(e);
  HIPCHK(hipMemcpyAsync(e->api_dev, msgs, sizeof(gx_fd_msg) * n, hipMemcpyHostToDevice, e->stream));
  k_fd_api_notify<<<1, 64, 0, e->stream>>>(e->d, host, (const gx_fd_msg *)e->api_dev, n);
  return sync_check(e);
}

int gx_fd_get_broadcasts(gx_engine *e, uint32_t host, uint32_t limit, gx_fd_msg *out, uint32_t *n_out) {
  if (!fd_ok(e, host) || !n_out || limit > 64 || (!out && limit)) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  int rc = ensure_api(e, 64 + sizeof(gx_fd_msg) * 64);
  if (rc) return rc;
  set_round_fields(e);
  uint32_t *dn = (uint32_t *)e->api_dev;
  gx_fd_msg *dm = (gx_fd_msg *)((char *)e->api_dev + 64);
  k_fd_api_getb<<<1, 64, 0, e->stream>>>(e->d, host, limit, dm, dn);
  uint32_t n = 0;
  HIPCHK(hipMemcpyAsync(&n, dn, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  rc = sync_check(e);
  if (rc) return rc;
  if (n) {
    HIPCHK(hipMemcpyAsync(out, dm, sizeof(gx_fd_msg) * n, hipMemcpyDeviceToHost, e->stream));
    rc = sync_check(e);
    if (rc) return rc;
  }
  *n_out = n;
  return GX_OK;
}

int gx_fd_probe(gx_engine *e, uint32_t host, uint32_t *target, int *acked) {
  if (!fd_ok(e, host)) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  int rc = ensure_api(e, 64);
  if (rc) return rc;
  set_round_fields(e);
  k_fd_api_probe<<<1, 64, 0, e->stream>>>(e->d, host, (uint32_t *)e->api_dev);
  uint32_t x[2] = {0, 0};
  HIPCHK(hipMemcpyAsync(x, e->api_dev, sizeof(x), hipMemcpyDeviceToHost, e->stream));
  rc = sync_check(e);
  if (rc) return rc;
  if (target) *target = x[0];
  if (acked) *acked = (int)x[1];
  return GX_OK;
}

int gx_fd_timers(gx_engine *e, uint32_t host) {
  if (!fd_ok(e, host)) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  set_round_fields(e);
  k_fd_api_timers<<<1, 64, 0, e->stream>>>(e->d, host);
  return sync_check(e);
}

int gx_fd_merge_state(gx_engine *e, uint32_t host, const uint64_t *remote) {
  if (!fd_ok(e, host) || !remote) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  int rc = ensure_api(e, sizeof(uint64_t) * e->d.H);
  if (rc) return rc;
  set_round_fields(e);
  HIPCHK(hipMemcpyAsync(e->api_dev, remote, sizeof(uint64_t) * e->d.H, hipMemcpyHostToDevice, e->stream));
  k_fd_api_merge_state<<<1, 64, 0, e->stream>>>(e->d, host, (const uint64_t *)e->api_dev);
  return sync_check(e);
}

int gx_fd_converged(gx_engine *e, int *converged, uint64_t *n_disagree) {
  if (!e || !e->d.p.fd_enable) return GX_EINVAL;
  HIPCHK(hipSetDevice(e->device));
  set_round_fields(e);
  HIPCHK(hipMemsetAsync(e->conv_bad, 0, sizeof(unsigned long long), e->stream));
  k_fd_converged<<<nblk(e->d.H, 256), 256, 0, e->stream>>>(e->d, e->conv_bad);
  unsigned long long bad = 0;
  HIPCHK(hipMemcpyAsync(&bad, e->conv_bad, sizeof(bad), hipMemcpyDeviceToHost, e->stream));
  int rc = sync_check(e);
  if (rc) return rc;
  if (converged) *converged = bad == 0;
  if (n_disagree) *n_disagree = bad;
  return GX_OK;
}

// Diagnostics outside gx.h: out[0] = gx_exchange_plan calls that found their batch of slot bounds
// not computed yet and waited on the host, out[1] = all calls.
int gx_xplan_waits(gx_engine *e, uint64_t *out) {
  if (!e || !out) return GX_EINVAL;
  out[0] = e->xplan_waits[0];
  out[1] = e->xplan_waits[1];
  return GX_OK;
}

// Diagnostics outside gx.h (env GX_KPROF at gx_create): the wall-clock phase marks (100 MHz) of the
// last k_send launch, 8 per wave: start, ticks done, block barrier, sends begin, send_host begin,
// first chunk planned, first chunk's records stored, sends done (0 = not reached).
int gx_kprof_read(gx_engine *e, uint64_t *out, uint64_t cap, uint64_t *n_out) {
  if (!e || !n_out) return GX_EINVAL;
  *n_out = e->kprof_n;
  if (!e->kprof_n || !out) return GX_OK;
  HIPCHK(hipStreamSynchronize(e->stream));
  HIPCHK(hipMemcpy(out, e->d.kprof, sizeof(uint64_t) * (cap < e->kprof_n ? cap : e->kprof_n), hipMemcpyDeviceToHost));
  return GX_OK;
}

int gx_converged(gx_engine *e, int *converged, uint64_t *n_disagree) {
  if (!e || e->d.G > 1) return GX_EINVAL;
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

// full-state JSON codec: gx_set_names, gx_local_state_json, gx_decode_state_json,
// gx_merge_remote_state_json
#include "gx_codec_host.hpp"

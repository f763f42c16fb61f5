/*
 * gx.h — C-ABI of the sidecar-gx gossip-convergence engine (Sidecar catalog merge path).
 *
 * One engine handle simulates a cluster of H hosts x S services. Every host owns one
 * catalog view (the reference's `catalog.ServicesState`, catalog/services_state.go:70-80),
 * its broadcast FIFO (the unbuffered `state.Broadcasts` channel with its blocked senders,
 * services_state.go:94,377-392,579-604) and its memberlist delegate `pendingBroadcasts`
 * (services_delegate.go:20-27). The whole-round driver `gx_run_rounds` advances the
 * simulated cluster one 200 ms gossip round at a time (config/config.go:47).
 *
 * The per-host entry points keep the reference method set so a cgo (or ctypes) binding can
 * expose the same `ServicesState` / `servicesDelegate` API; each declaration cites the
 * reference function it replaces. See INTEGRATION.md for the cgo binding stub.
 *
 * Two implementations export this exact ABI:
 *   sidecar_amd/libgx.so           the product: HIP kernels for gfx950 (MI355X)
 *   oracle/liboracle_gx.so         the CPU restatement used ONLY by tests / bench cpu_baseline
 *
 * Conventions
 *   - All buffers are caller-allocated host memory; the engine never retains a caller pointer
 *     after a call returns (services_delegate.go:131-141 ownership hazard does not exist here).
 *   - Return codes: 0 = OK, negative errno-style on failure (GX_EINVAL, GX_ENOMEM, GX_EIO,
 *     GX_ENOSYS). No C++ exception crosses the ABI. Hot-path drops (stale records, full
 *     queues) are never errors: they are counted in gx_stats (the reference logs and continues,
 *     services_state.go:302-308, services_delegate.go:50-53).
 *   - A handle is NOT thread-safe; callers serialise (the reference's sync.RWMutex,
 *     services_state.go:79). Every call is synchronous at return.
 *   - "now" is the simulated clock: t0_ns + round * round_ns.
 */
#ifndef SIDECAR_GX_H
#define SIDECAR_GX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GX_ABI_VERSION 11

#define GX_OK 0
#define GX_EIO (-5)
#define GX_ENOMEM (-12)
#define GX_EINVAL (-22)
#define GX_ENOSYS (-38)
#define GX_ENOENT (-2)

/* service.Service.Status values, service/service.go:17-23. GX_ABSENT marks an empty slot. */
#define GX_ALIVE 0
#define GX_TOMBSTONE 1
#define GX_UNHEALTHY 2
#define GX_UNKNOWN 3
#define GX_DRAINING 4
#define GX_ABSENT 7

/* A view slot is one packed 64-bit word: ((updated_ns - epoch) << 3) | status, the time relative
 * to the engine epoch (gx_epoch) in [0, 2^61). The epoch centres the 73-year window on t0_ns:
 * epoch = t0_ns - 2^60 rounded down to a whole second, or 0 when t0_ns < 2^60 (the window is then
 * 1970 .. 2043). With t0 in November 2023 the window is May 1987 .. May 2060. Times are clamped
 * into the window where records enter (gx_service inputs, Decode): a time before it stores as
 * the window's start, which IsStale drops for every lifespan (the reference drops such records
 * too: a pre-1970 or zero time.Time Updated is stale); a time after it stores as the window's
 * end, which still wins every merge, as the reference's far-future record does, and reads back
 * as that end. Every gx_service, event and server time handed out is absolute (epoch added back;
 * a server time or state.LastChanged never set reads 0, the reference's time.Unix(0, 0)); the
 * packed words of gx_read_views, gx_read_job and the sharded wire formats are epoch-relative
 * (the shards of a cluster share t0_ns, so its epoch). The empty slot is GX_SLOT_ABSENT. */
#define GX_TS_SHIFT 3
#define GX_SLOT_ABSENT ((uint64_t)GX_ABSENT)
#define GX_TS_LIMIT ((int64_t)1 << 61)
#define GX_SEC_NS 1000000000ll
static inline int64_t gx_epoch_of(int64_t t0_ns) {
  const int64_t half = (int64_t)1 << 60;
  return t0_ns < half ? 0 : (t0_ns - half) / GX_SEC_NS * GX_SEC_NS;
}
/* absolute Unix ns -> epoch-relative slot time, clamped to [0, 2^61) */
static inline int64_t gx_ts_in(int64_t abs_ns, int64_t epoch) {
  if (abs_ns <= epoch) return 0;
  const int64_t d = abs_ns - epoch; /* epoch >= 0: no overflow */
  return d >= GX_TS_LIMIT ? GX_TS_LIMIT - 1 : d;
}

/* Record across the ABI: the fields of service.Service (service/service.go:32-42) that the
 * merge path reads. Hostname and ID strings are interned to (host, svc) indices by the caller;
 * the record key is r = host * S + svc. */
typedef struct gx_service {
  int64_t updated_ns; /* Service.Updated, UTC nanoseconds */
  uint32_t host;      /* Service.Hostname -> owner host index */
  uint16_t svc;       /* Service.ID -> service index within the owner, < S */
  uint8_t status;     /* Service.Status, 0..6 */
  uint8_t flags;      /* reserved, 0 */
} gx_service;

/* Broadcast-queue job descriptor, 16 B (the FIFO's entry; read-back for parity checks).
 *   kind NIL_BS / NIL_BT : the `Broadcasts <- nil` of an idle looper (services_state.go:569,628)
 *   kind RETX            : retransmit of one accepted record (services_state.go:377-392);
 *                          a = packed record word, c = record key r
 *   kind SEND            : SendServices job (services_state.go:579-604); list in the host's
 *                          list arena, c = slot | len << 16
 *   kind EXPIRE          : SendServices job of ExpireServer (services_state.go:150-192);
 *                          a = mask of tombstoned services, c = round of the call (the tombstones'
 *                          Updated is that round's now), owner = the expired host
 *   kind LOST            : a job whose contents the engine did not keep (below); dequeued as an
 *                          empty batch and counted in gx_stats.queue_drops
 * meta = kind | pass << 3 | n_passes << 9 | owner << 15 (GX_JOB_* accessors below).
 *
 * The FIFO holds every job the reference would hold: the reference's queue is unbounded (every
 * blocked sender is a goroutine, services_state.go:94,384-391,581-603), so no job is ever
 * refused. Each host stores the first queue_cap jobs of its queue (the "stored window", which
 * the head dequeues from); a job pushed while the window is full, or behind such a job, is
 * DEFERRED: counted in its place in the queue (fifo_tail) with its contents dropped. A deferred
 * job is reached by GetBroadcasts only after all queue_cap stored jobs in front of it were
 * dequeued, i.e. after at least queue_cap / (fanout * GossipMessages) rounds; until then every
 * observable (every packet, every looper state) is the reference's. The loopers' nil sends are
 * never lost (their positions are kept: nil_pos_bs / nil_pos_bt). A deferred job that reaches the
 * head is dequeued as LOST: gx_stats.queue_drops counts those and first_drop_round holds the
 * round of the first, so a run is faithful to the reference's queue iff queue_drops == 0. A
 * SendServices job whose list does not fit the list arena (list_slots) is queued as LOST. */
#define GX_JOB_NIL_BS 0
#define GX_JOB_NIL_BT 1
#define GX_JOB_RETX 2
#define GX_JOB_SEND 3
#define GX_JOB_EXPIRE 4
#define GX_JOB_LOST 5
/* c of a SendServices job queued past the stored window: it holds no list (only a LOST dequeue
 * could reach it), so nothing is released for it */
#define GX_LIST_NONE 0xffffu
typedef struct gx_job {
  uint64_t a;
  uint32_t c;
  uint32_t meta;
} gx_job;
/* A SendServices pass sleeping TOMBSTONE_RETRANSMIT before it re-enters the FIFO tail. */
typedef struct gx_sleeper {
  gx_job job;
  uint32_t wake; /* round the pass re-enters the FIFO */
  uint32_t pad[3];
} gx_sleeper;
#define GX_JOB_MAX_PASSES 63u   /* n_passes field: 6 bits (alive_count, tombstone_count <= 63) */
#define GX_MAX_HOSTS (1u << 17) /* owner field: 17 bits */
#define GX_MAX_LIST_SLOTS 1024u
#define GX_MAX_ROUND ((int64_t)1 << 31) /* rounds are 32-bit in jobs and sleepers (2^31 x 200 ms = 13 years) */
#define GX_JOB_KIND(m) ((m) & 7u)
#define GX_JOB_PASS(m) (((m) >> 3) & 63u)
#define GX_JOB_NPASSES(m) (((m) >> 9) & 63u)
#define GX_JOB_OWNER(m) ((m) >> 15)
#define GX_JOB_META(kind, pass, n_passes, owner) \
  ((uint32_t)(kind) | (uint32_t)(pass) << 3 | (uint32_t)(n_passes) << 9 | (uint32_t)(owner) << 15)

/* Engine parameters. gx_params_default() fills the reference constants. */
#define GX_INIT_EMPTY 0 /* no view knows anything; owners announce at their first tick */
#define GX_INIT_OWN 1   /* each view holds only its own S records (ALIVE, ts = t0 - U[0,1s)) */
#define GX_INIT_WARM 2  /* every view holds every record (a converged catalog) */
typedef struct gx_params {
  uint32_t n_hosts;                   /* H */
  uint32_t n_services;                /* S, 1..64 */
  uint32_t fanout;                    /* k: peers per gossip round (memberlist GossipNodes, LAN 3) */
  uint32_t packet_cap;                /* records per GetBroadcasts packet (broadcast cap, 32) */
  uint32_t pending_cap;               /* MAX_PENDING_LENGTH, services_delegate.go:17 (100) */
  uint32_t queue_cap;                 /* Q: stored FIFO jobs per host (the stored window, see gx_job) */
  uint32_t list_slots;                /* A: live SendServices lists per host (engine bound, <= 1024) */
  uint32_t gossip_stop_on_empty;      /* memberlist gossip(): stop the round at the first empty packet */
  uint32_t alive_interval_rounds;     /* ALIVE_SLEEP_INTERVAL 1s = 5 rounds (services_state.go:34) */
  uint32_t tombstone_interval_rounds; /* TOMBSTONE_SLEEP_INTERVAL 2s = 10 rounds (:30) */
  uint32_t retransmit_rounds;         /* TOMBSTONE_RETRANSMIT 1s = 5 rounds (:31) */
  uint32_t alive_count;               /* ALIVE_COUNT 5 (:29) */
  uint32_t tombstone_count;           /* TOMBSTONE_COUNT 10 (:28) */
  uint32_t ae_period_rounds;          /* anti-entropy push-pull period, 0 = off */
  uint32_t ae_phase;                  /* AE rounds are those with round % period == phase */
  uint32_t init_mode;                 /* GX_INIT_* */
  int64_t t0_ns;                      /* simulated clock at round 0, Unix ns in [0, 2^62] */
  int64_t round_ns;                   /* GossipInterval 200ms (config/config.go:47) */
  int64_t alive_lifespan_ns;          /* ALIVE_LIFESPAN 80s (:32) */
  int64_t draining_lifespan_ns;       /* DRAINING_LIFESPAN 10min (:33) */
  int64_t tombstone_lifespan_ns;      /* TOMBSTONE_LIFESPAN 3h (:27) */
  int64_t stale_fudge_ns;             /* IsStale clock-drift fudge 1min (service/service.go:71) */
  int64_t alive_broadcast_interval_ns;/* ALIVE_BROADCAST_INTERVAL 1min (:35) */
  int64_t pass_increment_ns;          /* SendServices +50ns per pass (:599) */
  int64_t tombstone_bump_ns;          /* expired records are tombstoned at Updated+1s (:675) */
  uint64_t seed;                      /* schedule seed (peer sampling, phases, churn, AE pairing) */
  uint32_t churn_ppm;                 /* per owner per round: probability (ppm) of one start/stop */
  uint32_t aged_ppm;                  /* init: fraction (ppm) of records with age U[0, aged_max_ns) */
  int64_t aged_max_ns;
  int32_t partition_start;            /* rounds [start, end): two halves gossip only internally */
  int32_t partition_end;
  int32_t storm_round;                /* round at which every host ExpireServer()s the other half, -1 = none */
  int32_t device;                     /* HIP device ordinal (ignored by the oracle) */
  uint32_t n_shards;                  /* host sharding: 0/1 = this engine owns every host */
  uint32_t shard_id;                  /* this engine owns hosts [id*H/n, (id+1)*H/n) */
  /* Byte-accurate packPacket (services_delegate.go:186-223). limit_bytes = 0 keeps the
   * record-count budget (packet_cap records per GetBroadcasts call, BASELINE "cap 32
   * records/msg"). limit_bytes > 0 is memberlist's GetBroadcasts(overhead, limit): messages are
   * packed while total + len(message) + overhead <= limit, where len(message) is the ffjson
   * encoding length of the record's Service (gx_message_bytes); packet_cap then only bounds the
   * packet buffer (a cut it causes is counted in gx_stats.cap_cuts). memberlist passes limit =
   * UDPBufferSize 1400 - 2 = 1398 and overhead = 2 + 1 = 3. */
  uint32_t limit_bytes;
  uint32_t overhead_bytes;
  /* memberlist failure detection (see "memberlist" below).
   * fd_enable = 0 keeps the scripted model: partitions restrict peer sampling to a side and
   * storm_round scripts NotifyLeave. fd_enable = 1 runs memberlist's SWIM detector on every host:
   * partitions and departures drop packets, and NotifyLeave -> ExpireServer follows the
   * detector's dead declarations. Defaults are DefaultLANConfig (main.go:243); the fields
   * memberlist derives from the cluster size are filled by gx_fd_defaults(). */
  uint32_t fd_enable;
  uint32_t fd_probe_rounds;        /* ProbeInterval 1 s = 5 rounds */
  uint32_t fd_indirect_checks;     /* IndirectChecks 3 */
  uint32_t fd_retransmit_limit;    /* RetransmitMult 4 * ceil(log10(n + 1)), 1..GX_FD_MAX_TX */
  uint32_t fd_msg_cap;             /* memberlist messages per gossip packet, 1..64 */
  uint32_t fd_msg_bytes;           /* byte mode: encoded length of one memberlist message */
  uint32_t fd_gossip_dead_rounds;  /* GossipToTheDeadTime 30 s = 150 rounds */
  uint32_t fd_suspicion_k;         /* SuspicionMult - 2 confirmations (0 when n - 2 < k), <= 2 */
  uint32_t fd_suspicion_rounds[8]; /* suspicion timeout after c confirmations, c = 0..k */
  /* Host departures (crash): from depart_round on, a seeded depart_ppm fraction of the hosts
   * stops every activity and drops every packet sent to it (both models). -1 = none. */
  int32_t depart_round;
  uint32_t depart_ppm;
  /* fd_enable: push-pull also merges memberlist state (state.go mergeState): each side merges the
   * other's round-start member list, alive -> aliveNode, suspect or dead -> suspectNode{From: us}.
   * 1 = memberlist's behaviour (default), 0 = catalog only. */
  uint32_t fd_push_pull_state;
  /* GossipMessages (config/config.go:46, main.go:257-259; README.md:180 "How many times to gather
   * messages per round", Sidecar's default 15): memberlist gathers up to this many GetBroadcasts
   * results per gossip target per round, each sent to that target as its own packet. 0 or 1 = one
   * call per target. With fd_enable, each gather takes memberlist's queued messages first and the
   * delegate's GetBroadcasts the bytes left. The memberlist fork is absent, so this reading is
   * parity unpinned. */
  uint32_t gossip_messages;
  /* Push-pull pairing on anti-entropy rounds (memberlist pushPullTrigger every PushPullInterval,
   * config/config.go:45). GX_PP_MATCHING: a seeded perfect matching, every host in one exchange.
   * GX_PP_INITIATE: every live host initiates one exchange with a peer drawn at random, so a host
   * takes part in 1 + (number of initiators that drew it) exchanges, as with memberlist's
   * per-node timers. Both sides of an exchange merge the other's round-start state. */
  uint32_t push_pull_mode;
  /* Engine bound (no reference counterpart): inbox slots per receiver, 1..256 (0 = 64, or 256 with
   * gossip_messages > 1). A receiver with more packets in a round takes the serial overflow path;
   * results are identical. */
  uint32_t inbox_slots;
  /* The ServicesState lock held by a blocked looper. BroadcastServices holds
   * state.RLock() while it blocks on its `Broadcasts <- nil` (services_state.go:535-536,569) and
   * BroadcastTombstones holds state.Lock() while it blocks on its own (:610-611,628), so while
   * either looper waits for its nil to reach the FIFO head, AddServiceEntry's Lock() (:296),
   * ExpireServer's Lock() (:151) and, behind a pending writer, LocalState's RLock()
   * (services_delegate.go:148) all wait too. lock_model = 1 (default) models it:
   *   - a host is locked for round n iff one of its loopers was blocked on its nil at the start of
   *     round n (gx_host_state.lock holds that snapshot per round parity);
   *   - a looper whose tick finds the other looper holding the lock waits for it: BroadcastServices
   *     does not tick while BroadcastTombstones is blocked, and vice versa;
   *   - gossip records sent to a locked host queue in its inbound pipeline in arrival order:
   *     memberlist's handoff queue (HandoffQueueDepth 1024, config/config.go:48), the packet
   *     handler blocked in NotifyMsg (1), the delegate's notifications channel (25,
   *     services_delegate.go:38), its goroutine blocked in UpdateService (1), ServiceMsgs (25,
   *     services_state.go:97) and ProcessServiceMsgs blocked in AddServiceEntry (1): lock_buffer
   *     records (default 1077). memberlist drops what arrives at a full handoff queue
   *     (gx_stats.lock_drops); the buffered records run through AddServiceEntry, in arrival order,
   *     at the receive phase of the first round the host is unlocked, before that round's packets;
   *   - a push-pull exchange with a locked side does not run (gx_stats.ae_locked): the locked
   *     side's LocalState blocks behind the pending writer past memberlist's TCP deadline;
   *   - ExpireServer calls (the storm's NotifyLeave, the failure detector's deaths) on a locked host
   *     wait: they run in owner order at the end of the owner phase of its first unlocked round.
   * lock_model = 0 lets merges proceed on locked hosts (rounds 1-4) and counts them
   * (gx_stats.locked_merges). lock_buffer is 1..65535. Memory: every engine keeps lock_buffer
   * records of 16 B for each of its hosts (ceil(n_hosts / n_shards)), allocated at create; more
   * than GX_LOCK_BUF_MAX_BYTES of them is GX_EINVAL (the default 1077 at 131072 hosts: 2.3 GB). */
  uint32_t lock_model;
  uint32_t lock_buffer;
  /* memberlist piggybacks the delegate's broadcasts on every UDP message it sends, not only on
   * gossip(): sendMsg -> getBroadcasts (memberlist net.go, the absent fork). probe_piggyback = 1
   * adds the probe traffic of the scripted model (fd_enable = 0) as GetBroadcasts calls: every
   * fd_probe_rounds (ProbeInterval 1 s) at a seeded phase a host pings one target, the target of
   * a keyed Feistel permutation of the hosts for that round (a host drawing itself does not
   * probe), and the ping carries one GetBroadcasts result; a target the ping reaches answers with
   * an ack that carries one GetBroadcasts result of its own. Both calls run before the host's
   * owner phase (ping, then ack), are their own packets (entries K * NG and K * NG + 1 of the host,
   * so a receiver folds them after the sender's gossip packets) and do not stop on an empty
   * result; a ping across the partition or to a departed host is lost after GetBroadcasts took
   * its records, and gets no ack. In byte mode the ping or ack message takes fd_msg_bytes + 2 of
   * limit_bytes. Parity unpinned (the fork is absent); 0 (default) = gossip() only, the rounds 1-5
   * model. Unsharded engines without the failure detector only (GX_EINVAL otherwise). */
  uint32_t probe_piggyback;
  /* GX_PP_INITIATE only: 1 = memberlist's staggered push-pull timers (pushPullTrigger waits a random
   * stagger in [0, PushPullInterval) before its first tick, so the nodes' exchanges spread over the
   * interval instead of all starting together): host i initiates in the rounds with
   * round % ae_period_rounds == its seeded phase, every round being a push-pull round for some
   * hosts. 0 (default) = every live host initiates in the rounds with round % period == ae_phase.
   * Parity unpinned (the fork is absent). memberlist also scales the interval with the cluster
   * size (pushPullScale: x (ceil(log2 n - 5) + 1) above 32 nodes); that is ae_period_rounds. */
  uint32_t push_pull_stagger;
  /* lock_model = 1 only: Go's sync.RWMutex lets LocalState's RLock() (services_delegate.go:148)
   * through while the only holder is BroadcastServices' read lock (services_state.go:535) and no
   * writer waits. lock_readers = 1 models it: a push-pull exchange whose locked sides are all
   * read-locked with no writer waiting runs. A writer waits when the host's inbound pipeline holds
   * a record (ProcessServiceMsgs blocked in AddServiceEntry's Lock()), an ExpireServer call waits, a
   * merge already waits, the BroadcastTombstones tick is due, or BroadcastTombstones held the lock at
   * the start of the round. The unlocked side merges the other's state as usual. The read-locked
   * side's MergeRemoteState cannot merge: its records wait behind the lock
   * (UpdateService -> ServiceMsgs -> AddServiceEntry), taking min(n, 26) of the pipeline's places
   * (ServiceMsgs 25 + the blocked AddServiceEntry), and merge at the start of the receive phase of
   * the host's first unlocked round, before its pipeline (an unpinned order: the reference
   * interleaves the two blocked senders). The engine keeps the partner's pre-exchange state in a
   * pool of lock_defer_slots rows per engine: host v uses slot v % lock_defer_slots. When the slot
   * is taken, the merge is dropped and counted (gx_stats.ae_defer_lost); a run is faithful while
   * that stays 0. Of several hosts claiming one free slot in a round (or push-pull batch), the
   * lowest host id gets it. 0 (default) = every exchange with a locked side fails, the round-5
   * model. Unsharded engines only (GX_EINVAL otherwise). lock_defer_slots: 1..4096 (0 = 64). */
  uint32_t lock_readers;
  uint32_t lock_defer_slots;
  /* lock_model = 1 with fd_enable, unsharded engines: memberlist's own alive / suspect / dead
   * messages share the packet handler's handoff queue with the delegate's user messages (upstream
   * memberlist's net.go handleCommand at the fork's date queues all four kinds on one handoff
   * channel that one packetHandler goroutine drains in order; the fork, github.com/NinesStack/
   * memberlist cfac2b5cf519, is absent, so parity unpinned). While the host's catalog lock blocks
   * NotifyMsg, the handler stops once it holds the 53rd record of the pipeline (1 + notifications 25 +
   * 1 + ServiceMsgs 25 + 1, gx.h lock_buffer): a memberlist message of a packet arriving before that
   * is handled at once; after it, it queues in the handoff queue in arrival order (memberlist's own
   * messages come first in a compound packet: gossip() takes its broadcasts before the delegate's)
   * and takes a place of the pipeline, or is dropped at a full one (gx_stats.fd_handoff_drops). The
   * queued messages are handled in the memberlist phase of the host's first unlocked round, before
   * that round's packets' (gx_fd_host.hq_len). 0 (default) = memberlist messages never wait for the
   * catalog lock (the round-5 model). */
  uint32_t fd_handoff_shared;
} gx_params;
#define GX_LOCK_HANDLER_AT 53u /* pipeline records at which memberlist's packet handler blocks */
#define GX_LOCK_BUF_MAX_BYTES (1ull << 36) /* 64 GiB of lock_buffer records per engine */
#define GX_PP_MATCHING 0
#define GX_PP_INITIATE 1

/* Per-host bookkeeping (read-back for parity). */
typedef struct gx_host_state {
  uint32_t fifo_head, fifo_tail;   /* broadcast FIFO ring counters (count = tail - head) */
  uint32_t sleep_head, sleep_tail; /* SendServices jobs sleeping TOMBSTONE_RETRANSMIT */
  uint32_t dq_head, dq_len;        /* delegate pendingBroadcasts (dq_len <= pending_cap between calls) */
  uint32_t arena_used;             /* bit w: list slots [32w, 32w + 32) all live (the lowest free slot
                                      is allocated: a two-level bitmap, slots >= list_slots count as live) */
  uint32_t flags;                  /* bit0 BroadcastServices blocked on nil, bit1 BroadcastTombstones blocked */
  int64_t bs_next;                 /* next BroadcastServices looper round */
  int64_t bt_next;                 /* next BroadcastTombstones looper round */
  int64_t last_bcast_ns;           /* BroadcastServices lastTime (services_state.go:526,560) */
  uint64_t running;                /* owner's local services currently running (discovery) */
  uint32_t fifo_stored;            /* end of the stored window: jobs [fifo_head, fifo_stored) are kept,
                                      [fifo_stored, fifo_tail) deferred (gx_job) */
  uint32_t nil_pos_bs, nil_pos_bt; /* queue position of each looper's last nil send */
  uint32_t lock;                   /* the ServicesState lock (gx_params.lock_model): bit (n & 1) = a
                                      looper held it at the start of round n (written for round n + 1
                                      when the host's round-n GetBroadcasts calls end, and by calls
                                      that block or unblock a looper between rounds); bit 2 =
                                      ExpireServer calls wait for it; bits 8..31 = records in the
                                      host's lock buffer */
} gx_host_state;
#define GX_LOCK_PENDING_EXPIRE 4u
#define GX_LOCK_DEFER_MERGE 8u /* bit 3 (lock_readers): a push-pull merge waits for the host's lock */
/* lock_readers: BroadcastTombstones (the write lock) held the lock at the start of round n */
#define GX_LOCK_W_AT(lock, round) (((lock) >> (4 + ((round) & 1))) & 1u)
#define GX_LOCK_DEFER_RES 26u  /* pipeline places a waiting merge takes: ServiceMsgs 25 + AddServiceEntry */
#define GX_LOCK_BUF_SHIFT 8
#define GX_LOCK_AT(lock, round) (((lock) >> ((round) & 1)) & 1u)
#define GX_LOCK_BUF(lock) ((lock) >> GX_LOCK_BUF_SHIFT)

typedef struct gx_stats {
  int64_t round;             /* current round */
  uint64_t gossip_merges;    /* AddServiceEntry evaluations from gossip packets */
  uint64_t ae_merges;        /* ... from anti-entropy push-pull (Merge) */
  uint64_t local_merges;     /* ... from owners (TrackNewServices) and API calls */
  uint64_t gossip_accepts;
  uint64_t ae_accepts;
  uint64_t local_accepts;
  uint64_t stale_drops;      /* IsStale gate, services_state.go:302-308 */
  uint64_t retransmits;      /* RETX jobs enqueued */
  uint64_t queue_drops;      /* LOST jobs dequeued: jobs the reference would have sent whose contents the
                                engine did not keep (gx_job); 0 = the run is faithful to the queue */
  uint64_t list_drops;       /* SendServices jobs queued as LOST because the list arena was full */
  uint64_t sleep_drops;      /* re-armed passes dropped because the sleep ring was full (engine bound) */
  uint64_t pending_drops;    /* records cut by MAX_PENDING_LENGTH (services_delegate.go:111-112):
                                the reference's own truncation, not an engine bound */
  uint64_t dequeues;         /* batches taken off the FIFO (nil included) */
  uint64_t nil_batches;
  uint64_t packets;          /* non-empty GetBroadcasts results */
  uint64_t records_sent;
  uint64_t expired;          /* records tombstoned by lifespan (services_state.go:655-679) */
  uint64_t gc;               /* tombstones removed after TOMBSTONE_LIFESPAN (:645-653) */
  uint64_t own_tombstones;   /* TombstoneServices (:685-715) */
  uint64_t expire_server;    /* ExpireServer calls that tombstoned something (:150-192) */
  uint64_t send_jobs;        /* SendServices jobs created */
  uint64_t ae_exchanges;     /* push-pull pairs */
  uint64_t churn_events;
  int64_t last_change_round; /* last round in which any view slot changed, -1 = none */
  uint64_t scan_slots;       /* view slots streamed by expiry scans */
  uint64_t ae_slots;         /* view slots streamed by anti-entropy merges (both directions) */
  uint64_t bytes_sent;       /* byte-limit mode: sum of len(message) + overhead of sent records */
  uint64_t cap_cuts;         /* byte-limit mode: packets cut by packet_cap before the byte limit */
  uint64_t change_events;    /* ServiceChanged calls (services_state.go:195-199), all views */
  uint64_t listener_drops;   /* ChangeEvents a full listener channel did not take (:230-236) */
  uint64_t lost_packets;     /* packets sent to a departed or partitioned-off peer (records lost) */
  uint64_t fd_probes;        /* probeNode calls */
  uint64_t fd_probe_failures;/* probes without a direct or indirect ack -> suspectNode */
  uint64_t fd_suspicions;    /* suspicion timers started (alive -> suspect) */
  uint64_t fd_confirmations; /* independent suspicion confirmations (Lifeguard) */
  uint64_t fd_deaths;        /* deadNode accepted: NotifyLeave calls */
  uint64_t fd_refutes;       /* refute(): a host raised its own incarnation */
  uint64_t fd_alive_updates; /* aliveNode accepted about another host */
  uint64_t fd_msgs_sent;     /* memberlist broadcasts put into gossip packets */
  uint64_t fd_msgs_received; /* memberlist broadcasts handled by receivers */
  uint64_t fd_state_merges;  /* remote node states merged by push-pull (mergeState) */
  uint64_t queue_deferred;   /* jobs queued past the stored window (kept as a count, gx_job) */
  int64_t first_drop_round;  /* round of the first queue_drops dequeue, -1 = none */
  /* The ServicesState lock (gx_params.lock_model) */
  uint64_t locked_merges;    /* lock_model = 0: AddServiceEntry calls the reference would not have made
                                then: gossip records merged by a host whose looper held the lock, and
                                both sides' merges of a push-pull exchange with such a host */
  int64_t first_locked_round;/* first round a locked host received gossip records or was in a push-pull
                                pair, -1 = none (both modes) */
  uint64_t lock_buffered;    /* records queued in a locked host's inbound pipeline */
  uint64_t lock_drops;       /* records that found the pipeline full (memberlist's handoff queue) */
  uint64_t lock_drained;     /* buffered records merged once the host was unlocked (also gossip_merges) */
  uint64_t ae_locked;        /* push-pull exchanges that did not run: a side held the lock */
  uint64_t expire_deferred;  /* ExpireServer calls that waited for the lock */
  uint64_t ae_deferred;      /* lock_readers: push-pull merges of a read-locked side that waited for its lock */
  uint64_t ae_defer_lost;    /* ... and that the engine could not keep (its pool slot was taken); 0 = faithful */
  uint64_t fd_handoff_queued; /* fd_handoff_shared: memberlist messages queued behind a blocked handler */
  uint64_t fd_handoff_drops;  /* ... and dropped at a full pipeline */
  uint64_t false_expiries;   /* of `expired`: alive-lifespan expiries (services_state.go:655-679) of a
                                record whose owner host has not departed (the owner is live; with
                                churn it may have stopped the service and its tombstone not arrived) */
} gx_stats;

/* Device time per kernel class, accumulated since create (HIP events; zeros for the oracle). */
#define GX_K_OWNER 0
#define GX_K_SCAN 1
#define GX_K_STORM 2
#define GX_K_SEND 3
#define GX_K_ROUTE 4
#define GX_K_MERGE 5
#define GX_K_AE 6
#define GX_K_CONVERGE 7
#define GX_K_ENCODE 8 /* LocalState JSON encoder (gx_local_state_json) */
#define GX_K_DECODE 9 /* Decode JSON parser (gx_decode_state_json, gx_merge_remote_state_json) */
#define GX_K_FD 10    /* memberlist failure detection: timers + probes, messages in and out */
#define GX_K_COUNT 11
typedef struct gx_timing {
  double ms[GX_K_COUNT];
  uint64_t launches[GX_K_COUNT];
  uint64_t bytes[GX_K_COUNT]; /* algorithmic bytes moved ("Algorithmic bytes") */
  uint64_t units[GX_K_COUNT]; /* slots / records processed */
} gx_timing;

typedef struct gx_engine gx_engine;

/* ---- lifecycle --------------------------------------------------------------------------- */
int gx_abi_version(void);
const char *gx_backend(void);               /* "hip-gfx950" or "oracle-cpu" */
void gx_params_default(gx_params *p);
int gx_create(const gx_params *p, gx_engine **out);
int gx_destroy(gx_engine *e);
int gx_set_round(gx_engine *e, int64_t round); /* advance the clock; wakes due sleepers */
int gx_get_round(gx_engine *e, int64_t *round);
int gx_epoch(gx_engine *e, int64_t *epoch_ns); /* gx_epoch_of(t0_ns): packed words' time origin */
int gx_enable_timing(gx_engine *e, int on);
/* Where this engine's device work goes. mode 0: its own stream. GX_STREAM_CALLER: the caller's
 * HIP stream `stream` (NULL = the default stream), e.g. the stream an exchange layer runs its
 * collectives on. GX_STREAM_ASYNC: the sharded phase calls below (round_send, outbox_pack,
 * inbox_unpack, round_merge, ae_pack, ae_delta_pack, ae_return_pack, ae_merge, round_end) return
 * once their work is queued; the stream orders the exchange after them, and a device error
 * surfaces at the next call that waits. Calls that return sizes or data wait as before. The
 * oracle accepts and ignores it. */
#define GX_STREAM_CALLER 1
#define GX_STREAM_ASYNC 2
int gx_set_stream(gx_engine *e, void *stream, int mode);

/* ---- whole-round driver (the hot path) ---------------------------------------------------- */
/* Runs n_rounds rounds of the seeded schedule (DESIGN.md "Round model"). */
int gx_run_rounds(gx_engine *e, uint32_t n_rounds);

/* ---- sharded rounds ----------------------------------------------------------
 * A round of a sharded engine is driven phase by phase by an exchange layer (sidecar_amd/dist.py,
 * torch.distributed: RCCL between GPUs, gloo for the CPU oracle). Exchange buffers are device
 * memory for the HIP engine and host memory for the oracle; `bytes_per_shard` has n_shards
 * entries. Wire formats (both little-endian):
 *   packet: u32 key (= sender * fanout + j), u32 receiver, u32 len, u32 n_fd, then packet_cap x
 *           {u64 word, u32 record key, u32 0} (the first len used); with fd_enable then fd_msg_cap x
 *           {u32 incarnation, u32 node | from << 16, u32 kind, u32 0} (the first n_fd used, the
 *           packet's memberlist messages); fixed-size slots grouped by destination shard, ascending
 *           key.
 *   digest: u32 pair index, u32 host, u32 n_blocks, u32 runs, then n_blocks x {u64 d0, u64 d1}, then
 *           with fd_enable and fd_push_pull_state H x u64 (the host's round-start member list:
 *           incarnation << 32 | state, 0xff = not in the list): the
 *           host's round-start row in blocks of GX_DIGEST_SLOTS slots (GX digest below); one
 *           message per cross-shard push-pull pair, grouped by destination shard, ascending pair.
 *           `runs` (fd_enable only, else 0): 1 if the sender holds the pair's initiator (first
 *           host) and the pair runs (path up, partner ALIVE in the initiator's list); the other
 *           side follows it, and a pair that does not run ships no blocks. Bit 1 of `runs`: the
 *           sender's host holds the ServicesState lock this round (lock_model): the pair fails, and
 *           with lock_model = 1 the sender's digests are all zero (its row is not read).
 *   lead:   u32 pair index, u32 host, u32 n_lead, u32 0, then n_lead encoded blocks (below): the
 *           row's blocks whose digests differ from the partner's and that this side leads,
 *           ascending. The side whose block has fewer literals leads it (the count rides in the
 *           digest); on a tie the pair's first host. A lead block encodes the sender's own words
 *           (own bits = the padding past the row's end). Grouped like the digests.
 *   return: per destination shard a table of u64 message sizes (one per pair, in message order),
 *           then the messages: u32 pair index, u32 host, u32 n_ret, u32 0, then n_ret u32 literal
 *           counts (padded with a 0 to an even number), then n_ret encoded blocks: for each block
 *           the partner leads, ascending, this side's words for the partner's merge. Slot i is an
 *           own slot (the partner merges its own word instead) when merging this side's word y
 *           into the partner's word x has exactly the effect of merging x into x: both absent, or
 *           both present, y not stored, and IsStale(y) == IsStale(x).
 *   encoded block: u64 own[8], u64 neu[8] (bit i of the 512-bit masks = slot i of the block),
 *           then one u64 word per neu bit. Slot i is the receiver's own word if own bit i is set,
 *           else literal number popcount(neu bits 0..i) - 1. neu bit i is set iff slot i is not an
 *           own slot and i = 0, slot i-1 is an own slot, or word(i) != word(i-1).
 * The follower merges the partner's lead blocks; the leader merges the follower's return blocks,
 * so a block's words cross the link once, run-length coded, plus the partner's winning words.
 * gx_run_rounds(e, n) on an unsharded engine equals n x (round_send, round_merge, ae_merge with
 * nothing received, round_end). */
int gx_round_send(gx_engine *e);  /* phases 0-3: wake, owner ticks, storm, GetBroadcasts */
int gx_outbox_bytes(gx_engine *e, uint64_t *bytes_per_shard);
int gx_outbox_pack(gx_engine *e, void *buf, uint64_t cap);
/* gx_outbox_bytes without waiting: the sizes are written to `bytes_per_shard` in the engine's
 * memory (device memory for the HIP engine) by work queued on its stream, so an exchange layer
 * can hand them to a collective (all-gather of the size matrix) with one host wait for both. The
 * following gx_outbox_pack packs as many slots as the device counted; a `cap` smaller than that
 * is reported as GX_EINVAL at the next call that waits. */
int gx_outbox_sizes_async(gx_engine *e, uint64_t *bytes_per_shard);
int gx_inbox_unpack(gx_engine *e, const void *buf, uint64_t bytes);
/* The gossip exchange with sizes every shard knows ahead, so no exchange layer waits on the device
 * for them: the packets shard s sends shard g in round n are bounded by the seeded peer sample
 * (GossipMessages slots per sampled peer of a host of s on g), which every shard can compute.
 * gx_exchange_plan fills sizes[s * G + g] = that bound in packet-slot bytes for the engine's current
 * round (from a batch of rounds computed ahead on the device); gx_outbox_pack_planned packs this
 * shard's packets for shard g into its sizes[me * G + g] bytes: the packets first (as
 * gx_outbox_pack), then empty slots (sender key 0xffffffff), which gx_inbox_unpack skips. Not with
 * the failure detector, whose targets come from the member lists: GX_ENOSYS. */
#define GX_SLOT_EMPTY 0xffffffffu
int gx_exchange_plan(gx_engine *e, uint64_t *sizes);
int gx_outbox_pack_planned(gx_engine *e, void *buf, uint64_t cap);
int gx_round_merge(gx_engine *e); /* phase 4: gather-then-merge of local + received packets */
/* Push-pull across shards exchanges block digests first and then only the blocks that differ
 * (Dynamo-style anti-entropy), each once: its leader ships it run-length coded, the follower
 * merges it and returns only the words that change the leader's merge. Views and every counter
 * equal those of a full-row exchange: a block whose digests match merges the host's own copy,
 * which is the same record set. Per AE round: gx_ae_bytes -> gx_ae_pack (digests) ->
 * [gx_ae_merge_local] -> exchange -> gx_ae_delta_bytes (received digests) -> gx_ae_delta_pack
 * (lead blocks) -> exchange -> gx_ae_return_bytes (received lead blocks) -> gx_ae_return_pack ->
 * exchange -> gx_ae_merge (both inboxes).
 * Digest of block b = slots [b*512, min(R, (b+1)*512)) of a row, i = slot index in the row,
 * w = slot word, sums mod 2^64, L = literal count of the block's lead encoding, u32 arithmetic
 * mod 2^32 in h: x = w ^ (i << 40) ^ i, lo/hi = its halves, a = (lo ^ rotl32(hi, 16)) * 0x85EBCA6B,
 * b = (hi ^ a >> 15) * 0xC2B2AE35, a = (a ^ b >> 13) * 0x27D4EB2F, a ^= a >> 16,
 * b = (b ^ a >> 11) * 0x165667B1, b ^= b >> 15, h_i = a << 32 | b:
 *   d0 = sum_i h_i,  d1 = (sum_i (h_i ^ (h_i >> 29)) mod 2^54) | L << 54 */
#define GX_DIGEST_SLOTS 512
int gx_ae_bytes(gx_engine *e, uint64_t *bytes_per_shard); /* digest messages; 0s unless a push-pull round */
int gx_ae_pack(gx_engine *e, void *buf, uint64_t cap);
int gx_ae_delta_bytes(gx_engine *e, const void *digests, uint64_t bytes, uint64_t *bytes_per_shard);
int gx_ae_delta_pack(gx_engine *e, void *buf, uint64_t cap); /* lead blocks */
int gx_ae_return_bytes(gx_engine *e, const void *lead, uint64_t lead_bytes, uint64_t *bytes_per_shard);
int gx_ae_return_pack(gx_engine *e, const void *lead, uint64_t lead_bytes, void *buf, uint64_t cap);
int gx_ae_merge(gx_engine *e, const void *lead, uint64_t lead_bytes, const void *ret, uint64_t ret_bytes);
/* Optional, between gx_ae_pack and gx_ae_merge: start the push-pull merges of the pairs whose two
 * hosts are both on this shard, asynchronously on the engine's stream, so they overlap the
 * exchanges; gx_ae_merge then merges only the cross-shard pairs. Pairs are disjoint (every
 * host is in at most one), so the result is identical either way. */
int gx_ae_merge_local(gx_engine *e); /* phase 5 */
int gx_round_end(gx_engine *e);   /* round += 1, wake due sleepers */
/* The ServicesState lock across shards (lock_model): *unlocked = this shard's hosts that do not
 * hold the lock this round (a synchronizing call). When the sum over every shard is 0 at a
 * push-pull round, every pair fails, and gx_ae_skip_locked stands for the whole exchange
 * (gx_ae_bytes .. gx_ae_merge; then gx_round_end): the same counts (ae_locked once per pair, by
 * the shard of its first host; first_locked_round), nothing moved. GX_EINVAL if a host here is
 * free, for an unsharded engine (G = 1), or with the failure detector or departures. */
int gx_lock_census(gx_engine *e, uint32_t *unlocked);
int gx_ae_skip_locked(gx_engine *e);
/* A planned gossip round in two calls (fewer host calls per round for an exchange layer; the same
 * work as the calls they stand for):
 *   gx_round_gossip_begin = gx_round_send + gx_exchange_plan(plan) + gx_outbox_pack_planned(buf, cap)
 *   gx_round_gossip_end   = gx_inbox_unpack(buf, bytes) + gx_round_merge, then, unless this round
 *                           is a push-pull round (*ae_round = 1: the caller runs the gx_ae_* steps
 *                           and gx_round_end), gx_round_end (*ae_round = 0).
 * plan: G * G entries as gx_exchange_plan. Same conditions and errors as those calls. The HIP
 * engine packs the buffer inside the send itself when GossipMessages is 1 and the planned
 * GetBroadcasts path runs (record budget, no failure detector or departures): a packet for
 * another shard is written straight into a slot of its destination's region, so the slots of a
 * region are in arrival order rather than sender order (the receiver ranks packets by sender key;
 * the merge is the same). gx_outbox_pack_planned must not be called after it for that round. */
int gx_round_gossip_begin(gx_engine *e, uint64_t *plan, void *buf, uint64_t cap);
int gx_round_gossip_end(gx_engine *e, const void *buf, uint64_t bytes, int *ae_round);
/* Per-record min and max slot word over this engine's views (R entries each; device memory for
 * the HIP engine), written as (word XOR 2^63) so that signed 64-bit MIN/MAX reductions across
 * shards order them like the unsigned words. All views agree on record r iff the reduced min
 * equals the reduced max. */
int gx_view_minmax(gx_engine *e, uint64_t *min_out, uint64_t *max_out);
/* The owner's own word of every record: out[r] = slot r of host r / S's own view (the version the
 * owner holds), for the owners this engine holds, 0 for the others (R entries; device memory for
 * the HIP engine, so a MAX reduction across shards gives every owner's word). */
int gx_owner_words(gx_engine *e, uint64_t *out);

/* ---- catalog.ServicesState ---------------------------------------------------------------- */
/* AddServiceEntry, services_state.go:293-347, applied in array order (views[i] <- svcs[i]). */
int gx_add_service_entries(gx_engine *e, const uint32_t *views, const gx_service *svcs,
                           uint32_t n, uint32_t *n_accepted);
/* Merge(otherState), services_state.go:367-373: every present record of src_view -> dst_view. */
int gx_merge(gx_engine *e, uint32_t dst_view, uint32_t src_view);
/* TombstoneOthersServices, services_state.go:635-683. Returns the tombstoned records in key
 * order; n_out = total count (may exceed cap; excess not written). */
int gx_tombstone_others(gx_engine *e, uint32_t view, gx_service *out, uint32_t cap,
                        uint32_t *n_out);
/* TombstoneServices(self, containerList), services_state.go:685-715: own services not in
 * `running` are tombstoned (each returned twice). */
int gx_tombstone_services(gx_engine *e, uint32_t host, const uint16_t *running, uint32_t n_running,
                          gx_service *out, uint32_t cap, uint32_t *n_out);
/* ExpireServer(hostname), services_state.go:150-192 (incl. SendServices(TOMBSTONE_COUNT)). */
int gx_expire_server(gx_engine *e, uint32_t view, uint32_t owner, int *expired);
/* SendServices(services, looper(n_passes)), services_state.go:579-604. */
int gx_send_services(gx_engine *e, uint32_t host, const gx_service *svcs, uint32_t n,
                     uint32_t n_passes);
/* One BroadcastServices looper body with fn() = list, services_state.go:525-574. */
int gx_broadcast_services(gx_engine *e, uint32_t host, const gx_service *list, uint32_t n);
/* One BroadcastTombstones looper body with fn() = list, services_state.go:606-633. */
int gx_broadcast_tombstones(gx_engine *e, uint32_t host, const gx_service *list, uint32_t n);
/* IsNewService, services_state.go:509-521. */
/* Dynamic key space (host mirror, catalog.hpp): bit s of *mask is set when some view of this engine
 * holds a record of any status for (owner, s). A slot that no view holds (never written, or
 * removed everywhere after TOMBSTONE_LIFESPAN, services_state.go:645-653) can take a service ID
 * seen for the first time. A sharded engine answers for its own views. */
int gx_owner_slots_in_use(gx_engine *e, uint32_t owner, uint64_t *mask);
int gx_is_new_service(gx_engine *e, uint32_t view, const gx_service *svc, int *is_new);

/* ---- catalog readers (catalog/view.go, services_state.go:726-748) ----------------------------
 * EachServiceSorted (view.go:14-26): the view's present records ordered by Updated; records with
 * equal Updated stay in key order (Go's sort.Sort leaves their order unspecified). With owner =
 * GX_ALL_OWNERS every server's records, else one server's: Server.SortedServices (view.go:48-58).
 * n_out = count (at most cap written). Sorted on the device (stable radix sort). */
#define GX_ALL_OWNERS 0xffffffffu
int gx_each_service_sorted(gx_engine *e, uint32_t view, uint32_t owner, gx_service *out, uint32_t cap,
                           uint32_t *n_out);
/* Service.Name of every record, for ByService: names[off[r] .. off[r + 1]) is the Name of record
 * r = host * S + svc (R + 1 offsets, off[0] = 0). Replaces any earlier table. */
int gx_set_service_names(gx_engine *e, const char *names, const uint64_t *off);
/* ByService (services_state.go:738-748): the view's present records grouped by Service.Name, in
 * EachServiceSorted order inside each group; groups in bytewise Name order (the reference returns a
 * Go map); group_out[i] (optional) = index of out[i]'s Name among the distinct names of the table.
 * GX_ENOENT if no names were set. */
int gx_by_service(gx_engine *e, uint32_t view, gx_service *out, uint32_t *group_out, uint32_t cap,
                  uint32_t *n_out);

/* ---- memberlist Delegate (services_delegate.go) ------------------------------------------- */
/* NotifyMsg (:72-83) + Start() decode loop (:46-56): the records of one packet -> UpdateService. */
int gx_notify_msg(gx_engine *e, uint32_t host, const gx_service *recs, uint32_t n);
/* Batched NotifyMsg over many hosts in one call: recs[i] is delivered to
 * hosts[i]; each run of consecutive entries with the same host is one message, in order. */
int gx_notify_msgs(gx_engine *e, const uint32_t *hosts, const gx_service *recs, uint32_t n);
/* GetBroadcasts(overhead, limit) (:85-144) with packPacket (:186-223). `limit` is the packet
 * budget in records (the caller converts memberlist's byte limit and per-message overhead);
 * GX_LIMIT_DEFAULT = params.packet_cap. 0 means nothing fits (the whole batch stays pending).
 * n_out = 0 means the reference returned nil. cap must be >= the effective limit. */
#define GX_LIMIT_DEFAULT 0xffffffffu
int gx_get_broadcasts(gx_engine *e, uint32_t host, uint32_t limit, gx_service *out, uint32_t cap,
                      uint32_t *n_out);
/* GetBroadcasts(overhead, limit) with the byte limit of the reference signature: packPacket
 * keeps the greedy prefix with total + len(message) + overhead <= limit (:194-203); a first
 * message that does not fit sends nothing and keeps everything pending (:205-221). At most cap
 * records are returned (pass cap >= packet_cap + 2 * pending_cap for the unbounded reference
 * result; a cut is counted in gx_stats.cap_cuts). */
int gx_get_broadcasts_bytes(gx_engine *e, uint32_t host, uint32_t overhead, uint32_t limit,
                            gx_service *out, uint32_t cap, uint32_t *n_out);
/* Encoded message length of records: Service.Encode() = ffjson MarshalJSONBuf
 * (service/service_ffjson.go:370-436) = the record's static bytes (every field except Updated
 * and Status: ID, Name, Image, Created, Hostname, Ports, ProxyMode and the JSON punctuation,
 * set with gx_set_static_bytes) + len of time.Time.MarshalJSON(Updated) (quoted RFC3339Nano,
 * UTC "Z", fraction with trailing zeros trimmed) + len of the decimal Status. */
#define GX_STATIC_BYTES_DEFAULT 192 /* services_delegate_test.go:16 fixture minus Updated/Status */
int gx_set_static_bytes(gx_engine *e, uint32_t owner_lo, uint32_t owner_hi,
                        const uint16_t *bytes /* [(owner_hi - owner_lo) * S] */);
int gx_message_bytes(gx_engine *e, const gx_service *recs, uint32_t n, uint32_t *out_bytes);
/* LocalState (:146-151): present records of the view in key order (n_out = total). */
int gx_local_state(gx_engine *e, uint32_t view, gx_service *out, uint32_t cap, uint32_t *n_out);
/* MergeRemoteState (:153-167): a decoded remote state -> Merge. */
int gx_merge_remote_state(gx_engine *e, uint32_t view, const gx_service *svcs, uint32_t n);
/* NotifyLeave (:173-176) -> ExpireServer(node). */
int gx_notify_leave(gx_engine *e, uint32_t view, uint32_t node);

/* ---- change bookkeeping and listeners --------------------------------------
 * Every ServiceChanged (services_state.go:195-199) of a view sets its Server's LastUpdated and
 * LastChanged and the view's state.LastChanged to the changed record's Updated, and notifies the
 * view's listeners. A newer record that keeps its status sets only LastUpdated (:321-323). The
 * call sites are AddServiceEntry (insert, previous status UNKNOWN; status change), the lifespan
 * expiry of TombstoneOthersServices (Updated + 1 s), TombstoneServices and ExpireServer (now).
 * "Last" is processing order: arrival order for gossip packets, key order for push-pull,
 * Merge and expiry scans, owner then service order for ExpireServer storms.
 * Initial catalogs (GX_INIT_OWN/WARM) count as inserted in key order, without events. */
typedef struct gx_server_times {
  int64_t last_updated_ns; /* Server.LastUpdated; 0 = time.Unix(0, 0) (NewServer, :57-66) */
  int64_t last_changed_ns; /* Server.LastChanged */
} gx_server_times;
typedef struct gx_change_event { /* catalog.ChangeEvent (services_state.go:38-43) */
  gx_service service;            /* the record after the change */
  int64_t time_ns;               /* Time = state.LastChanged at the notification */
  uint32_t previous_status;      /* PreviousStatus; GX_UNKNOWN for a new record */
  uint32_t pad;
} gx_change_event;
#define GX_MAX_LISTENERS 64
#define GX_LISTENER_MAX_CAPACITY 65536
/* Server times of owners [owner_lo, owner_hi) in `view`; meaningful while the server exists
 * (the view holds a record of it). */
int gx_read_server_times(gx_engine *e, uint32_t view, uint32_t owner_lo, uint32_t owner_hi,
                         gx_server_times *out);
int gx_read_last_changed(gx_engine *e, uint32_t view_lo, uint32_t view_hi, int64_t *out);
/* AddListener (:253-268): listener `id` of `view` with a channel buffered for `capacity` events.
 * Capacity 0 is refused like an unbuffered channel (GX_EINVAL); re-adding an id replaces it.
 * Events reach it with the channel's non-blocking send: a full channel drops the event
 * (listener_drops), :230-236. */
int gx_add_listener(gx_engine *e, uint32_t view, uint32_t id, uint32_t capacity);
int gx_remove_listener(gx_engine *e, uint32_t view, uint32_t id); /* :272-284; GX_ENOENT */
/* Receive the listener's buffered events, oldest first (at most cap; n_out = received). */
int gx_listener_drain(gx_engine *e, uint32_t view, uint32_t id, gx_change_event *out, uint32_t cap,
                      uint32_t *n_out);

/* ---- full-state JSON codec ------------------------------------------------
 * The wire format of memberlist push-pull: LocalState() = state.Encode() (services_delegate.go:
 * 146-151, services_state.go:117-125) and MergeRemoteState(buf) = catalog.Decode(buf) + Merge
 * (services_delegate.go:153-167, services_state.go:367-373, 774-782). The JSON is ffjson's
 * ServicesState/Server/Service marshal (catalog/services_state_ffjson.go:771-803, 334-375;
 * service/service_ffjson.go:370-436) with the Servers and Services maps falling back to
 * encoding/json (sorted keys, HTML-escaped strings, no trailing newline).
 *
 * Names. The record model carries indices, so the codec needs the strings once:
 *   hosts[host_off[o] .. host_off[o+1])  raw hostname of host o (Servers key, Server.Name,
 *                                         Service.Hostname, state.Hostname of view o)
 *   ids[id_off[r] .. id_off[r+1])        raw Service.ID of record r = host * S + svc
 *   pre/post of record r                 its encoded Service JSON around the Updated value:
 *       pre  = {"ID":..,"Name":..,"Image":..,"Created":..,"Hostname":..,"Ports":..,"Updated":
 *       post = ,"ProxyMode":..,"Status":
 *     exactly the bytes of Service.MarshalJSON after encoding/json's compaction (HTML-escaped);
 *     the record's JSON is pre + time.MarshalJSON(Updated) + post + decimal Status + "}".
 * gx_set_names also sets every record's static message bytes (gx_set_static_bytes) to
 * len(pre) + len(post) + 1, so packPacket lengths and the codec agree.
 * Times are formatted in UTC ("Z"): the reference formats time.Unix(0, 0) in the local zone,
 * which is UTC in Sidecar's containers.
 *
 * Decoding accepts RFC 8259 JSON whose types match the Go structs (ffjson would fail otherwise:
 * nothing is merged and GX_EINVAL is returned, the reference's "Failed to MergeRemoteState" log
 * and return, services_delegate.go:158-162). Object keys match fields ASCII-case-insensitively,
 * the last duplicate field wins, unknown fields are skipped. Deviations, all rejected with
 * GX_EINVAL because the reference result is undefined or depends on Go map order: a null server
 * or service (the reference panics in Merge), a repeated key inside the Servers map or one
 * Services map, two records with the same (Hostname, ID), nesting deeper than GX_JSON_MAX_DEPTH.
 * Records whose Hostname/ID are not in the names table are skipped and counted (`unknown`; the
 * reference would create them, the engine's key space is fixed). Status outside 0..6 is skipped
 * and counted (`invalid`). Updated is clamped into the engine's time window (GX_TS_SHIFT above):
 * a pre-1970, zero or otherwise pre-window time merges as the window's start, which IsStale drops
 * exactly like the original time; a time past the window merges as its end. The decoded records
 * are merged in key order (the model's Merge order), as anti-entropy merges. */
#define GX_JSON_MAX_DEPTH 16
typedef struct gx_names {
  const char *cluster_name;
  uint64_t cluster_name_len;
  const char *hosts;
  const uint64_t *host_off; /* [H + 1] */
  const char *ids;
  const uint64_t *id_off;   /* [R + 1] */
  const char *pre;
  const uint64_t *pre_off;  /* [R + 1] */
  const char *post;
  const uint64_t *post_off; /* [R + 1] */
} gx_names;
typedef struct gx_decode_stats {
  uint64_t bytes;    /* input length */
  uint64_t tokens;   /* JSON tokens (brackets, ':', ',', strings, scalars) */
  uint32_t services; /* Service objects under the winning Servers / Services members */
  uint32_t records;  /* records decoded (merged, for the merge call) */
  uint32_t unknown;  /* Hostname/ID not in the names table */
  uint32_t invalid;  /* Status outside 0..6 */
  int64_t error_at;  /* byte offset of the first error found, -1 = none (diagnostic only) */
} gx_decode_stats;
int gx_set_names(gx_engine *e, const gx_names *names);
/* LocalState(): the view's ServicesState JSON. n_out = its length; with cap < n_out nothing is
 * written (call again with a larger buffer). GX_ENOENT if no names were set. */
int gx_local_state_json(gx_engine *e, uint32_t view, char *out, uint64_t cap, uint64_t *n_out);
/* catalog.Decode(): the records of a ServicesState JSON in document order (n_out = total, at
 * most cap written), without merging. */
int gx_decode_state_json(gx_engine *e, const char *buf, uint64_t len, gx_service *out, uint32_t cap,
                         uint32_t *n_out, gx_decode_stats *ds);
/* MergeRemoteState(buf): Decode + Merge into `view`. */
int gx_merge_remote_state_json(gx_engine *e, uint32_t view, const char *buf, uint64_t len,
                               gx_decode_stats *ds);

/* ---- memberlist failure detection -------------------------------------------
 * memberlist is a dependency absent from the reference tree: github.com/NinesStack/memberlist
 * v0.0.0-20170522194404-cfac2b5cf519 (go.mod:6), a fork of hashicorp/memberlist. Sidecar uses
 * DefaultLANConfig (main.go:243-261) and reacts only to NotifyLeave -> go ExpireServer(node)
 * (services_delegate.go:173-176); NotifyJoin/NotifyUpdate only log (:169-171, :178-180). The
 * engine restates memberlist's published SWIM + Lifeguard algorithm (state.go probe/probeNode,
 * aliveNode/suspectNode/deadNode/refute, suspicion.go, queue.go TransmitLimitedQueue,
 * util.go kRandomNodes/retransmitLimit/suspicionTimeout) per simulated host; the resolutions
 * the round model makes are listed in DESIGN.md §3b. Parity against the fork is unpinned (no
 * reference test exercises it); the oracle and the GPU engine agree bit for bit.
 *
 * Each host keeps a member list over all H hosts (gx_member per (host, node)) and a broadcast
 * queue of memberlist messages: at most one queued message per node (a newer one invalidates
 * it), sent fewest-transmits first and newest first among equal counts, each sent
 * fd_retransmit_limit times. Host ids are 16-bit here: fd_enable requires n_hosts <= 65534. On a
 * sharded engine the per-host calls below take this shard's hosts. */
#define GX_M_ALIVE 0
#define GX_M_SUSPECT 1
#define GX_M_DEAD 2
#define GX_FD_NONE 0xffffu
#define GX_FD_MAX_TX 32
#define GX_FD_NO_DEADLINE 0x7fffffff
typedef struct gx_member {    /* memberlist nodeState of `node` in one host's list */
  uint32_t incarnation;
  uint32_t msg_incarnation;   /* the queued message about the node (when tx > 0) */
  int32_t change_round;       /* StateChange (suspicion start for SUSPECT) */
  int32_t deadline;           /* suspicion timer: fires at the first round >= deadline */
  uint8_t state;              /* GX_M_* */
  uint8_t n_conf;             /* independent confirmations of the suspicion */
  uint8_t tx;                 /* queued message: transmits + 1; 0 = none queued */
  uint8_t msg_kind;           /* GX_M_* kind of the queued message (alive / suspect / dead) */
  uint16_t msg_from;          /* From of the queued suspect / dead message */
  uint16_t susp_from[3];      /* suspicion: the accuser, then the confirmers (n_conf of them) */
  uint16_t q_prev, q_next;    /* queue links, GX_FD_NONE = end */
} gx_member;
typedef struct gx_fd_host {
  uint32_t probe_pass;        /* probe-list shuffles so far (resetNodes) */
  uint32_t probe_index;       /* probeIndex into the pass's permutation */
  int32_t wrap_round;         /* round of the last resetNodes; dead nodes older than
                                 GossipToTheDeadTime at that round are reaped */
  int32_t min_deadline;       /* earliest suspicion deadline of the host (exact lower bound) */
  uint32_t q_len;             /* queued memberlist messages */
  uint32_t departed;          /* 1 from depart_round on if this host crashed */
  uint16_t q_head[GX_FD_MAX_TX]; /* per transmit count: the newest queued node */
  uint32_t hq_len;            /* fd_handoff_shared: memberlist messages waiting in the handoff queue */
} gx_fd_host;
typedef struct gx_fd_msg {    /* alive / suspect / dead message (memberlist net.go) */
  uint32_t incarnation;
  uint16_t node;
  uint16_t from;              /* suspect / dead: the accuser; alive: the node itself */
  uint8_t kind;               /* GX_M_* */
  uint8_t pad[3];
} gx_fd_msg;
/* Derived memberlist parameters for n = p->n_hosts (util.go, suspicion.go):
 *   fd_retransmit_limit = RetransmitMult(4) * ceil(log10(n + 1))
 *   min = SuspicionMult(4) * max(1, log10(max(1, n))) * ProbeInterval (ms precision),
 *   max = SuspicionMaxTimeoutMult(6) * min; k = SuspicionMult - 2, 0 if n - 2 < k
 *   timeout(c) = max(min, max - (max - min) * log(c + 1) / log(k + 1)), floored to ms
 *   (c = 0: max, or min when k < 1), stored in rounds rounded up. */
int gx_fd_defaults(gx_params *p);
int gx_fd_read_members(gx_engine *e, uint32_t host, uint32_t node_lo, uint32_t node_hi, gx_member *out);
int gx_fd_read_hosts(gx_engine *e, uint32_t lo, uint32_t hi, gx_fd_host *out);
/* The host's queued memberlist messages in send order, with their transmit counts. */
int gx_fd_read_queue(gx_engine *e, uint32_t host, gx_fd_msg *out, uint8_t *transmits, uint32_t cap,
                     uint32_t *n_out);
/* memberlist packet handlers on one host, in order: aliveNode / suspectNode / deadNode
 * (state.go); a dead declaration calls NotifyLeave -> ExpireServer on the host's catalog view. */
int gx_fd_notify(gx_engine *e, uint32_t host, const gx_fd_msg *msgs, uint32_t n);
/* TransmitLimitedQueue.GetBroadcasts of one host with a budget of `limit` messages. */
int gx_fd_get_broadcasts(gx_engine *e, uint32_t host, uint32_t limit, gx_fd_msg *out, uint32_t *n_out);
/* One probe() of the host at the current round: target selection over the shuffled list, direct
 * and IndirectChecks probes, suspectNode on failure. target = GX_FD_NONE if nothing to probe. */
int gx_fd_probe(gx_engine *e, uint32_t host, uint32_t *target, int *acked);
/* Suspicion timers of the host due at the current round -> deadNode, in node order. */
int gx_fd_timers(gx_engine *e, uint32_t host);
/* pushPull's membership half (state.go mergeState) on one host: `remote` is a member list as
 * pushPull sends it, H x u64 (incarnation << 32 | state, 0xff = not in the list); alive ->
 * aliveNode, suspect or dead -> suspectNode{From: host}, in node order. */
int gx_fd_merge_state(gx_engine *e, uint32_t host, const uint64_t *remote);
/* Membership agreement with the truth: n_disagree = nodes that some live host of this engine sees
 * otherwise than they are (a crashed node not DEAD, a live node not ALIVE); converged iff 0 (on
 * every shard). */
int gx_fd_converged(gx_engine *e, int *converged, uint64_t *n_disagree);

/* ---- read-back, import, parity ------------------------------------------------------------ */
int gx_read_views(gx_engine *e, uint32_t view_lo, uint32_t view_hi, uint64_t *out_words);
/* One view unpacked (SURVEY.md §8b gx_read_view): ts_ns[R] absolute Updated (INT64_MIN where empty)
 * and status[R] (GX_ABSENT where empty), R = n_hosts * n_services. */
int gx_read_view(gx_engine *e, uint32_t view, int64_t *ts_ns, uint8_t *status);
int gx_write_views(gx_engine *e, uint32_t view_lo, uint32_t view_hi, const uint64_t *words);
int gx_write_slot(gx_engine *e, uint32_t view, const gx_service *svc); /* raw store, no merge rule */
int gx_read_hosts(gx_engine *e, uint32_t lo, uint32_t hi, gx_host_state *out);
/* The host's stored FIFO jobs [fifo_head, fifo_stored) in queue order (n_out = their count). */
int gx_read_queue(gx_engine *e, uint32_t host, gx_job *out, uint32_t cap, uint32_t *n_out);
int gx_read_sleepers(gx_engine *e, uint32_t host, gx_sleeper *out, uint32_t cap, uint32_t *n_out);
int gx_read_pending(gx_engine *e, uint32_t host, gx_service *out, uint32_t cap, uint32_t *n_out);
int gx_read_list(gx_engine *e, uint32_t host, uint32_t slot, gx_service *out, uint32_t cap,
                 uint32_t *n_out);
/* Order-sensitive 64-bit digest per host of (FIFO jobs, sleepers, pending, live lists). */
int gx_host_digests(gx_engine *e, uint64_t *out_per_host);
int gx_stats_get(gx_engine *e, gx_stats *out);
int gx_timing_get(gx_engine *e, gx_timing *out);
/* Catalog agreement: n_disagree = records r whose slot word differs between any two views. */
int gx_converged(gx_engine *e, int *converged, uint64_t *n_disagree);

#ifdef __cplusplus
}
#endif
#endif /* SIDECAR_GX_H */

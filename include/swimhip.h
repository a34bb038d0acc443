/*
 * swimhip.h — C ABI of libswimhip.so, the MI355X-native SWIM membership simulator.
 *
 * The library replaces, for N simulated members at once, the per-period hot path of
 * scalecube-cluster (reference @ /root/reference, v2.4.2-SNAPSHOT):
 *
 *   FailureDetectorImpl.doPing / doPingReq / onPing / onPingReq / onTransitPingAck
 *       cluster/src/main/java/io/scalecube/cluster/fdetector/FailureDetectorImpl.java:126-305
 *   GossipProtocolImpl.doSpreadGossip / onGossipReq / selectGossipMembers / sweepGossips
 *       cluster/src/main/java/io/scalecube/cluster/gossip/GossipProtocolImpl.java:139-304
 *   MembershipProtocolImpl.updateMembership / onFailureDetectorEvent / doSync / onSync /
 *       onSyncAck / onSuspicionTimeout
 *       cluster/src/main/java/io/scalecube/cluster/membership/MembershipProtocolImpl.java:304-673
 *   MembershipRecord.isOverrides
 *       cluster/src/main/java/io/scalecube/cluster/membership/MembershipRecord.java:66-84
 *   NetworkEmulator loss / block (fault injection seam)
 *       cluster-testlib/src/main/java/io/scalecube/cluster/utils/NetworkEmulator.java:166-180,348-351
 *
 * The reference has no SPI for these protocols: ClusterImpl hard-wires them
 * (cluster/src/main/java/io/scalecube/cluster/ClusterImpl.java:180-210). This ABI sits
 * *below* MembershipProtocol (MembershipProtocol.java:14-65) for all members at once; a
 * host binds it through Panama FFM / ctypes. Discrete replay
 * semantics (period = pingInterval, G gossip rounds per period, SYNC stagger) are fixed in
 * DESIGN.md §3.
 *
 * Conventions: plain C types only; the caller owns every buffer passed in; handles are
 * opaque; every entry point returns 0 or a negative SWIM_E* status (no exceptions cross
 * the ABI, mirroring the reference, which never throws protocol failures to callers —
 * FailureDetectorImpl.java:307-309, MembershipProtocolImpl.java:540). Message loss is
 * protocol semantics, never an error. One host thread per handle.
 */
#ifndef SWIMHIP_H
#define SWIMHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------------------ */
#define SWIM_OK 0
#define SWIM_EINVAL (-22)    /* bad argument / config                                    */
#define SWIM_ENOMEM (-12)    /* device allocation failed                                 */
#define SWIM_EHIP (-5)       /* HIP runtime error (incl. "no GPU")                       */
#define SWIM_ERCCL (-6)      /* RCCL error (multi-GPU)                                   */
#define SWIM_EOVERFLOW (-75) /* a bounded simulator buffer (events, gossips, syncs) overflowed */

/* ---- packed membership record (MembershipRecord.java:12-16, MemberStatus.java:3-16) ---
 * cell = incarnation << 2 | code ; code 1 = ALIVE, 2 = SUSPECT ; 0 = absent (no record in
 * membershipTable) ; 0xFFFFFFFF = DEAD. isOverrides(r1, r0) (MembershipRecord.java:66-84)
 * becomes:  r0 == 0 ? code(r1) == ALIVE : r1 > r0  (unsigned).                           */
#define SWIM_ABSENT 0u
#define SWIM_ALIVE 1u
#define SWIM_SUSPECT 2u
#define SWIM_DEAD 0xFFFFFFFFu
#define SWIM_PACK(inc, code) ((((uint32_t)(inc)) << 2) | (uint32_t)(code))

/* ---- membership events (api/membership/MembershipEvent.java:13-67) -------------------- */
#define SWIM_EV_ADDED 1
#define SWIM_EV_REMOVED 2
#define SWIM_EV_UPDATED 3
/* the other listen() streams of the reference, in the same ring (not MembershipEvents):
 * GossipProtocol.listen() (GossipProtocolImpl.java:171-183, sink.next on a new gossip id): a member's
 * first receipt of a user gossip of swim_spread; subject = the gossip's origin, record = its tag */
#define SWIM_EV_GOSSIP 8
/* FailureDetector.listen() (FailureDetectorImpl.java:365-368): one FailureDetectorEvent; subject =
 * the probed member, record = its status (SWIM_ALIVE, SWIM_SUSPECT or SWIM_DEAD), reason = its index
 * among the probe's events. Recorded only while swim_trace(SWIM_TRACE_FD) is on. */
#define SWIM_EV_FD 9
#define SWIM_TRACE_FD 1u

/* update reasons (MembershipProtocolImpl.java:58-64) */
#define SWIM_R_FAILURE_DETECTOR_EVENT 0
#define SWIM_R_MEMBERSHIP_GOSSIP 1
#define SWIM_R_SYNC 2
#define SWIM_R_INITIAL_SYNC 3
#define SWIM_R_SUSPICION_TIMEOUT 4

typedef struct swim_event {
  uint64_t period;   /* protocol period in which the event was emitted                   */
  uint32_t observer; /* member whose MembershipProtocol emitted it                       */
  uint32_t subject;  /* member the event is about                                        */
  uint32_t record;   /* packed record (REMOVED: the record that was removed)             */
  uint8_t type;      /* SWIM_EV_*                                                        */
  uint8_t reason;    /* SWIM_R_*                                                         */
  uint8_t phase;     /* sub-phase of the period (0 = FD, 1..G = gossip rounds, ...)      */
  uint8_t pad;
} swim_event;

/* ---- configuration: 1:1 with the reference config surface + simulator-only fields ----
 * FailureDetectorConfig (api/fdetector/FailureDetectorConfig.java:8-24)
 * GossipConfig          (api/gossip/GossipConfig.java:8-22)
 * MembershipConfig      (api/membership/MembershipConfig.java:13-30)
 * ClusterConfig         (api/ClusterConfig.java:24-43)                                    */
typedef struct swim_config {
  uint32_t n_members;   /* N simulated members (ids 0..N-1)                               */
  uint32_t mode;        /* 0 = dense N x N views; 1 = N x K tracked-subject views (below)  */
  uint64_t seed;        /* Philox key                                                     */
  int32_t ping_interval_ms;
  int32_t ping_timeout_ms;
  int32_t ping_req_members;
  int32_t gossip_fanout;
  int32_t gossip_interval_ms;
  int32_t gossip_repeat_mult; /* infection rounds are kept mod 2^8: swim_create rejects
                               gossip_repeat_mult * bit_length(n_members) > 83 (sweep + infectedFrom
                               horizon past 255 rounds), e.g. 4 at 2^20 members or 5 at 65,536; the
                               reference's presets (3, local 2) pass at every size up to 2^27 */
  int32_t sync_interval_ms;
  int32_t sync_timeout_ms;
  int32_t suspicion_mult;   /* suspicionMult * bit_length(n_members) + 64 must stay below 2^14 periods
                               (u16 deadline cells; larger: SWIM_EINVAL)                    */
  int32_t metadata_timeout_ms;
  uint32_t n_seeds;         /* MembershipConfig.seedMembers = members [0, n_seeds)        */
  uint32_t gossip_capacity; /* live gossip slots (a multiple of 1,024: a power of two masks ids,
                               any other size takes them mod the size; 0 = default)         */
  uint32_t event_capacity;  /* buffered MembershipEvents (0 = events not recorded)        */
  uint32_t sync_capacity;   /* SYNC requests per period (0 = default)                     */
  uint32_t tracked_subjects; /* mode 1: K subject columns. A subject gets a column the first time
                               any observer's record of it leaves the converged baseline (ALIVE,
                               incarnation 0); untracked subjects read as that baseline in every
                               view. More than K such subjects -> SWIM_EOVERFLOW */
  uint32_t n_initial;       /* members started (converged) at create: ids [0, n_initial); 0 = all
                               N. Ids [n_initial, N) are spare slots, absent from every view, for
                               swim_join / swim_restart (dense handles, sharded or not)          */
  int32_t device;           /* HIP device ordinal the handle lives on                     */
  uint32_t shard_rank;      /* observer-row shard of this handle (0 .. shard_world-1)     */
  uint32_t shard_world;     /* shards of the cluster (0 or 1 = unsharded); see swim_shard_step */
  uint32_t gossip_batching; /* 0 = gossips one member creates in one phase share one ring slot while
                               no probabilistic loss is set (exact: they travel identically, DESIGN.md
                               §3.12); 1 = one slot per gossip always                             */
  uint32_t record_capacity; /* gossip records live at once in batch slots (power of two; 0 = default) */
  uint32_t infection_round_bits; /* per (member, ring slot) storage of the gossip's infection round:
                               8 = the round mod 2^8; 4 = a 4-bit offset from the slot's creation round,
                               rounds 15 or more after it in an escape table (exact either way; halves the
                               largest array); 0 = 4 when the 8-bit array would exceed
                               96 GiB on this handle, else 8 */
  uint32_t dict_subjects;   /* record dictionary of the batched apply: subjects with live
                               gossip records that each get a block of 8 entries (a power of two, 4 ..
                               2^17; 0 = 8,192). A subject without a block merges through the spill table;
                               each receiver in flight keeps dict_subjects bytes of entry bitmap in LDS, so
                               larger dictionaries run fewer receivers per CU, and a receiver's bitmap must
                               fit a workgroup's 160 KiB of LDS (larger: SWIM_EINVAL) */
} swim_config;

typedef struct swim_stats {
  uint64_t period;            /* periods stepped so far                                   */
  uint64_t fd_probes;         /* doPing calls that selected a target                      */
  uint64_t fd_direct_ok;      /* direct PING acknowledged                                 */
  uint64_t fd_ping_req;       /* probes that went to ping-req                             */
  uint64_t fd_suspect_events; /* FailureDetectorEvent(SUSPECT) published                  */
  uint64_t fd_alive_events;   /* FailureDetectorEvent(ALIVE) published                    */
  uint64_t gossips_created;   /* GossipProtocol.spread() calls                            */
  uint64_t gossip_first_receipts; /* onGossipReq with a new gossip id                     */
  uint64_t gossip_sends;      /* GossipRequest messages to alive peers (window x peers)    */
  uint64_t syncs_sent;        /* SYNC messages (periodic + FD-triggered)                  */
  uint64_t syncs_delivered;
  uint64_t sync_acks_delivered;
  uint64_t records_accepted;  /* updateMembership calls that changed the table            */
  uint64_t events_added;
  uint64_t events_removed;
  uint64_t suspicion_timeouts;
  uint64_t refutations;       /* onSelfMemberDetected                                     */
  uint64_t overflow;          /* bit mask of overflowed buffers (0 = none)                */
  uint64_t live_gossip_slots; /* gossip slots currently in use                            */
  uint64_t not_converged;     /* (alive observer, crashed subject) cells still present    */
  /* work counters for the bench's algorithmic-byte model; 0 in the oracle */
  uint64_t gossip_scanned;    /* active bitmap words scanned by k_gossip_select (x members) */
  uint64_t gossip_probes;     /* receiver holds-now bitmap words read by k_gossip_send     */
  uint64_t sweep_cells;       /* deadline cells streamed by k_susp_sweep                  */
  uint64_t merge_cells;       /* table cells merged by k_sync_merge                       */
  uint64_t ack_cells;         /* table cells merged by k_sync_ack                         */
  uint64_t gossip_hd_words;   /* active words whose infection rounds k_gossip_select read  */
  uint64_t gossip_window_words; /* window words written by k_gossip_select (x members)    */
  uint64_t gossip_pull_words; /* active window words examined by k_gossip_pull (x receivers) */
  /* GossipState.infectedFrom (GossipProtocolImpl.java:181,248); 0 in the oracle
   * except infected_suppressed */
  uint64_t infected_pruned_pairs; /* (sender, peer) pairs whose window was pruned              */
  uint64_t infected_records;  /* deliveries recorded in full                                  */
  uint64_t infected_suppressed; /* GossipRequests not sent: peer in infectedFrom (alive peers) */
  /* k_gossip_apply's work, for its HBM byte model; 0 in the oracle */
  uint64_t apply_words;       /* receipt words folded into holdings / infection rounds        */
  uint64_t apply_runs;        /* subject-run representatives read from the ring               */
  uint64_t apply_subjects;    /* updateMembership calls (one per subject per receiver)        */
  uint64_t fd_dead_events;    /* FailureDetectorEvent(DEAD): an ACK with DEST_GONE (FDI:231-235,383) */
  uint64_t apply_spills;      /* subjects k_gossip_apply merged through the global inbox (LDS hash full); 0 in the oracle */
  uint64_t apply_records;     /* gossip records of batch slots expanded by k_gossip_apply; 0 in the oracle */
  uint64_t live_gossip_records; /* gossips held in the live ring slots (live_gossip_slots counts batches) */
  uint64_t events_updated;    /* MembershipEvent UPDATED: an accepted ALIVE record whose fetched
                                 metadata differs from the stored one (MembershipProtocolImpl.java:589-610) */
  uint64_t apply_pairs;       /* receiver pairs k_gossip_apply processed two to a workgroup; 0 in the oracle */
  uint64_t commit_radix;      /* commit phases sorted by the chip-wide radix sort; 0 in the oracle      */
  uint64_t escape_entries;    /* 4-bit infection rounds: live escape-table entries after the last period's
                                 sweep; 0 in the oracle and on 8-bit handles */
  uint64_t escape_capacity;   /* the escape table's entries (0 on 8-bit handles)                      */
  uint64_t apply_skipped;     /* dictionary blocks the batched apply skipped by their merge mark: every
                                 received record already found not to override the cell (DESIGN.md
                                 §3.15); 0 in the oracle */
  uint64_t apply_bitmaps;     /* long record ranges the batched apply ORed as their slot's entry bitmap
                                 instead of walking their ids; 0 in the oracle */
  uint64_t apply_bitmap_records; /* the records of those ranges (their ids were not read)          */
  uint64_t quiet_periods;     /* periods whose gossip rounds were skipped: no member held a gossip
                                 (quiet periods; SWIMHIP_QUIET=0 in the environment
                                 at swim_create runs every round, for A/B tests); 0 in the oracle */
} swim_stats;

typedef struct swim_handle swim_handle;

/* Lifecycle. ClusterImpl.doStart0 wiring (core/ClusterImpl.java:170-227) for N members that
 * start converged: every view holds every member ALIVE inc 0. */
int swim_create(const swim_config* cfg, swim_handle** out);
int swim_destroy(swim_handle* h);

/* Fault injection (NetworkEmulator.java:81-98,166-180): uniform outbound loss in basis
 * points (0..10000; 10000 = blockAllOutbound). A probabilistic loss (0 < loss < 10000) draws
 * per gossip, so batch slots cannot follow it: setting one while a slot holding several gossips
 * is still live returns SWIM_EINVAL (set the loss before the gossips are created, or create the
 * handle with gossip_batching = 1). */
int swim_set_loss(swim_handle* h, uint32_t loss_bp);
/* Mean message delay in ms on every link (NetworkEmulator.setDefaultOutboundSettings(loss, meanDelay)
 * :81-84, tryDelayOutbound :189-201, evaluateDelay :358-368; 0 = none; <= 60,000). Each message draws
 * an exponential delay: a GossipRequest is handled delay / gossipInterval rounds after it was sent,
 * and a ping, ping-req relay or metadata round trip counts only if it returns within its timeout
 * (DESIGN.md §3.16). Draws per message, so, like a probabilistic loss, it needs one gossip per ring
 * slot (SWIM_EINVAL while batch slots are live). Messages already in flight keep their arrival rounds
 * when the mean changes (or is reset to 0). Up to 65,536 observer rows per handle (shard). */
int swim_set_delay(swim_handle* h, uint32_t mean_ms);
/* Partition groups: messages a->b are lost while period in [t0, t1) and group[a] != group[b]
 * (NetworkEmulator.blockOutbound on both sides of a cut). n must equal n_members. */
int swim_set_partition(swim_handle* h, const uint8_t* group, uint32_t n, uint64_t t0, uint64_t t1);
/* Directed outbound block src->dst (NetworkEmulator.blockOutbound(Address...) :105-119): the
 * sender's send fails immediately (tryFailOutbound :166-180). */
int swim_block_link(swim_handle* h, uint32_t src, uint32_t dst, int blocked);
/* Inbound block at dst of messages from src (NetworkEmulator.blockInbound :255-269): dst's
 * transport silently drops them (NetworkEmulatorTransport.java:64-68,73-77); the send succeeds. */
int swim_block_inbound(swim_handle* h, uint32_t dst, uint32_t src, int blocked);
/* Crash = transport.stop() (MembershipProtocolTest.java:991-1000): the member stops
 * sending, receiving, answering and firing timers, from the next period on. */
int swim_crash(swim_handle* h, const uint32_t* ids, uint32_t n);

/* Graceful leave = Cluster.shutdown() (ClusterImpl.java:370-408): each member's own record
 * becomes DEAD and is spread as a gossip (MembershipProtocolImpl.leaveCluster :203-212); the member
 * keeps running until its own sweep drops that gossip (spread() completes at sweep,
 * GossipProtocolImpl.java:299-302), then stops at the end of that gossip round. On a sharded handle the
 * member's shard announces the stop in the next commit exchange (liveness is replicated). */
int swim_leave(swim_handle* h, const uint32_t* ids, uint32_t n);

/* Cluster.updateMetadata (ClusterImpl.java:364-367): each member's metadata changes (a new version;
 * MetadataStoreImpl.updateMetadata) and MembershipProtocolImpl.updateIncarnation (:184-196) makes its
 * own record ALIVE with incarnation + 1 and spreads it. Observers that accept the new record fetch the
 * metadata (MetadataStoreImpl.fetchMetadata :151-193) and, for a member they already had, emit UPDATED
 * when it differs from the one they stored (onAliveMemberDetected :589-610). Takes effect before the
 * next period. */
int swim_update_metadata(swim_handle* h, const uint32_t* ids, uint32_t n);

/* Join = a new member's ClusterImpl.start() (ClusterImpl.java:170-227): spare slot `ids[k]` (never
 * started) starts before the next period at an address of its own with a table holding only itself
 * (MembershipProtocolImpl.java:130-139), and in that period's SYNC phase makes the initial SYNC to
 * every seed address (start0, :222-257); the first SYNC_ACK that comes back (lowest seed address
 * whose round trip is delivered) is merged with reason INITIAL_SYNC (not re-spread, :649-656).
 * Periodic doSync follows the usual stagger from the next period on. Dense handles; a sharded handle
 * takes the same call on every rank (an initial SYNC to a seed on another shard travels in the SYNC
 * exchange). */
int swim_join(swim_handle* h, const uint32_t* ids, uint32_t n);
/* Restart on the same address (MembershipProtocolTest.testRestartStoppedMembersOnSameAddresses,
 * :453-520): stopped member old_ids[k]'s address is taken by spare slot new_ids[k], a NEW member id
 * joining as in swim_join. Messages sent to the old id reach the new member: a PING answers
 * DEST_GONE, so the prober's FD emits DEAD for the old id (FailureDetectorImpl.java:231-235,383);
 * a metadata request for the old id fails (MetadataStoreImpl.java:216-223); gossip and SYNC are
 * handled by the new member, which ignores records of other ids at its own address
 * (MembershipProtocolImpl.java:499-505). Dense handles, sharded or not (as swim_join). */
int swim_restart(swim_handle* h, const uint32_t* old_ids, const uint32_t* new_ids, uint32_t n);

/* GossipProtocol.spread (GossipProtocol.java:12-29, GossipProtocolImpl.java:124-128): member
 * `origin` spreads a user gossip carrying `tag` (the payload stand-in); it is created before the
 * next period (infectionPeriod = that period's first round), travels like every gossip, and each
 * member's first receipt is a SWIM_EV_GOSSIP event. */
int swim_spread(swim_handle* h, uint32_t origin, uint32_t tag);
/* A message of an external node delivered to simulated member `observer` before the next period
 * (the wire bridge, swimhip/wire.py: a real JVM member's SYNC / SYNC_ACK / membership gossip, decoded
 * from the reference's JSON). Each (subjects[k], records[k]) goes through updateMembership in order
 * (MembershipProtocolImpl.java:481-547) with `reason` SWIM_R_SYNC, SWIM_R_INITIAL_SYNC (syncMembership,
 * :463-473) or SWIM_R_MEMBERSHIP_GOSSIP (onMembershipGossip, :407-414); records accepted under SYNC
 * spread as gossips created for the next period's first round (:649-656); a metadata fetch for an
 * accepted ALIVE record draws with counter SWIM_DELIVER_ATTEMPT | k in that period's FD tick. A stopped
 * member receives nothing. records[k] must not be SWIM_ABSENT (a SyncData carries present records). */
#define SWIM_DELIVER_ATTEMPT 0x80000000u
/* reason flag (with SWIM_R_MEMBERSHIP_GOSSIP): the records are gossips with ids new to the observer
 * (GossipProtocolImpl.onGossipReq, :171-183): each one's GossipState is put before membership handles
 * it, so the observer forwards it in later rounds like a gossip it created (with its next gossip
 * sequence number as the id); the host drops ids it delivered to the observer before (swimhip/wire.py) */
#define SWIM_DELIVER_FORWARD 0x100u
int swim_deliver_records(swim_handle* h, uint32_t observer, const uint32_t* subjects, const uint32_t* records,
                         uint32_t n, uint32_t reason);
/* Optional trace streams into the event ring (mask of SWIM_TRACE_*; 0 = off, the default). */
int swim_trace(swim_handle* h, uint32_t mask);

/* Advance `periods` protocol periods (FD, G gossip rounds, suspicion
 * timeouts, SYNC/SYNC_ACK). Asynchronous to the host only inside the call. */
int swim_step(swim_handle* h, uint32_t periods);
/* Same, enqueued on the handle's stream without a final device sync (bench timing). */
int swim_step_async(swim_handle* h, uint32_t periods);
int swim_sync(swim_handle* h);

/* ---- observer-row sharding over several GPUs ----------------------------
 * A cluster of N members may be split into W = shard_world handles (one per GPU / process),
 * handle r owning observers [r*N/W, (r+1)*N/W) (N % W == 0). Every handle is created with
 * the same config except shard_rank, and receives the same fault-injection calls. A period
 * is then advanced with swim_shard_step, which runs the period's kernels up to the next
 * cross-shard exchange and describes it in a swim_xchg; the host performs the collective
 * over its communicator (RCCL all-gather / all-to-all-v / all-reduce) on the two device
 * buffers it attached, fills recv_counts, and calls swim_shard_step again. The exchanges of
 * one period: gossip-id commits (all-gather of the gossips created in a phase; each rank's block
 * also carries its per-word gossip liveness and bit-length bounds, merged by element-wise max),
 * the per-round sender windows bound for receivers on other shards (all-to-all-v), and the
 * SYNC / SYNC_ACK membership-table rows of cross-shard pairs (all-to-all-v). Results are
 * identical to the unsharded handle's. The library currently emits SWIM_X_ALLGATHER and
 * SWIM_X_ALLTOALLV only; SWIM_X_ALLREDUCE_MAX stays reserved (an element-wise *unsigned* max). */
#define SWIM_MAX_WORLD 64
#define SWIM_X_DONE 0          /* the period is complete                                   */
#define SWIM_X_ALLGATHER 1     /* every rank contributes send_words (host pads to the max)  */
#define SWIM_X_ALLTOALLV 2     /* send_counts[q] words to rank q, consecutive in rank order */
#define SWIM_X_ALLREDUCE_MAX 3 /* element-wise u32 max of send_words words, in place       */
typedef struct swim_xchg {
  uint32_t op;
  uint32_t world;
  uint64_t send_words;
  uint64_t send_counts[SWIM_MAX_WORLD];
  uint64_t recv_counts[SWIM_MAX_WORLD]; /* host: words received from each rank             */
  uint64_t recv_stride;                 /* host, ALLGATHER: words per rank block in recv;
                                           ALLTOALLV: words sent by all ranks together      */
} swim_xchg;
/* Device buffer sizes (u32 words) the host must allocate and attach before stepping. */
int swim_shard_buffer_words(swim_handle* h, uint64_t* send_words, uint64_t* recv_words);
int swim_shard_attach(swim_handle* h, void* send_dev, void* recv_dev);
/* Begin a period (when none is in flight) or resume it after the described exchange. */
int swim_shard_step(swim_handle* h, swim_xchg* x);

/* Library-driven exchanges. With a transport attached, swim_step / swim_step_async advance a sharded
 * handle through whole periods: at each exchange the library gathers every rank's status row (error
 * code, op, send counts: one small all-gather and one host stop, so an error any rank detects fails
 * every rank together; the counts and the errors the device state raises are written into the row on
 * the device, so the status read is the exchange's only host stop), then moves the data itself (an all-gather padded to the largest block, or an
 * all-to-all-v) and resumes. The handle allocates its exchange buffers unless swim_shard_attach gave
 * some. Either the library's own RCCL communicator over xGMI (swim_shard_comm_init: rank 0 makes a
 * unique id with swim_rccl_unique_id and the host hands it to every rank; the collectives run on the
 * handle's stream), or the host's collectives through a swim_transport (host_staged = 1: the library
 * stages through host memory and calls back with host pointers, e.g. gloo; 0: device pointers on
 * `stream`). Both calls return 0 on success; rank order everywhere. */
typedef struct swim_transport {
  void* ctx;
  uint32_t host_staged;
  /* every rank contributes `bytes` from send; recv gets world blocks of `bytes`, in rank order */
  int (*allgather)(void* ctx, const void* send, void* recv, uint64_t bytes, void* stream);
  /* send_bytes[q] bytes to rank q (consecutive in send, in rank order); recv_bytes[q] from rank q */
  int (*alltoallv)(void* ctx, const void* send, const uint64_t* send_bytes, void* recv, const uint64_t* recv_bytes,
                   void* stream);
} swim_transport;
int swim_shard_set_transport(swim_handle* h, const swim_transport* t);
int swim_rccl_unique_id(uint8_t unique_id[128]);
/* rank / world must equal the handle's shard_rank / shard_world */
int swim_shard_comm_init(swim_handle* h, const uint8_t unique_id[128], uint32_t rank, uint32_t world);

/* Events in canonical order (period, observer, phase, subject, type, reason, record). buf = NULL
 * with cap = 0 discards the pending events and returns their count (no copy, no sort). */
int swim_drain_events(swim_handle* h, swim_event* buf, uint64_t cap, uint64_t* n_out);
/* One observer's membershipTable as packed cells (n = n_members; the observer's shard). */
int swim_read_view(swim_handle* h, uint32_t observer, uint32_t* row, uint32_t n);
/* Suspicion deadlines (period at which the timer fires, 0 = none) for one observer. */
int swim_read_deadlines(swim_handle* h, uint32_t observer, uint32_t* row, uint32_t n);
/* Order-independent 64-bit digests of all views and all deadlines. */
int swim_digest(swim_handle* h, uint64_t* view_digest, uint64_t* deadline_digest);
/* Per-subject convergence: number of alive observers whose view holds the subject, and the
 * last period in which any observer removed it. Arrays of n_members entries. */
int swim_read_presence(swim_handle* h, uint32_t* present, uint32_t* last_removed, uint32_t n);
int swim_stats_get(swim_handle* h, swim_stats* out);
const char* swim_last_error(swim_handle* h);

/* Device known-answer check of the packed isOverrides (MembershipRecordTest.java:46-108):
 * out[i] = isOverrides(r1[i], r0[i]) computed by a gfx950 kernel. No handle needed. */
int swim_kat_is_overrides(const uint32_t* r1, const uint32_t* r0, uint8_t* out, uint64_t n);
/* Device Philox4x32-10 draws (counter = {a,b,c,tick}, key = seed ^ kind) for RNG parity. */
int swim_kat_philox(uint64_t seed, uint32_t kind, const uint32_t* abc_tick, uint32_t* out, uint64_t n);
/* All four output words (out4[4i .. 4i+3]); with kind = 0 the key is {seed lo, seed hi}, so the
 * Random123 philox4x32_10 known-answer vectors apply directly (tests/test_philox_kat.py). */
int swim_kat_philox4(uint64_t seed, uint32_t kind, const uint32_t* abc_tick, uint32_t* out4, uint64_t n);

/* Device check of the scans every compaction is built on (no reference counterpart): for n
 * inputs (a multiple of 1,024), the exclusive prefix sum within each 64-lane wave and each wave's
 * total (n / 64 entries), and the exclusive prefix sum within each 1,024-thread workgroup and each
 * workgroup's total (n / 1,024 entries), computed by gfx950 kernels. No handle needed. */
int swim_kat_scan(const uint32_t* in, uint64_t n, uint32_t* wave_excl, uint32_t* wave_tot, uint32_t* block_excl,
                  uint32_t* block_tot);

/* Debug: the gossips a member holds, as (gossip hash, infection round) pairs. */
int swim_debug_holdings(swim_handle* h, uint32_t member, uint32_t* out_hash, uint32_t* out_inf, uint32_t cap,
                        uint32_t* n_out);

/* Debug: per-member protocol cursors, 6 arrays of n: FD epoch, FD cursor, gossip epoch,
 * gossip cursor, gossip counter, member count (others). */
int swim_debug_member_state(swim_handle* h, uint32_t* out6n, uint32_t n);

/* Debug: per sender, cumulative GossipRequests to alive peers before infectedFrom suppression
 * (out2n[2i]) and the ones suppressed (out2n[2i+1]); gossip_sends = sum(before) - sum(suppressed). */
int swim_debug_sends(swim_handle* h, uint64_t* out2n, uint32_t n);

/* Kernel timing for the bench: the last step's per-kernel-class device time (ms, HIP events
 * on the handle's stream). idx: 0 fd, 1 gossip_pull, 2 gossip_apply, 3 suspicion, 4 sync_merge,
 * 5 sync_ack, 6 sync_snapshot, 7 bookkeeping, 8 gossip_select, 9 gossip_inhist, 10 gossip_pairwin
 * (fill + prune), 11 gossip_record. Returns accumulated time since the last reset. */
int swim_kernel_time(swim_handle* h, uint32_t idx, double* ms, uint64_t* launches);
/* enable: 0 = off, 1 = every class, otherwise a mask of (1 << class) bits: only those launches are
 * bracketed by events (each event pair costs the stream a few microseconds). */
int swim_kernel_time_reset(swim_handle* h, int enable);

#ifdef __cplusplus
}
#endif

#endif /* SWIMHIP_H */

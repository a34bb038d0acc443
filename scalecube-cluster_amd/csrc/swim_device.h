// swim_device.h — device-side state, kernel parameters and the shared updateMembership.
//
// Data layout in HBM (dense mode, N members, GC gossip slots):
//   view   u32[N][N]  observer-major packed records  (MembershipProtocolImpl.java:87)
//   dl     u16[N][N]  SUBJECT-major suspicion deadlines (dl_enc, 0 = none) so the timeout sweep
//                     streams one subject column over all observers (MembershipProtocolImpl.java:101)
//   sp_*   spill table: lattice max per (observer, subject) of a round's records that found no LDS
//                     slot / dictionary entry (bounded open addressing, emptied after every round)
//   hb     u32[N][GC/32] member-major "holds gossip slot s now" bitmap
//   hd     u8[N][GC]     infection round (mod 2^8) of each held gossip
//                     (GossipProtocolImpl.java:49, GossipState.java:14)
//   act    u32[GC/32]    this round's active bitmap words (k_gossip_prep): the words where some
//                     holder's send window or sweep can change; every other word is skipped
//   wb, nb u32[N][GC/32] per member, indexed by position in `act`: start-of-round send window and
//                     the round's first receipts (k_gossip_pull)
// plus per-member vectors (cursors, counts, liveness) and per-slot gossip metadata.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/swimhip.h"
#include "swim_rng.h"

namespace swim {

// control block counters (device, zeroed at create)
enum StatIdx : int {
  ST_FD_PROBES = 0,
  ST_FD_DIRECT_OK,
  ST_FD_PING_REQ,
  ST_FD_SUSPECT_EV,
  ST_FD_ALIVE_EV,
  ST_GOSSIPS_CREATED,
  ST_GOSSIP_RECEIPTS,
  ST_GOSSIP_SENDS,
  ST_SYNCS_SENT,
  ST_SYNCS_DELIVERED,
  ST_ACKS_DELIVERED,
  ST_ACCEPTED,
  ST_ADDED,
  ST_REMOVED,
  ST_SUSP_TIMEOUTS,
  ST_REFUTATIONS,
  ST_G_SCANNED,
  ST_G_PROBES,
  ST_SWEEP_CELLS,
  ST_MERGE_CELLS,
  ST_ACK_CELLS,
  ST_G_HDREAD,
  ST_G_WINW,
  ST_G_PULLW,
  ST_GOSSIP_SUPP,  // GossipRequests not sent because the peer is in infectedFrom (GPI:248)
  ST_IF_PAIRS,     // (sender, peer) pairs whose window was pruned by infectedFrom records
  ST_IF_RECORDS,   // deliveries recorded as infectedFrom sets
  ST_APPLY_WORDS,  // receipt words k_gossip_apply folded into holdings and infection rounds
  ST_APPLY_RUNS,   // subject-run representatives it read from the ring and hashed
  ST_APPLY_SUBJ,   // updateMembership calls it made (one per subject per receiver)
  ST_FD_DEAD_EV,   // FailureDetectorEvent(DEAD): a DEST_GONE ack (FailureDetectorImpl.java:231-235,383)
  ST_APPLY_SPILL,  // subjects k_gossip_apply merged through the spill table
  ST_APPLY_RECS,   // gossip records of batch slots k_gossip_apply_b expanded into its entry bitmap
  ST_UPDATED,      // MembershipEvent UPDATED (MembershipProtocolImpl.java:599-600)
  ST_APPLY_PAIRS,  // receiver pairs k_gossip_apply processed in two half-workgroups (SWIM_APPLY_PAIR)
  ST_COMMIT_RADIX, // commit phases sorted by the chip-wide radix sort (more than CS_SMALL gossips)
  ST_APPLY_SKIP,   // dictionary blocks k_gossip_apply_b skipped by their merge mark (no cell read)
  ST_APPLY_RBM,    // long record ranges k_gossip_apply_b ORed as a slot entry bitmap (k_slot_bm)
  ST_APPLY_RBREC,  // ... and their records
  ST_COUNT
};

enum Overflow : uint32_t {
  OV_EVENTS = 1u,
  OV_GOSSIP = 2u,
  OV_SYNC = 4u,
  OV_SPILL = 8u,  // the spill table (or a receiver's LDS spill list) is out of slots
  OV_BUCKET = 16u,
  OV_BUG = 32u,  // a device-side invariant check failed (bounded loop exhausted)
  OV_IFROM = 64u,  // infectedFrom bookkeeping out of capacity or a delivery predicted never to
                   // matter did: results would no longer be exact
  OV_TRACK = 128u,  // N x K: more subjects left the baseline than there are columns
  OV_HDX = 256u,    // 4-bit infection rounds: the escape table of rounds that do not fit is full
};

// OV_IFROM causes (Ctl::ov_detail), named in the error message
enum IfromOverflow : uint32_t {
  IF_MISPREDICT = 1u,  // a selected peer delivered within the horizon without a record (may_select)
  IF_MAXREC = 2u,      // one pair needs more than MAXREC records
  IF_PAIRS = 4u,       // pruned pairs of a round over spcap / pwcap
  IF_RECORDS = 8u,     // delivery records or their bodies over rcap / bcap within the horizon
  IF_INHIST = 16u,     // a member's in-history ring (IHCAP) wrapped inside the horizon
  IF_DELAYQ = 32u,     // a receiver's delayed-message ring (dqcap) wrapped over a message still in flight
                       // or inside the horizon
};

// the gossip-id sequence of gossips a simulated member forwards for a real node (k_deliver): a real
// node's gossip keeps its own id in the reference (GossipProtocolImpl.onGossipReq puts it under its
// gossipId, :171-183) and never advances the forwarding member's gossipCounter (:48, createAndPutGossip
// :163-169); here it is re-emitted by the forwarding member under FOREIGN_SEQ | fseq[member]
constexpr uint32_t FOREIGN_SEQ = 0x80000000u;

// the request word of a SYNC exchange record that carries a joiner's initial SYNC (MembershipProtocolImpl
// .start0, :222-257) to a seed on another shard: JOIN_REQ | joiner (periodic / FD requests are 2i + kind)
constexpr uint32_t JOIN_REQ = 0x40000000u;

constexpr uint32_t BASELINE = 1u;  // SWIM_PACK(0, SWIM_ALIVE): every view's record at the start

constexpr uint32_t STAT_SHARDS = 64;  // power of two
constexpr uint32_t STAT_STRIDE = 64;  // u64 per shard (512 B), >= ST_COUNT
static_assert(ST_COUNT <= (int)STAT_STRIDE, "stat shard too small");

// SYNC work lists are striped by local member id over SY_STRIPES counters: one counter per list
// serialised ~1,000 same-address atomics per fault-free period
constexpr uint32_t SY_STRIPES = 64;

struct Ctl {
  unsigned long long rsv_stats[ST_COUNT];
  uint32_t gcount;      // gossips ever created (ids); slot = id & (GC-1)
  uint32_t glo;         // oldest possibly-live gossip id
  uint32_t scan_lo;     // [scan_lo, scan_hi) ids scanned by the send kernel this round
  uint32_t scan_hi;
  uint32_t rsv0;
  uint32_t event_count;
  uint32_t stage_count; // staged SYNC requests this period
  uint32_t due_count;   // subject columns due for the suspicion sweep
  uint32_t overflow;
  uint32_t stg_count;   // gossips staged by emit_gossip since the last commit
  uint32_t n_stop;      // sharded: local members stopped since the last commit (stop_list)
  uint32_t n_act;       // active bitmap words this round (k_gossip_prep)
  uint32_t w_beg;       // unwrapped index of the live range's first bitmap word this round
  uint32_t n_alist;     // receivers with first receipts this round (k_gossip_pull)
  uint32_t n_inov;      // entries of in_ov this round
  uint32_t hx_live;     // hd4: escape entries left by the last k_hx_sweep (a gauge)
  uint32_t bl_hist[32]; // alive members per bit_length(others + 1) (spread/sweep bounds)
  // infectedFrom bookkeeping: monotone counters of the record pools, and the
  // pools' fill at the start of each round (mod 256), so an allocation can check that it does
  // not overwrite a record still inside the horizon
  uint32_t rec_cnt, body_cnt, sp_cnt, rp_cnt, pw_used;
  uint32_t ncols;        // N x K: columns allocated
  uint32_t alive_count;  // alive members (N x K: presence of untracked subjects)
  uint32_t ov_detail;    // which infectedFrom bound OV_IFROM hit (IfromOverflow bits)
  // gossip batches: records ever committed (the record ring's unwrapped end),
  // the ring id count before the last commit, and the batches the last chip-wide commit made
  uint32_t ccount, g_prev, rs_ncls;
  uint32_t ntrack;       // N x K: subjects listed in track_list for the coming allocation
  // record dictionary: the record count before the last commit, blocks ever
  // handed out (high-water mark), free blocks on the stack, blocks the last claim took off it, and
  // the unwrapped end of the newest record that got no dictionary entry
  uint32_t c_prev, d_hw, d_nfree, d_taken, d_none_last;
  uint32_t rs_rec[256], rs_body[256];
  uint32_t wbeg_hist[256];  // w_beg of each round's active list (act_ring)
  uint32_t xg_cnt[SWIM_MAX_WORLD];  // this round's (sender, remote peer) pairs per peer shard
  uint32_t xs_cnt[SWIM_MAX_WORLD];  // this period's SYNC requests per remote receiver shard
  uint32_t js_n;        // initial SYNCs of local joiners bound for other shards this period (jsend)
  uint32_t xr_n;        // SYNC requests received from other shards this period (k_sync_unpack)
  uint32_t sp_n;        // spill-table slots claimed this round (sp_used): cleared by k_finalize, reset by k_gossip_prep
  uint32_t ntouched;    // dense SYNC rows: touched columns listed by k_tlist for this period's SYNC
  uint32_t rb_next;     // slot entry bitmaps handed out (mod rb_cap)
  uint32_t sy_mcnt[SY_STRIPES];  // this period's SYNC receivers per work-list stripe (recv_one)
  uint32_t sy_acnt[SY_STRIPES];  // and requesters awaiting a SYNC_ACK (k_sync_select, k_join_select)
};

// act[] entry: word offset from w_beg in bits 0..25, window class in 26..27, sweep class in 28..29
constexpr uint32_t ACT_OFF_MASK = (1u << 26) - 1u;
enum WordClass : uint32_t { WC_NONE = 0, WC_MIXED = 1, WC_ALL = 2 };

// Everything a kernel needs, passed by value.
struct KP {
  // sizes / config
  uint32_t N, GC, gmask, G, S, f, kreq, rm, mult, n_seeds, time_left_pos;
  uint32_t gpow2;  // GC is a power of two (gmask = GC - 1); else ids map to slots mod GC (gmod)
  // observer-row shard of this handle: members [row0, row0 + nloc) live here;
  // view/hb/wb/nb/hd rows and dl columns are indexed by the local row m - row0
  uint32_t row0, nloc, rank, world;
  // view geometry: a row holds W cells; dense W = N (cell = subject), N x K mode (nxk = 1) W = K
  // (cell = the subject's column, colmap); an untracked subject reads as BASELINE everywhere
  uint32_t W, nxk;
  uint32_t* colmap;    // [N] subject -> column, NONE while untracked (N x K only)
  uint32_t* colsubj;   // [K] column -> subject
  uint32_t* colorder;  // [K] the allocated columns in subject order (SYNC merges walk it)
  // Touched columns of dense views: a subject whose record some row ever changed
  // from the converged BASELINE. Every other column holds BASELINE in every row, and equal records
  // never override (MembershipProtocolImpl.java:489), so SYNC / SYNC_ACK payloads carry the touched
  // columns only, in subject order (tmode: dense handles without spare slots)
  uint32_t tmode;
  uint32_t* tbits;     // [N / 32] touched columns (sharded: OR-merged by every commit exchange)
  uint32_t* tlist;     // [N] the touched columns in ascending order (k_tlist, each SYNC phase)
  uint32_t* track_req;   // [N] subject listed for a column (k_fd_track / k_track_one)
  uint32_t* track_list;  // [tcap] subjects the coming FD phase changes first (k_track_alloc)
  uint32_t tcap;
  uint32_t sweepmax;  // max gossipPeriodsToSweep + 1: last round a holder may still count a gossip
  uint32_t ecap, scap;
  uint64_t seed;
  // clock
  uint32_t period, round, phase, tick, create_round;
  // link model
  uint32_t loss_thr;  // lost iff draw < loss_thr (when 0 < loss < 100 %)
  uint32_t loss_mode; // 0 none, 1 probabilistic, 2 all lost
  uint32_t part_active;
  const uint8_t* group;
  const uint8_t* link;    // outbound block bitmap [src][dst] (send error) or nullptr
  const uint8_t* inlink;  // inbound block bitmap [dst][src] (silent drop at dst) or nullptr
  // addresses. Until the first swim_restart (rerouted == 0) member x lives at
  // address x and is reached iff alive; afterwards a message to x reaches occ[addr[x]], the running
  // member at x's address, and partition groups / blocks apply per address
  uint32_t rerouted;
  uint32_t* addr;     // [N] member -> address
  uint32_t* occ;      // [N] address -> running member or NONE (kept current in every mode)
  uint32_t* mv_head;  // [N] address -> the last member restarted on it, or NONE
  uint32_t* mv_next;  // [N] member -> the member restarted on the same address before it, or NONE
  // joins (swim_join / swim_restart) of the current period: initial SYNC to the seeds
  uint32_t njoin;     // members joining this period (0: none, the join kernels are not launched)
  uint8_t* joining;   // [N]
  uint32_t* jslot;    // [N] a joiner's SYNC staging slot (its table, one payload for every seed)
  uint32_t* jwin;     // [N] the seed member whose SYNC_ACK the joiner merges (first round trip), or NONE
  // sharded joins: initial SYNCs whose seed lives on another shard travel in the SYNC exchange as
  // records [JOIN_REQ | joiner, seed, joiner's table]; the seed's SYNC_ACK comes back in the same slot
  uint2* jsend;       // [world * nloc] {joiner, seed} of this period's initial SYNCs bound for other shards
  uint32_t* jack_ref; // [N] requester side: record index of the SYNC_ACK of a joiner's remote initial SYNC
  // state
  uint32_t* view;
  uint16_t* dl;  // [W cells][nloc observers] suspicion deadline (dl_enc; 0 = none), subject-major
  uint32_t* colmin;
  // Spill table of the gossip apply (replaces a dense [nloc][W] inbox): the lattice
  // max per (local row, cell) of the round's records that found no LDS slot / dictionary entry. Open
  // addressing on key = row * W + cell + 1; a key is claimed by CAS and never freed inside the round
  // (probe chains never break), the claimed slots are listed in sp_used and emptied after the round's
  // apply (k_spill_clear). A key that finds no slot within SP_PROBE raises OV_SPILL.
  unsigned long long* sp_key;  // [spmask + 1]
  uint32_t* sp_val;            // [spmask + 1]
  uint32_t* sp_used;           // [spmask + 1] slots claimed this round (Ctl::sp_n of them)
  uint32_t spmask;
  const uint32_t* none_last;   // [N] per subject: unwrapped end of its newest record without a
                               // dictionary entry (k_dict_entries); such a subject merges via the spill table
  uint32_t* hb;  // [N][GC/32] holds-now bitmap (set on receipt, cleared by the owner's sweep)
  uint16_t* mm;   // [N][GC/32] oldest (low byte) / newest (high byte) infection round (mod 2^8) the
                  // member holds in the word (valid while it holds any): most MIXED words resolve per
                  // member. One u16 per (member, word): a receipt word touches one line for both
  uint8_t* hd;   // [N][GC] infection round mod 2^8, valid where the hb bit is set (exact: an
                 // alive member's held entry is at most sweep+1 <= sweepmax rounds old, < 2^8).
                 // hd4 handles: [N][GC/2], per slot a 4-bit offset of the round from the slot's
                 // creation round (gc8); offset 15 = the round is in the escape table hx
  uint32_t hd4;           // infection rounds stored as 4-bit offsets
  const uint8_t* gc8;     // [GC] creation round mod 2^8 of each slot (hd4 handles)
  unsigned long long* hx; // [hxmask + 1] escape table: (1 + local row * GC + slot) << 8 | round; 0 empty
  uint32_t hxmask;
  uint32_t* wb;  // [N][GC/32] start-of-round window bitmap written by k_gossip_select (act-indexed)
  uint32_t* nb;  // [N][GC/32] first receipts of the round found by k_gossip_pull (act-indexed)
  uint32_t nsumw;  // summary words per member: min(NSUM, GC / 1024) (a list has <= GC / 32 positions)
  uint32_t* nsum;  // [N][nsumw] bit k: nb[k] != 0 this round (written for receivers with receipts)
  uint32_t* lack;  // [N][NSUM] bit k: after its sweep the member lacks a live gossip of word k of
                   // this round's list that someone may send (k_gossip_select); k_gossip_pull visits only those
  uint32_t* lack_round;  // [N] the round `lack` was last written for the member (otherwise no bitmap)
  uint32_t* cnt;
  int32_t* cnt_delta;
  uint8_t* alive;
  uint8_t* leaving;      // [N] graceful leave in progress (MembershipProtocolImpl.leaveCluster, :203-212)
  uint8_t* stopf;        // [N] the leave gossip was swept this round: stop at the round's end
  uint32_t* stop_list;   // [nloc] sharded: members of this shard stopped since the last commit; the
                         // commit exchange carries them to every shard (alive / occ are replicated)
  uint32_t* leave_slot;  // [N] ring slot of the member's leave gossip (NONE until committed)
  uint32_t* fd_epoch;
  uint32_t* fd_cursor;
  uint32_t* g_epoch;
  uint32_t* g_cursor;
  uint32_t* gseq;
  uint32_t* fseq;  // [N] gossips a member forwarded for a real node (SWIM_DELIVER_FORWARD): their own id
                   // namespace (FOREIGN_SEQ | fseq), so the member's gossipCounter (gseq) is not advanced
  uint32_t* sync_fd;
  uint32_t* peers;   // [N][f] gossip peers chosen this round
  uint32_t* npeers;  // [N]
  // Gossip batches. A ring slot holds one batch: the gossips one origin created
  // in one commit phase while no probabilistic loss is set (they travel identically), or a single
  // gossip (loss set, or batching off). Its records live in the record ring c_sr / c_hash at
  // absolute indices [g_cref.x, g_cref.y).
  uint2* g_cref;      // [GC] record range of each slot (absolute indices into c_sr, mod CC)
  uint2* g_sid;       // [GC] 16-bit entry ids: the ids of a slot whose range holds at most SID_INLINE
                      // records, copied from c_id16 after its commit (k_slot_ids), read beside g_cref
  // slot entry bitmaps: a long record range's dictionary entries as one bitmap
  // (dsids / 4 words), built once at its commit, ORed by a receiver instead of walking the ids
  uint32_t* rb_bits;  // [rb_cap][dsids / 4]
  uint32_t* rb_tag;   // [rb_cap] the range start (c_sr index) a bitmap was built for; NONE: unusable
  uint32_t* g_rb;     // [GC] a slot's bitmap (rb_tag must still name its range), or NONE
  uint32_t rb_cap;    // bitmaps in the pool (a ring: a newer range takes the oldest)
  uint2* c_sr;        // [CC] (subject, packed record) of every gossip of a live slot
  uint32_t* c_hash;   // [CC] its canonical id hash (GossipProtocolImpl.generateGossipId, :211-213)
  uint32_t cmask;     // CC - 1
  uint32_t* wsum;     // [GC/32] gossips in a word's slots (counters weight a slot by its gossips)
  uint16_t* scnt;     // [GC] gossips of each slot (SCNT_SAT: that many or more, read g_cref), by word: a
                      // window's count is 4 x 16-B loads and masked adds, not one g_cref load per slot
  uint32_t batch_commit;  // this phase's commit groups gossips into batches by origin (loss_mode != 1)
  uint32_t batched;       // batching is on and has been used: counters weight slots, apply expands records
  uint32_t trace;         // swim_trace mask: SWIM_TRACE_FD puts FailureDetectorEvents into the event ring
  // member metadata (Cluster.updateMetadata, ClusterImpl.java:364-367): each member's current
  // version, and per (observer, cell) the version the observer fetched last (MetadataStoreImpl
  // membersMetadata). meta_view is allocated by the first swim_update_metadata: until then every
  // version is the initial one and no ALIVE record can carry different metadata.
  uint32_t* meta_cur;   // [N]
  uint32_t* meta_view;  // [nloc][W] or nullptr
  // Record dictionary: every distinct (subject, record) of the live record ring
  // is an entry of its subject's block of DICT_WAYS entries; c_id names each ring record's entry,
  // so a receiver ORs one bit per received record into an LDS bitmap and merges per block.
  uint32_t* sid_of;   // [N] subject -> its block, NONE
  uint32_t dsids;     // subject blocks (swim_config.dict_subjects; DICT_SIDS by default)
  uint32_t* d_subj;   // [dsids] block -> subject, NONE while free
  uint32_t* d_rec;    // [dsids * DICT_WAYS] packed record of each entry, 0 = empty (no record packs to 0)
  uint32_t* d_last;   // [dsids * DICT_WAYS] unwrapped index + 1 of the newest ring record naming the entry
  uint32_t* d_free;   // [dsids] stack of free blocks
  uint32_t* c_id;     // [CC] entry of each record-ring record; ID_USER, or ID_NONE (slow path)
  uint16_t* c_id16;   // [CC] the same as 16-bit ids (cid16: dictionaries of <= 8,192 blocks; ID16_USER,
                      // ID16_NONE): a 16-B load carries 8 records' entries instead of 4
  uint32_t cid16;
  // Merge marks of the batched apply: per (local row, block) the entries whose
  // records the receiver already found not to override its (present) cell, tagged with the block's
  // generation: mark = gen24 << 8 | way mask. A block's generation moves whenever one of its entries
  // is emptied or the block is freed (k_dict_free), and a removal of the cell clears the mark
  // (mark_clear), so a valid mark's entries are <= the cell: cells only grow while present.
  uint32_t* dmark;    // [nloc][dsids] or nullptr (no dictionary)
  uint32_t* d_gen;    // [dsids] generation of each block (low 24 bits never 0)
  uint2* g_sr;        // [GC] (subject, packed record) of each slot's first gossip (the gossip itself
                      // for a one-gossip slot)
  uint32_t* runw;     // [GC/32] bit s: slot s starts a run of one subject (a commit sorts its gossips
                      // by (subject, record), so within a run records ascend)
  uint32_t* g_hash;
  uint32_t* g_create;
  uint32_t* wlast;    // [GC/32] max infection round of any holder over the word's slots
  uint32_t* in_cnt;   // [N] senders that picked member p this round (k_gossip_select)
  uint32_t* in_list;  // [N][INCAP] the first INCAP of them
  uint32_t* in_ov;    // [N*f][2] (receiver, sender) pairs beyond INCAP
  uint32_t* alist;    // [N] receivers with first receipts this round
  uint32_t* act;      // [GC/32] active words of this round (k_gossip_prep): its slot of act_ring
  uint32_t* act_ring; // [256][astride] the active lists of the last 256 rounds (infectedFrom records)
  uint32_t astride;
  uint2* actpos;      // [GC/32] per ring word: {round it was last listed, its list position}
  uint32_t* held;     // [N] live gossips each member holds (GossipProtocolImpl.gossips.size())
  uint32_t* due;
  swim_event* events;
  uint32_t* pres;
  uint32_t* last_removed;
  // sync staging
  uint32_t* req_to;     // [2N] receiver of request 2i+k, or NONE
  uint32_t* req_stage;  // [2N] staging slot, or NONE
  uint32_t* stage_req;  // [scap] request index of a staging slot
  uint32_t* stage_sync; // [scap][N] SYNC payload (sender's table)
  uint32_t* stage_ack;  // [scap][N] SYNC_ACK payload (receiver's table after the merge)
  uint32_t* recv_count; // [N]
  uint32_t* recv_off;   // [N+1]
  uint32_t* recv_fill;  // [N]
  uint32_t* bucket;     // [scap]
  uint32_t* sy_mlist;   // [SY_STRIPES][sy_cap] local receivers of this period's SYNCs (k_sync_merge's work)
  uint32_t* sy_alist;   // [SY_STRIPES][sy_cap] local requesters that may take a SYNC_ACK (k_sync_ack's work)
  uint32_t sy_cap;      // ceil(nloc / SY_STRIPES): a stripe's capacity (a member is listed once per list)
  uint4* stg;         // [stg_cap] gossips created since the last commit: origin, subject, record, id hash
  uint32_t stg_cap;
  // cross-shard exchange (world > 1)
  const uint32_t* blx;  // global (max bit_length, 32 - min bit_length) after the round's all-reduce
  uint32_t* xsend;      // host-attached device buffers of the current exchange
  const uint32_t* xrecv;
  uint32_t nneed;       // words of a need bitmap over this round's active list
  uint32_t* rpairs;     // [(N-nloc)*f][2] received (sender, receiver) pairs of the round
  uint32_t* rneed;      // [pairs][W32/32] per pair: active words the receiver lacks something in
  uint32_t* rpref;      // [pairs][W32/32] exclusive prefix of the need bits' popcounts
  uint32_t* rtot;       // [pairs] needed words per received pair
  uint32_t* roff;       // [pairs] where its window words start in the received buffer
  uint32_t* wcnt;       // [nloc*f] words each sent pair ships
  uint32_t* woff;       // [nloc*f + 1] exclusive scan of wcnt
  uint32_t* xg_pend;    // [world][nloc*f][2] (sender, remote peer) pairs of the round
  uint32_t* xs_pend;    // [world][2*nloc] SYNC requests bound for each remote shard
  uint32_t* rs_ref;     // [2N] receiver side: record index of remote request q
  uint32_t* ack_ref;    // [2N] requester side: record index of the SYNC_ACK of remote request q
  // GossipState.infectedFrom (GossipState.java:17, GossipProtocolImpl.java:181,248), DESIGN.md §3.9
  uint32_t hzn;        // rounds a delivery can still suppress a send: gossipPeriodsToSpread(N) + 1
  uint32_t apply_hlog; // k_gossip_apply's LDS table: 2^apply_hlog slots (<= 2^SWIM_APPLY_HLOG)
  unsigned long long* dbg_send;  // [2N] debug: per sender, GossipRequests to alive peers before / by infectedFrom
  uint32_t dbg_watch;            // debug: member whose per-round sends go to dbg_log (NONE: off)
  uint32_t* dbg_log;             // [256][8] round, window bits, alive peers, peers, peer ids x3, suppressed
  uint4* ih;           // [nloc][IHCAP] in-history ring: {sender, round, record or NONE, 0}
  uint32_t* ih_head;   // [N] entries ever appended
  uint32_t* ih_snd;    // [nloc][IHCAP] the sender of each entry: select scans these 4 B only
  uint32_t* ih_rhead;  // [nloc][256] ih_head at the start of each round's k_gossip_inhist (mod 256)
  uint4* rec_hdr;      // [RCAP] delivery records: {deliverer, owner (receiver), round, body offset}
  uint32_t* rec_len;   // [RCAP] body words (the active list length of that round)
  uint32_t* rec_body;  // [BCAP] per position of that round's active list: the gossips delivered
  uint32_t rcap, bcap; // powers of two
  uint4* sp_list;      // [SPCAP] this round's pruned pairs: {sender, peer, records, window offset}
  uint32_t* sp_recs;   // [SPCAP][MAXREC] their records
  uint32_t* pw;        // [PWCAP] per pruned pair, its window over this round's active list
  uint4* rp_list;      // [SPCAP] this round's recorded deliveries: {in_list entry, receiver, record, sender}
  uint32_t spcap, pwcap;
  uint32_t* sp_dq;     // [SPCAP] the pair's sender also delivered delayed messages (k_gossip_pairdelay)
  // message delays (NetworkEmulator meanDelay); delay_on = 0: every message is
  // handled in the phase it was sent in, as before
  uint32_t delay_on;
  const uint32_t* dthr;  // [dthr_n] dthr[k]: the smallest 32-bit draw whose delay is >= k ms
  uint32_t dthr_n;
  uint32_t gint, pto, pint, mto;  // gossip interval, ping timeout, ping interval, metadata timeout (ms)
  uint4* dq;             // [nloc][dqcap] per receiver: delayed GossipRequests {sender, slot, arrival round, flags}
  uint32_t* dq_head;     // [N] entries ever appended
  uint32_t* dq_rhead;    // [nloc][256] dq_head at the start of each round's pull (mod 256)
  uint32_t dqcap;        // power of two
  uint32_t dq_live;      // rounds an entry can matter after it was pushed: longest delay + horizon + 1
  Ctl* ctl;
  unsigned long long* stat_shards;  // [STAT_SHARDS][STAT_STRIDE]
};

// Debug builds (-DSWIM_DEBUG_BOUNDS, tools/gpu_debug.sh): an index past its array prints the site
// and is redirected to element 0 instead of faulting the device. Release builds: the index as is.
#ifdef SWIM_DEBUG_BOUNDS
#define DBG_IDX(idx, cap, site)                                                                              \
  (((size_t)(idx) < (size_t)(cap))                                                                          \
       ? (size_t)(idx)                                                                                      \
       : (printf("swimhip bounds: %s idx %llu cap %llu block %u thread %u round %u\n", site,                \
                 (unsigned long long)(idx), (unsigned long long)(cap), blockIdx.x, threadIdx.x, P.round),   \
          (size_t)0))
#else
#define DBG_IDX(idx, cap, site) (idx)
#endif

__device__ __forceinline__ size_t lrow(const KP& P, uint32_t m) { return (size_t)(m - P.row0); }
__device__ __forceinline__ bool is_local(const KP& P, uint32_t m) { return m - P.row0 < P.nloc; }
// a receipt of word `mi` at infection round `round`: the newest round the member holds in the word,
// and (first holding: `first`) the oldest too — one u16 store, else the high byte alone
__device__ __forceinline__ void mm_received(const KP& P, size_t mi, bool first, uint32_t round) {
  if (first)
    P.mm[mi] = (uint16_t)((round & 0xFFu) * 0x101u);
  else
    reinterpret_cast<uint8_t*>(P.mm)[2u * mi + 1u] = (uint8_t)round;
}

// the cell of subject j in a row (dense: j itself; N x K: its column or NONE while untracked)
__device__ __forceinline__ uint32_t col_of(const KP& P, uint32_t j) { return P.nxk ? P.colmap[j] : j; }
__device__ __forceinline__ uint32_t subj_of(const KP& P, uint32_t c) { return P.nxk ? P.colsubj[c] : c; }
// cells in use per row: dense N, N x K the columns allocated so far
__device__ __forceinline__ uint32_t ncells(const KP& P);
// observer obs's record of subject j (membershipTable.get, MembershipProtocolImpl.java:487)
__device__ __forceinline__ uint32_t cell_get(const KP& P, uint32_t obs, uint32_t j) {
  const uint32_t c = col_of(P, j);
  return c == 0xFFFFFFFFu ? BASELINE : P.view[lrow(P, obs) * P.W + c];
}

constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint32_t NONE_U32 = NONE;

// record dictionary geometry; tests build a variant with a tiny one
#ifndef SWIM_DICT_SIDS
#define SWIM_DICT_SIDS 8192
#endif
constexpr uint32_t DICT_SIDS = SWIM_DICT_SIDS;   // subject blocks by default (swim_config.dict_subjects)
constexpr uint32_t DICT_WAYS = 8;                // distinct live records per subject
constexpr uint32_t DICT_IDS = DICT_SIDS * DICT_WAYS;
constexpr uint32_t DICT_WORDS = DICT_IDS / 32u;  // a receiver's entry bitmap
constexpr uint32_t ID_USER = 0xFFFFFFFEu;        // c_id of a user gossip (subject >= N)
constexpr uint32_t ID_NONE = NONE;               // c_id of a record that found no entry
constexpr uint32_t ID16_USER = 0xFFFEu, ID16_NONE = 0xFFFFu;  // their 16-bit forms (c_id16): entry ids of
                                                               // 16-bit handles stay below 0xFFFE
constexpr uint32_t DICT_LOCK = 0xFFFFFFFEu;      // sid_of while k_dict_claim allocates the block
// sid_of of a subject whose claim found no block: DICT_NOBLK | (the commit's first record index &
// DICT_TAG_MASK); a later commit may claim again (k_dict_claim). Never a block id (< 2^20).
constexpr uint32_t DICT_NOBLK = 0x80000000u;
constexpr uint32_t DICT_TAG_MASK = 0x3FFFFFFFu;
static_assert(DICT_SIDS >= 4 && (DICT_SIDS & (DICT_SIDS - 1)) == 0 && DICT_SIDS <= (1u << 16),
              "SWIM_DICT_SIDS: a power of two in 4 .. 65536");


// Ring slot of gossip id `id` and ring word of unwrapped word index `wi`. A power-of-two ring masks;
// any other multiple of 1,024 slots (C4's 5,128 * 1,024: DESIGN.md §4.2) takes the remainder, and its ids
// must not wrap 2^32 (k_commit raises OV_GOSSIP before they do)
__device__ __forceinline__ uint32_t gmod(const KP& P, uint32_t id) { return P.gpow2 ? (id & P.gmask) : id % P.GC; }
__device__ __forceinline__ uint32_t wmod(const KP& P, uint32_t wi) {
  return P.gpow2 ? (wi & ((P.GC >> 5) - 1u)) : wi % (P.GC >> 5);
}

// the unwrapped index of the live record ring's first record: the oldest possibly-live slot's
// first one (the ring's end when no slot is live)
__device__ __forceinline__ uint32_t live_rec_lo(const KP& P) {
  const uint32_t glo = P.ctl->glo, g0 = P.ctl->gcount;
  return (g0 != glo && g0 - glo <= P.GC) ? P.g_cref[gmod(P, glo)].x : P.ctl->ccount;
}

// the member whose transport receives a message sent to member x (TransportImpl sends to
// member.address()): x itself while alive, or after a restart on x's address the new member
__device__ __forceinline__ uint32_t route(const KP& P, uint32_t x) {
  return P.rerouted ? P.occ[P.addr[x]] : (P.alive[x] ? x : NONE);
}
__device__ __forceinline__ uint32_t addr_of(const KP& P, uint32_t x) { return P.rerouted ? P.addr[x] : x; }
constexpr uint32_t REMOTE = 0xFFFFFFFEu;   // req_stage of a request staged on another shard
constexpr uint32_t XREC = 0x80000000u;     // in_list entry: a received window record, not a local row
constexpr uint32_t INCAP = 16;  // in_list slots per receiver per round (random peers: in-degree ~ f)
constexpr uint32_t NSUM = 1024;  // receipt-summary words per receiver: active lists up to 32,768 words
constexpr uint32_t SPAIR = 0x40000000u;  // in_list entry: a pruned pair (window in pw), not a member id
constexpr uint32_t IHCAP = 512;  // in-history entries per member (~f per round over the horizon: ~2 f hzn,
                                 // with the in-degree tail of 10^6 members)
constexpr uint32_t MAXREC = 16;  // records one pruned pair may carry
constexpr uint32_t DQ_ARRIVED = 1u;      // delayed-message entry flag: handled by its receiver

// The positions [*lo, *hi) of receiver p's delayed-message ring that can still matter in this
// round: pushed within the last dq_live rounds (an older entry arrived and left the infectedFrom
// horizon), and still in the ring. A stale head of a round p's pull did not run in is older,
// so the window only grows (still exact).
__device__ __forceinline__ void dq_window(const KP& P, uint32_t p, uint32_t* lo, uint32_t* hi) {
  const uint32_t h = P.dq_head[p];
  uint32_t l = h > P.dqcap ? h - P.dqcap : 0u;
  if (P.round >= P.dq_live) {
    const uint32_t l1 = P.dq_rhead[lrow(P, p) * 256u + ((P.round - P.dq_live) & 255u)];
    if (l1 > l && l1 <= h) l = l1;
  }
  *lo = l;
  *hi = h;
}
constexpr uint32_t DQ_PAIR = 0x10000u;   // k_gossip_select: the chosen peer delivered delayed messages
#define SWIM_PCHUNK 256  // (1,024: C2 4.64 -> 4.25 ms per period at 256, C4's schedule and C3 a little faster too)
constexpr uint32_t PCHUNK = SWIM_PCHUNK;  // active-list positions per wave in the infectedFrom kernels
static_assert(PCHUNK % 64u == 0u, "SWIM_PCHUNK: a multiple of 64");

__device__ __forceinline__ void ifrom_overflow(const KP& P, uint32_t why) {
  atomicOr(&P.ctl->overflow, OV_IFROM);
  atomicOr(&P.ctl->ov_detail, why);
}

// ctl->ncols counts every column request, including the ones k_track_alloc refused with OV_TRACK:
// clamp to the K columns that exist, so no kernel run after an overflow indexes past them
__device__ __forceinline__ uint32_t ncells(const KP& P) {
  if (!P.nxk) return P.N;
  const uint32_t n = P.ctl->ncols;
  return n < P.W ? n : P.W;
}

// this period's SYNC payloads carry the touched columns only (in tlist order)
__device__ __forceinline__ bool tlisted(const KP& P) { return P.tmode && P.ctl->ntouched < P.N; }
// cells of a SYNC / SYNC_ACK payload row: the listed touched columns, else the row's cells in use
// (dense N, N x K the allocated columns)
__device__ __forceinline__ uint32_t sync_cells(const KP& P) { return tlisted(P) ? P.ctl->ntouched : ncells(P); }
// the words of one cross-shard SYNC record: request, receiver, then the payload
__device__ __forceinline__ size_t sync_rec_words(const KP& P) { return (tlisted(P) ? P.ctl->ntouched : P.W) + 2u; }

// gossips in the slots `bits` of bitmap word ws (GossipRequest / receipt counters count gossips,
// not slots): popcount while every slot holds one gossip, else the word's total when the mask
// covers it, else the slots' record ranges one by one
// scnt saturates here (a test build lowers it so the exact fallback runs)
#ifndef SWIM_SCNT_SAT
#define SWIM_SCNT_SAT 0xFFFF
#endif
constexpr uint32_t SCNT_SAT = SWIM_SCNT_SAT;
static_assert(SCNT_SAT >= 1u && SCNT_SAT <= 0xFFFFu, "SWIM_SCNT_SAT: 1 .. 65535");
__device__ __forceinline__ uint32_t slot_gossips(const KP& P, uint32_t ws, uint32_t bits) {
  if (!P.batched || !bits) return (uint32_t)__popc(bits);
  if (bits == 0xFFFFFFFFu) return P.wsum[ws];
  const uint4* cp = reinterpret_cast<const uint4*>(P.scnt + (size_t)ws * 32u);
  const uint4 c0 = cp[0], c1 = cp[1], c2 = cp[2], c3 = cp[3];  // all in flight together
  const uint32_t cw[16] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w,
                           c2.x, c2.y, c2.z, c2.w, c3.x, c3.y, c3.z, c3.w};
  uint32_t n = 0, big = 0;
#pragma unroll
  for (uint32_t q = 0; q < 16u; ++q) {
    const uint32_t lo = cw[q] & 0xFFFFu, hi = cw[q] >> 16;
    if ((bits >> (2u * q)) & 1u) {
      n += lo;
      big |= (lo == SCNT_SAT ? 1u : 0u) << (2u * q);
    }
    if ((bits >> (2u * q + 1u)) & 1u) {
      n += hi;
      big |= (hi == SCNT_SAT ? 1u : 0u) << (2u * q + 1u);
    }
  }
  while (big) {  // slots of SCNT_SAT gossips or more (a SYNC merge of a huge table): their exact count
    const uint32_t b = (uint32_t)__builtin_ctz(big);
    big &= big - 1u;
    const uint2 r = P.g_cref[ws * 32u + b];
    n += (r.y - r.x) - SCNT_SAT;
  }
  return n;
}

__device__ __forceinline__ uint32_t nibble_bytes(uint32_t n);

// ---- 4-bit infection rounds (hd4 handles) --------------------------------------
// A holder's infection round of slot s is never before the slot's creation round and, in a storm,
// a few rounds after it: the offset (round - creation) mod 2^8 is kept in 4 bits, and an offset of
// 15 or more goes to an open-addressing escape table keyed by (local row, slot). Decoding gives back
// exactly the bytes an 8-bit handle stores, so every age test is shared. A stale escape entry (its
// slot swept or rewritten with a small offset) is never read: lookups happen only for nibble 15,
// which is written together with a fresh entry; k_hx_sweep tombstones stale entries once a period.
constexpr unsigned long long HX_EMPTY = 0ull, HX_TOMB = ~0ull;
constexpr uint32_t HX_PROBE = 64;  // linear-probe bound; beyond it OV_HDX
__device__ __forceinline__ uint32_t hx_home(const KP& P, unsigned long long key) {
  return (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> 32) & P.hxmask;
}
// the escaped round of (row, slot); writers: the row's own wave (apply / commit), never two at once
__device__ __forceinline__ void hx_put(const KP& P, size_t row, uint32_t s, uint32_t round) {
  const unsigned long long key = 1ull + (unsigned long long)row * P.GC + s;
  const unsigned long long e = (key << 8) | (round & 0xFFu);
  uint32_t h = hx_home(P, key), tomb = NONE_U32;
  for (uint32_t k = 0; k < HX_PROBE; ++k, h = (h + 1u) & P.hxmask) {
    const unsigned long long v = P.hx[h];
    if (v == HX_TOMB) {
      if (tomb == NONE_U32) tomb = h;
      continue;
    }
    if (v != HX_EMPTY && (v >> 8) == key) {  // the key's entry: overwrite
      P.hx[h] = e;
      return;
    }
    if (v == HX_EMPTY) {  // not in the table: take the first tombstone passed, else this slot
      if (tomb != NONE_U32 && atomicCAS(&P.hx[tomb], HX_TOMB, e) == HX_TOMB) return;
      if (atomicCAS(&P.hx[h], HX_EMPTY, e) == HX_EMPTY) return;
      k = 0;  // lost a race for the slot: start over (bounded: each retry fills a slot)
      h = hx_home(P, key) - 1u;
      tomb = NONE_U32;
    }
  }
  atomicOr(&P.ctl->overflow, OV_HDX);
}
__device__ __forceinline__ uint32_t hx_get(const KP& P, size_t row, uint32_t s) {
  const unsigned long long key = 1ull + (unsigned long long)row * P.GC + s;
  uint32_t h = hx_home(P, key);
  for (uint32_t k = 0; k < HX_PROBE; ++k, h = (h + 1u) & P.hxmask) {
    const unsigned long long v = P.hx[h];
    if (v == HX_EMPTY) break;
    if (v != HX_TOMB && (v >> 8) == key) return (uint32_t)(v & 0xFFu);
  }
  atomicOr(&P.ctl->overflow, OV_BUG);  // a nibble 15 always has its entry
  return 0u;
}
// bytes b of a and b added mod 2^8 each
__device__ __forceinline__ uint32_t bytes_add(uint32_t a, uint32_t b) {
  return ((a & 0x7F7F7F7Fu) + (b & 0x7F7F7F7Fu)) ^ ((a ^ b) & 0x80808080u);
}
// the 32 infection rounds (mod 2^8) of word ws of local row `row`, as hd stores them (byte b of
// the 8 dwords = slot b); only the bytes of held slots mean anything. hd4: escapes are looked up for
// the slots of `need` only (held slots whose rounds the caller uses: a slot no longer held may keep a
// stale nibble 15 whose entry is gone)
template <bool HD4>
__device__ __forceinline__ void hd_load32(const KP& P, size_t row, uint32_t ws, uint4& d0, uint4& d1,
                                          uint32_t need = 0xFFFFFFFFu) {
  if (!HD4) {
    const uint4* dp = reinterpret_cast<const uint4*>(P.hd + row * P.GC + (size_t)ws * 32u);
    d0 = dp[0];
    d1 = dp[1];
    return;
  }
  const uint4 nb = *reinterpret_cast<const uint4*>(P.hd + row * (P.GC / 2u) + (size_t)ws * 16u);
  const uint4* gp = reinterpret_cast<const uint4*>(P.gc8 + (size_t)ws * 32u);
  const uint4 g0 = gp[0], g1 = gp[1];
  const uint32_t n[4] = {nb.x, nb.y, nb.z, nb.w};
  uint32_t o[8];
#pragma unroll
  for (uint32_t q = 0; q < 4u; ++q) {  // nibbles 8q .. 8q+7 -> bytes of dwords 2q, 2q+1
    const uint32_t lo = n[q] & 0x0F0F0F0Fu, hi = (n[q] >> 4) & 0x0F0F0F0Fu;
    o[2 * q] = __builtin_amdgcn_perm(hi, lo, 0x05010400u);      // lo.b0 hi.b0 lo.b1 hi.b1
    o[2 * q + 1] = __builtin_amdgcn_perm(hi, lo, 0x07030602u);  // lo.b2 hi.b2 lo.b3 hi.b3
  }
  const uint32_t g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
  uint32_t esc[8];
#pragma unroll
  for (uint32_t q = 0; q < 8u; ++q) {
    // bytes equal to 15 (escaped): x = o ^ 0x0F is zero there; exact per byte (no borrow crosses)
    const uint32_t x = o[q] ^ 0x0F0F0F0Fu;
    esc[q] = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u & nibble_bytes((need >> (4u * q)) & 0xFu);
    o[q] = bytes_add(o[q], g[q]);
  }
#pragma unroll
  for (uint32_t q = 0; q < 8u; ++q)
    while (esc[q]) {  // rare: rounds too far from the slot's creation
      const uint32_t bb = (uint32_t)__builtin_ctz(esc[q]) >> 3;
      esc[q] &= esc[q] - 1u;
      const uint32_t r = hx_get(P, row, ws * 32u + 4u * q + bb);
      o[q] = (o[q] & ~(0xFFu << (8u * bb))) | (r << (8u * bb));
    }
  d0 = make_uint4(o[0], o[1], o[2], o[3]);
  d1 = make_uint4(o[4], o[5], o[6], o[7]);
}
// store the rounds d0/d1 (byte per slot) of the slots in `mask` of word ws; the other slots of the
// word keep what they hold (their bytes in d0/d1 are ignored: hd4 merges nibbles into the stored word)
template <bool HD4>
__device__ __forceinline__ void hd_store32(const KP& P, size_t row, uint32_t ws, uint32_t mask, uint4 d0, uint4 d1) {
  if (!mask) return;
  if (!HD4) {
    uint4* dp = reinterpret_cast<uint4*>(P.hd + row * P.GC + (size_t)ws * 32u);
    if (mask & 0xFFFFu) dp[0] = d0;
    if (mask >> 16) dp[1] = d1;
    return;
  }
  uint4* np = reinterpret_cast<uint4*>(P.hd + row * (P.GC / 2u) + (size_t)ws * 16u);
  const uint4* gp = reinterpret_cast<const uint4*>(P.gc8 + (size_t)ws * 32u);
  const uint4 g0 = gp[0], g1 = gp[1];
  const uint32_t g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
  const uint32_t d[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
  uint4 cur = make_uint4(0u, 0u, 0u, 0u);
  if (mask != 0xFFFFFFFFu) cur = *np;
  uint32_t n[4] = {cur.x, cur.y, cur.z, cur.w};
#pragma unroll
  for (uint32_t b = 0; b < 32u; ++b) {
    if (!((mask >> b) & 1u)) continue;
    const uint32_t r = (d[b >> 2] >> (8u * (b & 3u))) & 0xFFu;
    uint32_t off = (r - ((g[b >> 2] >> (8u * (b & 3u))) & 0xFFu)) & 0xFFu;
    if (off >= 15u) {
      hx_put(P, row, ws * 32u + b, r);
      off = 15u;
    }
    const uint32_t sh = 4u * (b & 7u);
    n[b >> 3] = (n[b >> 3] & ~(0xFu << sh)) | (off << sh);
  }
  *np = make_uint4(n[0], n[1], n[2], n[3]);
}

// onGossipReq's new-gossip branch for the slots `bits` of word ws of local row `row`: their
// infection round becomes `round`; the word's other held slots (`prior`) keep theirs. v0 / v1 are
// the word's current rounds (8-bit handles: a 16-slot half is rewritten whole, so it needs them
// when it keeps some; hd4 handles merge nibbles themselves and ignore them).
template <bool HD4>
__device__ __forceinline__ void hd_receive(const KP& P, size_t row, uint32_t ws, uint32_t bits, uint32_t prior,
                                           uint4 v0, uint4 v1, uint32_t round) {
  const uint32_t rb = (round & 0xFFu) * 0x01010101u;
  if (HD4) {
    hd_store32<true>(P, row, ws, bits, make_uint4(rb, rb, rb, rb), make_uint4(rb, rb, rb, rb));
    return;
  }
  uint4* dp = reinterpret_cast<uint4*>(P.hd + row * P.GC + (size_t)ws * 32u);
#pragma unroll
  for (int q = 0; q < 2; ++q) {  // 16 slots per 16 B
    const uint32_t nb16 = (bits >> (16 * q)) & 0xFFFFu;
    if (!nb16) continue;
    if (!((prior >> (16 * q)) & 0xFFFFu)) {  // nothing held in these 16 slots: bytes of slots not
      dp[q] = make_uint4(rb, rb, rb, rb);   // held are never read, so no read-modify-write
      continue;
    }
    uint4 v = q == 0 ? v0 : v1;
    const uint32_t m0 = nibble_bytes(nb16 & 0xFu), m1 = nibble_bytes((nb16 >> 4) & 0xFu);
    const uint32_t m2 = nibble_bytes((nb16 >> 8) & 0xFu), m3 = nibble_bytes(nb16 >> 12);
    v.x = (v.x & ~m0) | (rb & m0);
    v.y = (v.y & ~m1) | (rb & m1);
    v.z = (v.z & ~m2) | (rb & m2);
    v.w = (v.w & ~m3) | (rb & m3);
    dp[q] = v;
  }
}

__device__ __forceinline__ bool bit_at(const uint8_t* bm, uint64_t bit) {
  return bm && (bm[bit >> 3] & (1u << (bit & 7)));
}

// Partition cut and directed blocks only (no liveness, no loss draw): can a message src -> dst
// reach dst's handlers? An outbound block (NetworkEmulator.blockOutbound, :105-119) fails the
// send; an inbound block at dst (blockInbound, :255-269) drops it silently
// (NetworkEmulatorTransport.java:73-77). For one-way messages both just lose the message.
__device__ __forceinline__ bool link_open(const KP& P, uint32_t src, uint32_t dst) {
  src = addr_of(P, src);
  dst = addr_of(P, dst);
  if (P.part_active && P.group[src] != P.group[dst]) return false;
  if (bit_at(P.link, (uint64_t)src * P.N + dst)) return false;
  return !bit_at(P.inlink, (uint64_t)dst * P.N + src);
}

// Sender side (tryFailOutbound, NetworkEmulator.java:166-180): false = the send fails at once
// (loss draw, blocked destination / partition cut, stopped transport on either end).
// src / dst are the member ids the message is addressed from / to; the loss draw is keyed by the
// two processes that send and receive it (route).
__device__ __forceinline__ bool out_ok(const KP& P, uint32_t kind, uint32_t src, uint32_t dst, uint32_t c,
                                       uint32_t tick) {
  uint32_t rs = src, rd = dst;
  if (P.rerouted) {
    rs = route(P, src);
    rd = route(P, dst);
    if (rs == NONE || rd == NONE) return false;
    src = P.addr[src];
    dst = P.addr[dst];
  } else if (!P.alive[src] || !P.alive[dst]) {
    return false;
  }
  if (P.part_active && P.group[src] != P.group[dst]) return false;
  if (bit_at(P.link, (uint64_t)src * P.N + dst)) return false;
  if (P.loss_mode == 0) return true;
  if (P.loss_mode == 2) return false;
  return draw1(P.seed, kind, rs, rd, c, tick) >= P.loss_thr;
}

// Receiver side: dst's inbound filter on the message's sender (NetworkEmulatorTransport.java:64-68,73-77).
__device__ __forceinline__ bool in_ok(const KP& P, uint32_t dst, uint32_t src) {
  return !bit_at(P.inlink, (uint64_t)addr_of(P, dst) * P.N + addr_of(P, src));
}

__device__ __forceinline__ bool delivered(const KP& P, uint32_t kind, uint32_t src, uint32_t dst, uint32_t c,
                                          uint32_t tick) {
  return out_ok(P, kind, src, dst, c, tick) && in_ok(P, dst, src);
}

// NetworkEmulator.evaluateDelay (NetworkEmulator.java:358-368) of a message whose draw's second
// word is u: (long)(-ln(1 - u/2^32) * meanDelay) ms, as the largest k with dthr[k] <= u (the host
// computes the table once; integer compares only, so the oracle and the device agree exactly).
__device__ __forceinline__ uint32_t delay_of_draw(const KP& P, uint32_t u) {
  uint32_t lo = 0, hi = P.dthr_n;  // dthr[0] = 0 <= u
  while (hi - lo > 1u) {
    const uint32_t mid = (lo + hi) >> 1;
    if (P.dthr[mid] <= u)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}
// the delay of message src -> dst (tryDelayOutbound, NetworkEmulator.java:189-201): the same draw as
// its loss (keyed by the two processes), second word
__device__ __forceinline__ uint32_t msg_delay(const KP& P, uint32_t kind, uint32_t src, uint32_t dst, uint32_t c,
                                              uint32_t tick) {
  if (!P.delay_on) return 0u;
  const uint32_t rs = route(P, src), rd = route(P, dst);
  if (rs == NONE || rd == NONE) return 0u;
  return delay_of_draw(P, draw4(P.seed, kind, rs, rd, c, tick).y);
}

__device__ __forceinline__ uint32_t susp_periods(const KP& P, uint32_t others) { return P.mult * bitlen(others + 1u); }
__device__ __forceinline__ uint32_t spread_rounds(const KP& P, uint32_t others) { return P.rm * bitlen(others + 1u); }
__device__ __forceinline__ uint32_t sweep_rounds(const KP& P, uint32_t others) {
  return 2u * (spread_rounds(P, others) + 1u);
}

__device__ __forceinline__ void push_event(const KP& P, uint32_t obs, uint32_t subj, uint32_t type, uint32_t reason,
                                           uint32_t record) {
  if (P.ecap == 0) return;
  const uint32_t idx = atomicAdd(&P.ctl->event_count, 1u);
  if (idx >= P.ecap) {
    atomicOr(&P.ctl->overflow, OV_EVENTS);
    return;
  }
  swim_event e;
  e.period = P.period;
  e.observer = obs;
  e.subject = subj;
  e.record = record;
  e.type = (uint8_t)type;
  e.reason = (uint8_t)reason;
  e.phase = (uint8_t)P.phase;
  e.pad = 0;
  P.events[idx] = e;
}

struct Tally {
  uint32_t accepted = 0, refut = 0, added = 0, removed = 0, updated = 0;
};

// GossipProtocolImpl.spread -> createAndPutGossip (GossipProtocolImpl.java:124-128,163-169),
// first half: stage the gossip. k_gossip_commit gives it a ring slot after the phase (on every
// shard, in shard order), publishes the record, and the origin holds it from `create_round`.
__device__ __forceinline__ void emit_gossip(const KP& P, uint32_t origin, uint32_t subject, uint32_t record,
                                            uint32_t seq) {
  const uint32_t idx = atomicAdd(&P.ctl->stg_count, 1u);
  if (idx >= P.stg_cap) {
    atomicOr(&P.ctl->overflow, OV_GOSSIP);
    return;
  }
  P.stg[idx] = make_uint4(origin, subject, record, gossip_hash(origin, seq));
}

// MetadataStoreImpl.fetchMetadata (MetadataStoreImpl.java:151-193) as a liveness round trip; the
// process at the subject's address answers only requests for its own id (:216-223).
__device__ __forceinline__ bool fetch_ok(const KP& P, uint32_t obs, uint32_t subj, uint32_t attempt) {
  if (P.rerouted && route(P, subj) != subj) return false;
  if (!delivered(P, K_MREQ, obs, subj, attempt, P.tick) || !delivered(P, K_MRESP, subj, obs, attempt, P.tick))
    return false;
  // with message delays the round trip must come back within metadataTimeout (:170)
  return !P.delay_on ||
         msg_delay(P, K_MREQ, obs, subj, attempt, P.tick) + msg_delay(P, K_MRESP, subj, obs, attempt, P.tick) < P.mto;
}

// the spill table (KP::sp_key): the record's lattice max into (receiver p, cell c); returns the slot,
// *first = this call claimed the key (its caller lists the slot for the round's merge)
constexpr uint32_t SP_PROBE = 128;
__device__ __forceinline__ uint32_t spill_put(const KP& P, uint32_t p, uint32_t c, uint32_t rec, bool* first) {
  const unsigned long long key = (unsigned long long)lrow(P, p) * P.W + c + 1ull;
  uint32_t h = (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> 40) & P.spmask;
  *first = false;
  for (uint32_t q = 0; q < SP_PROBE; ++q, h = (h + 1u) & P.spmask) {
    unsigned long long k = P.sp_key[h];
    if (k == 0ull) {
      k = atomicCAS(&P.sp_key[h], 0ull, key);
      if (k == 0ull) {
        atomicMax(&P.sp_val[h], rec);
        *first = true;
        P.sp_used[atomicAdd(&P.ctl->sp_n, 1u) & P.spmask] = h;  // (<= one claim per slot: never wraps)
        return h;
      }
    }
    if (k == key) {
      atomicMax(&P.sp_val[h], rec);
      return h;
    }
  }
  atomicOr(&P.ctl->overflow, OV_SPILL);
  return NONE_U32;
}
// the cell of a spill-table slot's key
__device__ __forceinline__ uint32_t spill_cell(const KP& P, uint32_t h) {
  return (uint32_t)((P.sp_key[h] - 1ull) % P.W);
}

// Suspicion deadlines are u16 cells: 0x8000 | (deadline mod 2^15), 0 = none. A
// stored deadline is never more than the suspicion timeout (mult * bit_length(N) <= 5 * 21 periods)
// ahead of the current period, nor behind it (the sweep fires or drops every due one), so the absolute
// period is the one within +-2^14 of any period of the run it is decoded at.
__host__ __device__ __forceinline__ uint16_t dl_enc(uint32_t dl) { return (uint16_t)(0x8000u | (dl & 0x7FFFu)); }
__host__ __device__ __forceinline__ uint32_t dl_dec(uint32_t e, uint32_t t) {
  int32_t diff = (int32_t)(((e & 0x7FFFu) - t) & 0x7FFFu);
  if (diff >= 0x4000) diff -= 0x8000;
  return t + (uint32_t)diff;
}

// a dense column whose cell leaves the converged BASELINE in some row (KP::tbits)
__device__ __forceinline__ void touch(const KP& P, uint32_t col) {
  if (!P.tmode) return;
  const uint32_t b = 1u << (col & 31u);
  if (!(P.tbits[col >> 5] & b)) atomicOr(&P.tbits[col >> 5], b);
}

// A removed cell (present -> absent) drops the batched apply's merge mark of its subject's block:
// records that did not override the present cell may override what the cell becomes next
__device__ __forceinline__ void mark_clear(const KP& P, uint32_t obs, uint32_t subj) {
  if (!P.dmark) return;
  const uint32_t sid = P.sid_of[subj];
  if (sid < P.dsids) P.dmark[lrow(P, obs) * P.dsids + sid] = 0u;
}
constexpr uint32_t GEN_MASK = 0xFFFFFFu;  // generation bits a merge mark keeps

// MembershipProtocolImpl.updateMembership (MembershipProtocolImpl.java:481-547) and callees
// (onSelfMemberDetected :549-569, onDeadMemberDetected :571-587, onAliveMemberDetected
// :589-610, schedule/cancelSuspicionTimeoutTask :612-635, spreadMembershipGossipUnlessGossiped
// :649-656). Returns the record to gossip (0 = none); the caller assigns the gossip sequence
// number so that every origin's ids are canonical.
__device__ __forceinline__ uint32_t apply_record(const KP& P, uint32_t obs, uint32_t subj, uint32_t r1,
                                                 uint32_t reason, uint32_t attempt, uint32_t others_snap, Tally& T) {
  const uint32_t col = col_of(P, subj);
  if (col == NONE) {  // N x K: k_fd_track gives every subject a column before its first change
    atomicOr(&P.ctl->overflow, OV_TRACK);
    return 0u;
  }
  uint32_t* cellp = P.view + lrow(P, obs) * P.W + col;
  const uint32_t r0 = *cellp;
  if (!is_overrides(r1, r0)) return 0u;
  // a record of another member id at the observer's own address is ignored (MPI:499-505)
  if (P.rerouted && subj != obs && P.addr[subj] == P.addr[obs]) return 0u;
  const bool spread = reason != SWIM_R_MEMBERSHIP_GOSSIP && reason != SWIM_R_INITIAL_SYNC;
  touch(P, col);  // every accepted record below writes the cell (a refutation too)
  if (subj == obs) {
    const uint32_t inc1 = (r1 == SWIM_DEAD) ? rec_inc(r0) : rec_inc(r1);
    const uint32_t inc0 = rec_inc(r0);
    const uint32_t r2 = SWIM_PACK((inc0 > inc1 ? inc0 : inc1) + 1u, rec_code(r0));
    *cellp = r2;
    T.accepted++;
    T.refut++;
    return r2;
  }
  uint16_t* dlp = P.dl + (size_t)col * P.nloc + lrow(P, obs);  // subject-major: a due column streams
  if (r1 == SWIM_DEAD) {
    *dlp = 0u;
    *cellp = SWIM_ABSENT;
    mark_clear(P, obs, subj);
    atomicSub(&P.cnt_delta[obs], 1);
    atomicSub(&P.pres[subj], 1u);
    atomicMax(&P.last_removed[subj], P.period + 1u);
    T.accepted++;
    T.removed++;
    push_event(P, obs, subj, SWIM_EV_REMOVED, reason, r0);
    return 0u;
  }
  if (rec_code(r1) == SWIM_SUSPECT) {
    *cellp = r1;
    T.accepted++;
    if (*dlp == 0u) {
      const uint32_t dl = P.period + susp_periods(P, others_snap);
      *dlp = dl_enc(dl);
      // every observer scheduling in a round computes the same deadline: read first, so the hot
      // column minimum takes one atomic per round instead of one per observer
      if (P.colmin[col] > dl) atomicMin(&P.colmin[col], dl);
    }
    return spread ? r1 : 0u;
  }
  if (!fetch_ok(P, obs, subj, attempt)) return 0u;
  *dlp = 0u;
  *cellp = r1;
  T.accepted++;
  // the fetched metadata (the subject's current version) replaces the stored one (MPI:537)
  bool updated = false;
  if (P.meta_view) {
    uint32_t* mp = P.meta_view + lrow(P, obs) * P.W + col;
    const uint32_t m1 = P.meta_cur[subj];
    updated = r0 != SWIM_ABSENT && *mp != m1;
    *mp = m1;
  }
  if (r0 == SWIM_ABSENT) {
    atomicAdd(&P.cnt_delta[obs], 1);
    atomicAdd(&P.pres[subj], 1u);
    T.added++;
    push_event(P, obs, subj, SWIM_EV_ADDED, reason, r1);
  } else if (updated) {  // MPI:599-600: a member it had, with metadata that differs
    T.updated++;
    push_event(P, obs, subj, SWIM_EV_UPDATED, reason, r1);
  }
  return spread ? r1 : 0u;
}

// ---- wave / block reductions (wave64) -------------------------------------------------
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// The wave scans below use GFX9 DPP row broadcasts (row_bcast:15 / row_bcast:31, controls 0x142 /
// 0x143), which exist only on GFX9-family targets, and assume 64-lane waves (every GFX9 target is
// wave64). They also need every lane of the wave active: callers run them in converged code only.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__GFX9__)
#error "swim_device.h: wave_excl_scan needs a GFX9 (wave64, DPP row_bcast) target such as gfx950"
#endif
// one DPP step of a wave scan: v from the lane the control selects, 0 where that lane is out of the
// row or masked off (old = 0, bound_ctrl off)
template <int CTRL, int ROWM>
__device__ __forceinline__ uint32_t dpp_in(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWM, 0xF, false);
}
// exclusive prefix sum over the 64 lanes; *total = sum over the wave (all lanes must call). DPP
// row shifts and broadcasts move the partial sums between lanes in the VALU instead of six
// LDS-routed lane shuffles (C3: k_gossip_apply_b 189 -> 183 ms per 20 periods)
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t* total) {
  uint32_t x = v;
  x += dpp_in<0x111, 0xF>(x);  // row_shr:1 .. row_shr:8: inclusive scans of the four 16-lane rows
  x += dpp_in<0x112, 0xF>(x);
  x += dpp_in<0x114, 0xF>(x);
  x += dpp_in<0x118, 0xF>(x);
  x += dpp_in<0x142, 0xA>(x);  // row_bcast:15 into rows 1 and 3
  x += dpp_in<0x143, 0xC>(x);  // row_bcast:31 into rows 2 and 3
  *total = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
  return x - v;
}

// list member v (local index l) in its stripe of a SYNC work list
__device__ __forceinline__ void sy_push(uint32_t* cnt, uint32_t* list, uint32_t cap, uint32_t l, uint32_t v) {
  const uint32_t st = l % SY_STRIPES;
  list[(size_t)st * cap + atomicAdd(&cnt[st], 1u)] = v;
}

// one more SYNC request for local receiver j: the first one lists j for k_sync_merge
__device__ __forceinline__ void recv_one(const KP& P, uint32_t j) {
  if (atomicAdd(&P.recv_count[j], 1u) == 0u) sy_push(P.ctl->sy_mcnt, P.sy_mlist, P.sy_cap, j - P.row0, j);
}

__device__ __forceinline__ void add_stat(const KP& P, int idx, uint32_t v) {
  v = wave_sum(v);
  // 64 counter shards on separate 256-B lines: one same-address atomic per wave would
  // serialize a 65,536-wave launch at the L2 (the host sums the shards)
  if ((threadIdx.x & 63) == 0 && v) {
    const uint32_t shard = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & (STAT_SHARDS - 1u);
    atomicAdd(&P.stat_shards[shard * STAT_STRIDE + idx], (unsigned long long)v);
  }
}

__device__ __forceinline__ void flush_tally(const KP& P, const Tally& T) {
  add_stat(P, ST_ACCEPTED, T.accepted);
  add_stat(P, ST_REFUTATIONS, T.refut);
  add_stat(P, ST_ADDED, T.added);
  add_stat(P, ST_REMOVED, T.removed);
  add_stat(P, ST_UPDATED, T.updated);
}

}  // namespace swim

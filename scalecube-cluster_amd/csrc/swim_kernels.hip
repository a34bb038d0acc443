// swim_kernels.hip — gfx950 kernels of one SWIM protocol period (dense N x N mode).
//
// Phase order per period, all on one HIP stream, no host round trips:
//   k_fd             FailureDetectorImpl.doPing/doPingReq (FailureDetectorImpl.java:126-209)
//                    + onFailureDetectorEvent (MembershipProtocolImpl.java:376-404)
//   k_commit (+ k_rs_* for storm phases) after every phase that creates gossips
//   G x { k_gossip_prep, k_gossip_select, k_gossip_pairfill/pairprune, k_gossip_inhist,
//         k_gossip_pull, k_gossip_record, k_gossip_apply, k_finalize }
//                    GossipProtocolImpl.doSpreadGossip/onGossipReq/sweepGossips
//                    (GossipProtocolImpl.java:139-304) + onMembershipGossip (MPI:407-414)
//   k_due, k_susp_sweep, k_finalize
//                    onSuspicionTimeout (MembershipProtocolImpl.java:637-647)
//   k_sync_select, k_sync_snapshot, k_scan, k_sync_scatter, k_sync_merge, k_finalize,
//   k_sync_ack, k_finalize
//                    doSync/onSync/onSyncAck (MembershipProtocolImpl.java:304-373,416-427)
// All kernels are HBM-bound integer work: no MFMA (no dense contraction on this path).
#include <hip/hip_runtime.h>

#include "swim_device.h"

namespace swim {

// A run whose buffers overflowed is dead (swim_sync reports SWIM_EOVERFLOW): every later kernel
// of it returns at once, so nothing runs on state an overflow left inconsistent (an N x K subject
// without a column, a wrapped ring) and the host never has to wait for a count mid-period.
#define SWIM_GUARD(P) \
  if ((P).ctl->overflow) return

constexpr int MAXF = 32;       // max gossipFanout handled on device
constexpr int MAXK = 16;       // max pingReqMembers handled on device
constexpr int BUCKET_MAX = 2048;  // SYNC requests one member can merge in one period

// ---------------------------------------------------------------------------------------
// init / bookkeeping
// ---------------------------------------------------------------------------------------
__global__ void k_fill_u32(uint32_t* p, size_t n, uint32_t v) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}

__global__ void k_finalize(KP P) {
  {  // the spill-table slots the round's apply claimed become empty again (the next round's
     // k_gossip_prep resets their count: the finalizes of later phases clear nothing new)
    const uint32_t n = min(P.ctl->sp_n, P.spmask + 1u);
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
      const uint32_t hs = P.sp_used[t];
      P.sp_key[hs] = 0ull;
      P.sp_val[hs] = 0u;
    }
  }
  SWIM_GUARD(P);
  const uint32_t i = P.row0 + blockIdx.x * blockDim.x + threadIdx.x;
  if (i < P.row0 + P.nloc) {
    const int32_t d = P.cnt_delta[i];
    if (d) {
      const uint32_t old = P.cnt[i], now = (uint32_t)((int32_t)old + d);
      P.cnt[i] = now;
      P.cnt_delta[i] = 0;
      const uint32_t b0 = bitlen(old + 1u), b1 = bitlen(now + 1u);
      if (b0 != b1 && P.alive[i]) {
        atomicSub(&P.ctl->bl_hist[b0], 1u);
        atomicAdd(&P.ctl->bl_hist[b1], 1u);
      }
    }
  }
}

// A leaving member whose leave gossip its own sweep dropped this round shuts down at the round's
// end (GossipProtocolImpl.spread completes at sweep, :299-302; ClusterImpl.doShutdown then stops
// the transport, ClusterImpl.java:376-388): the same as a crash. Leaves are rare, so each stopped
// member's row is walked by one thread.
__global__ void k_leave_stop(KP P) {
  SWIM_GUARD(P);
  const uint32_t c = P.row0 + blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= P.row0 + P.nloc || !P.stopf[c]) return;
  P.stopf[c] = 0;
  if (!P.alive[c]) return;
  atomicSub(&P.ctl->bl_hist[bitlen(P.cnt[c] + (uint32_t)P.cnt_delta[c] + 1u)], 1u);
  atomicSub(&P.ctl->alive_count, 1u);
  const uint32_t nc = ncells(P);
  for (uint32_t cc = 0; cc < nc; ++cc) {
    const uint32_t j = subj_of(P, cc);
    if (j != c && P.view[lrow(P, c) * P.W + cc] != 0u) atomicSub(&P.pres[j], 1u);
    P.dl[(size_t)cc * P.nloc + lrow(P, c)] = 0u;
  }
  P.alive[c] = 0;
  if (P.occ[P.addr[c]] == c) P.occ[P.addr[c]] = NONE;
  if (P.world > 1u) P.stop_list[atomicAdd(&P.ctl->n_stop, 1u)] = c;  // (<= nloc per commit)
}

// Sharded: members another shard stopped (k_leave_stop) since the last commit, from the commit
// exchange: the replicated liveness and address state follow (their rows live on that shard)
__global__ void k_stop_remote(KP P, const uint32_t* ids, uint32_t n) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t c = ids[k];
  if (c >= P.N || is_local(P, c)) return;
  P.alive[c] = 0;
  if (P.occ[P.addr[c]] == c) P.occ[P.addr[c]] = NONE;
}

// swim_leave: the member's own record becomes DEAD and is staged as a gossip (committed with the
// next phase's gossips, infectionPeriod = that period's first round, like the oracle's spread).
__global__ void k_leave(KP P, uint32_t i) {  // one wave; lane 0 does the work
  uint32_t created = 0;
  if (threadIdx.x == 0 && !P.leaving[i] && P.alive[i]) {
    P.leaving[i] = 1;
    P.leave_slot[i] = NONE;
    const uint32_t col = col_of(P, i);  // N x K: k_track_one asked for a column
    if (col == NONE) {                   // no column left (OV_TRACK): the run has failed
      atomicOr(&P.ctl->overflow, OV_TRACK);
    } else if (is_local(P, i)) {
      touch(P, col);
      P.view[lrow(P, i) * P.W + col] = SWIM_DEAD;
      emit_gossip(P, i, i, SWIM_DEAD, P.gseq[i]++);
      created = 1;
    }
  }
  add_stat(P, ST_GOSSIPS_CREATED, created);
}

// swim_spread: a user gossip (GossipProtocolImpl.spread, :124-128) staged like a leave's gossip;
// its subject is N + origin (no member: apply hands it to GossipProtocol.listen, not to membership)
__global__ void k_spread(KP P, uint32_t origin, uint32_t tag) {  // one wave; lane 0 does the work
  uint32_t created = 0;
  if (threadIdx.x == 0 && P.alive[origin] && is_local(P, origin)) {
    emit_gossip(P, origin, P.N + origin, tag, P.gseq[origin]++);
    created = 1;
  }
  add_stat(P, ST_GOSSIPS_CREATED, created);
}

// swim_deliver_records: an external node's message to member obs before the next period (the wire
// bridge): updateMembership of each record in order with the message's reason (MPI:463-473,
// :407-414), accepted SYNC records spread (MPI:649-656). One wave; lane 0 does the work in order.
// N x K: an untracked subject's BASELINE record is a no-op (equal records never override); the
// host requested columns for every other record's subject beforehand (k_deliver_track).
// SWIM_DELIVER_FORWARD: each record is a gossip new to obs (onGossipReq, GossipProtocolImpl.java:171-183):
// its GossipState is put first (the observer forwards it from the coming round on), then membership.
__global__ void k_deliver(KP P, uint32_t obs, const uint32_t* subj, const uint32_t* rec, uint32_t n, uint32_t reason) {
  Tally T;
  uint32_t created = 0;
  const bool fwd = (reason & SWIM_DELIVER_FORWARD) != 0u;
  reason &= ~SWIM_DELIVER_FORWARD;
  if (threadIdx.x == 0 && P.alive[obs] && is_local(P, obs)) {
    const uint32_t snap = P.cnt[obs];
    for (uint32_t k = 0; k < n; ++k) {
      const uint32_t j = subj[k], r1 = rec[k];
      if (fwd) {  // (its own id namespace: the member's gossipCounter does not move, GPI:171-183)
        emit_gossip(P, obs, j, r1, FOREIGN_SEQ | P.fseq[obs]++);
        ++created;
      }
      if (P.nxk && P.colmap[j] == NONE && r1 == BASELINE) continue;
      const uint32_t r = apply_record(P, obs, j, r1, reason, SWIM_DELIVER_ATTEMPT | k, snap, T);
      if (r) {
        emit_gossip(P, obs, j, r, P.gseq[obs]++);
        ++created;
      }
    }
  }
  add_stat(P, ST_GOSSIPS_CREATED, created);
  flush_tally(P, T);
}

__device__ __forceinline__ void track_request(const KP& P, uint32_t j);
// N x K: columns for the delivered records' subjects that leave the baseline (forwarded gossips: every
// subject, since the members they reach merge the record through their tables)
__global__ void k_deliver_track(KP P, const uint32_t* subj, const uint32_t* rec, uint32_t n, uint32_t all) {
  for (uint32_t k = threadIdx.x; k < n; k += blockDim.x)
    if (all || rec[k] != BASELINE) track_request(P, subj[k]);
}

// swim_update_metadata: MetadataStoreImpl.updateMetadata (a new version of the member's metadata)
// and MembershipProtocolImpl.updateIncarnation (MPI:184-196): the own record becomes ALIVE with
// incarnation + 1 and is staged as a gossip (spreadMembershipGossip: always spread)
__global__ void k_update_meta(KP P, uint32_t i) {  // one wave; lane 0 does the work
  uint32_t created = 0;
  if (threadIdx.x == 0 && P.alive[i] && !P.leaving[i]) {
    P.meta_cur[i] += 1u;
    const uint32_t col = col_of(P, i);  // N x K: k_track_one asked for a column
    if (col == NONE) {
      atomicOr(&P.ctl->overflow, OV_TRACK);
    } else if (is_local(P, i)) {
      touch(P, col);
      uint32_t* cellp = P.view + lrow(P, i) * P.W + col;
      const uint32_t r = SWIM_PACK(rec_inc(*cellp) + 1u, SWIM_ALIVE);
      *cellp = r;
      emit_gossip(P, i, i, r, P.gseq[i]++);
      created = 1;
    }
  }
  add_stat(P, ST_GOSSIPS_CREATED, created);
}

// converged start with spare slots: cell (row, col) = BASELINE for col < n0, absent otherwise
__global__ void k_init_rows(uint32_t* view, size_t n, uint32_t W, uint32_t n0) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    view[i] = (uint32_t)(i % W) < n0 ? BASELINE : SWIM_ABSENT;
}

// p[i] = i for i < n_id, NONE for the rest
__global__ void k_iota_u32(uint32_t* p, uint32_t n, uint32_t n_id) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = i < n_id ? i : NONE;
}

// swim_join / swim_restart: spare slot x starts at address a (ClusterImpl.start, ClusterImpl.java:
// 170-227) with a table holding only itself ALIVE inc 0 (MembershipProtocolImpl.java:138-142) and
// fresh protocol state; a restart on another member's address links x into that address's movers.
// Sharded handles launch it on every shard: the row (table, deadlines, histories, marks) and the shard's
// alive tallies only where it lives, liveness and addresses everywhere (they are replicated).
__global__ void k_join_one(KP P, uint32_t x, uint32_t a) {
  const bool mine = is_local(P, x);
  if (mine) {
    for (uint32_t c = threadIdx.x; c < P.W; c += blockDim.x) {
      P.view[lrow(P, x) * P.W + c] = c == x ? BASELINE : SWIM_ABSENT;
      P.dl[(size_t)c * P.nloc + lrow(P, x)] = 0u;
      if (P.meta_view) P.meta_view[lrow(P, x) * P.W + c] = 0u;
    }
    for (uint32_t t = threadIdx.x; t < 256u; t += blockDim.x) P.ih_rhead[lrow(P, x) * 256u + t] = 0u;
    if (P.dmark)  // a fresh table: no merge marks
      for (uint32_t t = threadIdx.x; t < P.dsids; t += blockDim.x) P.dmark[lrow(P, x) * P.dsids + t] = 0u;
  }
  if (threadIdx.x == 0) {
    P.cnt[x] = 0u;
    P.cnt_delta[x] = 0;
    P.fd_epoch[x] = P.fd_cursor[x] = P.g_epoch[x] = P.g_cursor[x] = 0u;
    P.gseq[x] = 0u;
    P.fseq[x] = 0u;
    P.sync_fd[x] = NONE;
    P.held[x] = 0u;
    P.ih_head[x] = 0u;
    P.alive[x] = 1;
    P.joining[x] = 1;
    if (a != x) {
      P.mv_next[x] = P.mv_head[a];
      P.mv_head[a] = x;
    }
    P.addr[x] = a;
    P.occ[a] = x;
    if (mine) {
      atomicAdd(&P.ctl->bl_hist[bitlen(1u)], 1u);
      atomicAdd(&P.ctl->alive_count, 1u);
    }
  }
}

// swim_crash: transport.stop() of n members at once (distinct, alive): presence no longer counted,
// timers dropped, the address goes quiet (unless a restarted member already holds it). Only the shard
// that owns a member's row has presence / timers to drop; workgroup b takes member b / chunks and
// the b % chunks-th piece of its row.
constexpr uint32_t CRASH_PIECE = 256u * 16u;  // cells per workgroup
__global__ void __launch_bounds__(256) k_crash_many(KP P, const uint32_t* ids, uint32_t n, uint32_t chunks) {
  const uint32_t k = blockIdx.x / chunks, piece = blockIdx.x % chunks;
  if (k >= n) return;
  const uint32_t c = ids[k];
  if (piece == 0u && threadIdx.x == 0u) {
    if (is_local(P, c)) {
      atomicSub(&P.ctl->bl_hist[bitlen(P.cnt[c] + 1u)], 1u);
      atomicSub(&P.ctl->alive_count, 1u);  // N x K: every untracked subject loses this observer
    }
    if (P.occ[P.addr[c]] == c) P.occ[P.addr[c]] = NONE;  // the address goes quiet (k_stop_addr)
  }
  if (!is_local(P, c)) return;
  const uint32_t nc = ncells(P);
  const uint32_t c0 = piece * CRASH_PIECE, c1 = min(nc, c0 + CRASH_PIECE);
  for (uint32_t cc = c0 + threadIdx.x; cc < c1; cc += blockDim.x) {
    const uint32_t j = subj_of(P, cc);
    if (j != c && P.view[lrow(P, c) * P.W + cc] != 0u) atomicSub(&P.pres[j], 1u);
    P.dl[(size_t)cc * P.nloc + lrow(P, c)] = 0u;
  }
}

// Second half of emit_gossip, step 1: sort keys of the phase's gossips. A batch commit
//  sorts by (origin, subject), so each origin's gossips form one run that becomes
// one ring slot; a one-gossip-per-slot commit sorts by (subject, record), so a subject's gossips
// take consecutive slots with ascending records (k_gossip_apply's subject runs). Sorting only
// permutes ring slots, which nothing observable depends on.
__device__ __forceinline__ unsigned long long stg_key(const KP& P, uint4 e) {  // e = {origin, subject, record, hash}
  return P.batch_commit ? (((unsigned long long)e.x << 32) | e.y) : (((unsigned long long)e.y << 32) | e.z);
}
__device__ __forceinline__ unsigned long long stg_val(const KP& P, uint4 e) {
  return P.batch_commit ? (((unsigned long long)e.z << 32) | e.w) : (((unsigned long long)e.x << 32) | e.w);
}
// back to {origin, subject, record, hash}
__device__ __forceinline__ uint4 kv_decode(const KP& P, unsigned long long k, unsigned long long v) {
  return P.batch_commit ? make_uint4((uint32_t)(k >> 32), (uint32_t)k, (uint32_t)(v >> 32), (uint32_t)v)
                        : make_uint4((uint32_t)(v >> 32), (uint32_t)(k >> 32), (uint32_t)k, (uint32_t)v);
}
// does sorted element i (key k, predecessor kp) open a new ring slot? a batch at each new origin,
// otherwise every gossip
__device__ __forceinline__ bool slot_start(const KP& P, uint32_t i, unsigned long long kp, unsigned long long k) {
  return i == 0u || !P.batch_commit || (kp >> 32) != (k >> 32);
}

__global__ void k_stage_keys(KP P, const uint4* ents, uint32_t n, uint32_t out_off, unsigned long long* keys,
                             unsigned long long* vals) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const uint4 e = ents[i];
    keys[out_off + i] = stg_key(P, e);
    vals[out_off + i] = stg_val(P, e);
  }
}

// Step 2: sorted gossip i is record c0 + i of the record ring, in slot g0 + ci (ci = the slots
// opened before it, minus one); every shard commits the same sorted batch, so the ring stays
// replicated. The element that opens a slot publishes it (record range start, first record, id
// hash, creation round, run mark) and, on the origin's shard, marks it held with infectionPeriod
// = create_round; the element that closes it sets the range's end. One-gossip slots mark runs of
// one subject in runw; a batch slot is a run of its own.
__device__ __forceinline__ void commit_one(const KP& P, uint32_t g0, uint32_t c0, uint32_t i, uint32_t ci,
                                           unsigned long long k, unsigned long long v, bool open, bool close,
                                           bool run) {
  const uint32_t W32 = P.GC >> 5;
  const uint4 e = kv_decode(P, k, v);
  const uint32_t origin = e.x, subject = e.y, record = e.z, hash = e.w;
  const uint32_t x = c0 + i;  // absolute record index
  P.c_sr[x & P.cmask] = make_uint2(subject, record);
  P.c_hash[x & P.cmask] = hash;
  const uint32_t id = g0 + ci;
  const uint32_t s = gmod(P, id);
  uint32_t* cref = reinterpret_cast<uint32_t*>(P.g_cref);
  // the DEAD record of a member about itself is only ever its leave gossip (MPI:203-212)
  if (subject == origin && record == SWIM_DEAD && P.leaving[origin]) P.leave_slot[origin] = s;
  if (close) {
    cref[2u * s + 1u] = x + 1u;
    // the live records start at the oldest live slot's first one: they must fit the record ring
    const uint32_t glo = P.ctl->glo;
    const uint32_t c_lo = (g0 != glo && g0 - glo <= P.GC) ? cref[2u * (gmod(P, glo))] : c0;
    if (x + 1u - c_lo > P.cmask + 1u) atomicOr(&P.ctl->overflow, OV_GOSSIP);
  }
  if (!open) return;
  // the live id range must stay below GC - 64 slots so bitmap words never alias across the
  // ring wrap, and the slot's previous gossip must be dead everywhere (glo passed it)
  if (id - P.ctl->glo >= P.GC - 64u) atomicOr(&P.ctl->overflow, OV_GOSSIP);
  if (!P.gpow2 && id >= 0xFFFFFFFFu - P.GC) atomicOr(&P.ctl->overflow, OV_GOSSIP);  // ids mod GC would jump
  cref[2u * s] = x;
  P.g_sr[s] = make_uint2(subject, record);
  P.g_hash[s] = hash;
  P.g_create[s] = P.create_round;
  if (run)
    atomicOr(&P.runw[s >> 5], 1u << (s & 31u));
  else
    atomicAnd(&P.runw[s >> 5], ~(1u << (s & 31u)));
  // a reused word's stale maximum is older than any live creation round, so max() resets it
  if (P.wlast[s >> 5] < P.create_round) atomicMax(&P.wlast[s >> 5], P.create_round);
  if (P.gc8) const_cast<uint8_t*>(P.gc8)[s] = (uint8_t)P.create_round;  // hd4: the slot's creation round
  if (is_local(P, origin)) {
    if (P.hd4)  // origin's infectionPeriod = the creation round: offset 0 (other nibbles untouched)
      atomicAnd(reinterpret_cast<uint32_t*>(P.hd) + lrow(P, origin) * (P.GC / 8u) + (s >> 3), ~(0xFu << (4u * (s & 7u))));
    else
      P.hd[lrow(P, origin) * P.GC + s] = (uint8_t)P.create_round;  // origin's infectionPeriod
    const uint32_t old = atomicOr(&P.hb[lrow(P, origin) * W32 + (s >> 5)], 1u << (s & 31u));
    if (!(old & (1u << (s & 31u)))) atomicAdd(&P.held[origin], 1u);
    // newest/oldest infection round the origin holds in the word (same value for the batch)
    mm_received(P, lrow(P, origin) * W32 + (s >> 5), old == 0u, P.create_round);
  }
}

// A phase's commit, sized on the device: n = the staged count (world 1, read by every kernel
// below, so the host never waits for it) or the gathered batch of every shard (n_host). The
// gossips are ordered by key (subject << 32 | record): a subject's gossips take consecutive slots
// with ascending records, which k_gossip_apply's subject runs rely on; ties (the same record from
// several origins) take any order, as slots are unobservable.
//   * n <= CS_SMALL (nearly every phase): k_commit alone, a bitonic sort in one workgroup's LDS;
//   * larger (storm phases): a least-significant-digit radix sort over 8-bit digits across the
//     chip: k_rs_hist (every pass's digit counts at once), one k_rs_pass per digit (tiles of
//     CS_TILE keys, tile order from an atomic counter, each tile's digit offsets from its
//     predecessors by decoupled look-back, stable ranks by wave ballots), k_rs_commit, k_rs_fin.
//     The look-back status word carries its value (flag | count, one agent-scope atomic store and
//     load), so no payload crosses workgroups inside a launch; spins are bounded (OV_BUG).
// Every kernel reads n itself and returns at once when the batch is not its size class.
#ifndef SWIM_CS_SMALL
#define SWIM_CS_SMALL 4096
#endif
constexpr uint32_t CS_SMALL = SWIM_CS_SMALL;  // LDS sort capacity (tests build a variant with a tiny one)
static_assert(CS_SMALL >= 1 && CS_SMALL <= 4096 && (CS_SMALL & (CS_SMALL - 1)) == 0, "CS_SMALL: a power of two <= 4096");
constexpr uint32_t CS_THREADS = 1024;
constexpr uint32_t CS_WAVES = CS_THREADS / 64u;
constexpr uint32_t CS_PER = 4;  // keys per thread in a radix tile
constexpr uint32_t CS_TILE = CS_THREADS * CS_PER;
constexpr uint32_t CS_MAXPASS = 8;
constexpr uint32_t CS_AGG = 0x40000000u, CS_INC = 0x80000000u, CS_CNT = 0x3FFFFFFFu;

struct CSort {
  unsigned long long *k0, *v0, *k1, *v1;  // ping-pong key / value buffers
  uint32_t* ghist;  // [CS_MAXPASS][256] digit counts of the whole batch per pass
  uint32_t* ctr;    // [CS_MAXPASS + 1] tiles handed out per pass; k_rs_fused's barrier count
  uint32_t* stat;   // [CS_MAXPASS][maxt][256] look-back status: flag | count
  uint32_t maxt, npass;
  uint32_t radix;   // tiles the host launched the radix kernels with (the phase's bound on its
                    // gossips); 0: none (the phase cannot stage > CS_SMALL)
};

__device__ __forceinline__ uint32_t cs_n(const KP& P, const uint4* stg, uint32_t n_host) {
  return stg ? min(P.ctl->stg_count, P.stg_cap) : n_host;
}

__device__ __forceinline__ uint32_t cs_block_scan(uint32_t v, uint32_t* total, uint32_t* lds) {
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  uint32_t wt;
  const uint32_t x = wave_excl_scan(v, &wt) + v;  // the wave's inclusive scan (DPP)
  if (lane == 63u) lds[w] = x;
  __syncthreads();
  uint32_t base = 0, tot = 0;
  for (uint32_t k = 0; k < blockDim.x / 64u; ++k) {
    const uint32_t t = lds[k];
    if (k < w) base += t;
    tot += t;
  }
  __syncthreads();
  *total = tot;
  return base + x - v;
}

// Elements 4t .. 4t+3 of a sorted block of CS_PER * CS_THREADS keys (at `base` of the batch,
// `cbase` slots opened before the block) committed by thread t; returns the slots the block opened.
// key(i) reads sorted key i of the batch (LDS or global).
template <typename KeyF, typename ValF>
__device__ __forceinline__ uint32_t commit_block(const KP& P, uint32_t g0, uint32_t c0, uint32_t n, uint32_t base,
                                                 uint32_t cbase, KeyF key, ValF val, uint32_t* lds) {
  const uint32_t t = threadIdx.x;
  unsigned long long kk[CS_PER + 1];
  bool op[CS_PER + 1];
  uint32_t cnt = 0;
  const uint32_t i0 = base + CS_PER * t;
  unsigned long long kp = (i0 > 0u && i0 <= n) ? key(i0 - 1u) : 0ull;
#pragma unroll
  for (uint32_t q = 0; q <= CS_PER; ++q) {
    const uint32_t i = i0 + q;
    kk[q] = i < n ? key(i) : 0ull;
    op[q] = i < n && slot_start(P, i, q ? kk[q - 1] : kp, kk[q]);
    if (q < CS_PER && op[q]) ++cnt;
  }
  uint32_t tot;
  uint32_t ci = cbase + cs_block_scan(cnt, &tot, lds);
#pragma unroll
  for (uint32_t q = 0; q < CS_PER; ++q) {
    const uint32_t i = i0 + q;
    if (i >= n) break;
    if (op[q]) ++ci;
    const unsigned long long prev = q ? kk[q - 1] : kp;
    // a subject run starts (a user gossip, subject >= N, is a run of its own: each is delivered)
    const bool run = P.batch_commit || i == 0u || (prev >> 32) != (kk[q] >> 32) || (uint32_t)(kk[q] >> 32) >= P.N;
    commit_one(P, g0, c0, i, ci - 1u, kk[q], val(i), op[q], i + 1u == n || op[q + 1], run);
  }
  return tot;
}

__global__ void __launch_bounds__(CS_THREADS) k_commit(KP P, const uint4* stg, uint32_t n_host, CSort C) {
  __shared__ unsigned long long s_key[CS_SMALL];
  __shared__ uint32_t s_idx[CS_SMALL];
  const uint32_t t = threadIdx.x;
  const uint32_t n = cs_n(P, stg, n_host);
  if (n > CS_SMALL) {  // a storm phase: reset the radix sort's counters for this batch
    const uint32_t nt = (n + CS_TILE - 1u) / CS_TILE;
    if (nt > C.radix) {  // the host's bound on this phase's gossips was wrong: fail loudly
      if (t == 0) atomicOr(&P.ctl->overflow, OV_BUG);
      return;
    }
    for (uint32_t i = t; i < CS_MAXPASS * 256u; i += CS_THREADS) C.ghist[i] = 0u;
    if (t <= CS_MAXPASS) C.ctr[t] = 0u;  // tile counters per pass, then k_rs_fused's barrier
    for (uint32_t p = 0; p < C.npass; ++p)
      for (uint32_t i = t; i < nt * 256u; i += CS_THREADS) C.stat[(size_t)p * C.maxt * 256u + i] = 0u;
    return;
  }
  __shared__ uint32_t s_lds[CS_WAVES];
  const uint32_t g0 = P.ctl->gcount, c0 = P.ctl->ccount;
  uint32_t m = 1;
  while (m < n) m <<= 1;
  for (uint32_t i = t; i < m; i += CS_THREADS) {
    unsigned long long k = ~0ull;
    if (i < n) k = stg ? stg_key(P, stg[i]) : C.k0[i];
    s_key[i] = k;
    s_idx[i] = i;
  }
  __syncthreads();
  for (uint32_t k = 2; k <= m; k <<= 1)
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = t; i < m; i += CS_THREADS) {
        const uint32_t l = i ^ j;
        if (l > i) {
          const unsigned long long a = s_key[i], b = s_key[l];
          const uint32_t ia = s_idx[i], ib = s_idx[l];
          const bool gt = a > b || (a == b && ia > ib);
          if (gt == ((i & k) == 0)) {
            s_key[i] = b;
            s_key[l] = a;
            s_idx[i] = ib;
            s_idx[l] = ia;
          }
        }
      }
      // a stage with j < 64 pairs elements of one wave (element i belongs to thread i mod 1,024):
      // the next stage of the same k reads only what this wave wrote, so a wave-level barrier
      // does; the workgroup barrier is needed after j >= 64 and at the end of each k
      if (j >= 64u || j == 1u) {
        __syncthreads();
      } else {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    }
  static_assert(CS_SMALL <= CS_PER * CS_THREADS, "k_commit: one commit_block covers the LDS sort");
  const uint32_t nslots = commit_block(
      P, g0, c0, n, 0u, 0u, [&](uint32_t i) { return s_key[i]; },
      [&](uint32_t i) { return stg ? stg_val(P, stg[s_idx[i]]) : C.v0[s_idx[i]]; }, s_lds);
  __syncthreads();
  if (t == 0) {
    P.ctl->g_prev = g0;
    P.ctl->gcount = g0 + nslots;
    P.ctl->c_prev = c0;
    P.ctl->ccount = c0 + n;
    if (stg) P.ctl->stg_count = 0u;
  }
}

// every pass's digit counts (a tile per workgroup); the stage moves into (k0, v0)
__device__ __forceinline__ void rs_hist_tile(const KP& P, const uint4* stg, uint32_t n, const CSort& C, uint32_t tile) {
  __shared__ uint32_t s_h[CS_MAXPASS][256];
  const uint32_t t = threadIdx.x;
  const uint32_t base = tile * CS_TILE;
  if (base >= n) return;
  __syncthreads();  // (a fused loop's previous tile has read s_h)
  for (uint32_t i = t; i < CS_MAXPASS * 256u; i += CS_THREADS) (&s_h[0][0])[i] = 0u;
  __syncthreads();
  for (uint32_t q = 0; q < CS_PER; ++q) {
    const uint32_t i = base + q * CS_THREADS + t;
    if (i >= n) break;
    unsigned long long k;
    if (stg) {
      const uint4 e = stg[i];
      k = stg_key(P, e);
      C.k0[i] = k;
      C.v0[i] = stg_val(P, e);
    } else {
      k = C.k0[i];
    }
    for (uint32_t p = 0; p < C.npass; ++p) atomicAdd(&s_h[p][(uint32_t)(k >> (8u * p)) & 255u], 1u);
  }
  __syncthreads();
  for (uint32_t i = t; i < C.npass * 256u; i += CS_THREADS) {
    const uint32_t c = (&s_h[0][0])[i];
    if (c) atomicAdd(&C.ghist[i], c);
  }
}

__global__ void __launch_bounds__(CS_THREADS) k_rs_hist(KP P, const uint4* stg, uint32_t n_host, CSort C) {
  const uint32_t n = cs_n(P, stg, n_host);
  if (n > CS_SMALL) rs_hist_tile(P, stg, n, C, blockIdx.x);
}

__device__ __forceinline__ bool rs_pass_tile(const KP& P, uint32_t n, const CSort& C, uint32_t p,
                                             const unsigned long long* sk, const unsigned long long* sv,
                                             unsigned long long* dk, unsigned long long* dv) {
  __shared__ uint32_t s_h[256], s_off[256], s_cnt[CS_WAVES][256], s_lds[CS_WAVES];
  __shared__ uint32_t s_tile;
  const uint32_t t = threadIdx.x;
  if (t == 0) s_tile = atomicAdd(&C.ctr[p], 1u);  // tiles in start order: predecessors are running
  if (t < 256u) s_h[t] = 0u;
  __syncthreads();
  const uint32_t tile = s_tile, base = tile * CS_TILE;
  if (base >= n) return false;  // uniform
  const uint32_t sh = 8u * p;
  unsigned long long key[CS_PER];
  uint32_t dg[CS_PER];
#pragma unroll
  for (uint32_t q = 0; q < CS_PER; ++q) {
    const uint32_t i = base + q * CS_THREADS + t;
    key[q] = i < n ? sk[i] : 0ull;
    dg[q] = (uint32_t)(key[q] >> sh) & 255u;
    if (i < n) atomicAdd(&s_h[dg[q]], 1u);
  }
  __syncthreads();
  // digit t: this tile's count, published at once; then the keys of digit t in earlier tiles
  uint32_t excl = 0;
  uint32_t* st = C.stat + (size_t)p * C.maxt * 256u;
  if (t < 256u) {
    const uint32_t own = s_h[t];
    __hip_atomic_store(&st[(size_t)tile * 256u + t], (tile == 0 ? CS_INC : CS_AGG) | own, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    if (tile > 0) {
      uint32_t j = tile - 1u, spins = 0;
      for (;;) {
        const uint32_t v = __hip_atomic_load(&st[(size_t)j * 256u + t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!(v & (CS_AGG | CS_INC))) {
          if (++spins > (1u << 22)) {  // a predecessor never published: fail loudly, never hang
            atomicOr(&P.ctl->overflow, OV_BUG);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        excl += v & CS_CNT;
        if ((v & CS_INC) || j == 0u) break;
        --j;
      }
      __hip_atomic_store(&st[(size_t)tile * 256u + t], CS_INC | (excl + own), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // + keys of smaller digits in the whole batch
  uint32_t all;
  const uint32_t gpre = cs_block_scan(t < 256u ? C.ghist[p * 256u + t] : 0u, &all, s_lds);
  if (t < 256u) s_off[t] = gpre + excl;
  __syncthreads();
  const uint32_t lane = t & 63u, w = t >> 6;
#pragma unroll
  for (uint32_t q = 0; q < CS_PER; ++q) {
    const uint32_t i = base + q * CS_THREADS + t;
    const bool ok = i < n;
    const uint32_t d = dg[q];
    // lanes of this wave with the same digit (8 ballots), and this lane's rank among them
    unsigned long long same = __ballot(ok);
#pragma unroll
    for (uint32_t bit = 0; bit < 8u; ++bit) {
      const unsigned long long bb = __ballot(ok && ((d >> bit) & 1u));
      same &= ((d >> bit) & 1u) ? bb : ~bb;
    }
    const uint32_t rank = (uint32_t)__popcll(same & ((1ull << lane) - 1ull));
    for (uint32_t x = t; x < CS_WAVES * 256u; x += CS_THREADS) (&s_cnt[0][0])[x] = 0u;
    __syncthreads();
    if (ok && rank == 0u) s_cnt[w][d] = (uint32_t)__popcll(same);
    __syncthreads();
    if (ok) {
      uint32_t pos = s_off[d] + rank;
      for (uint32_t y = 0; y < w; ++y) pos += s_cnt[y][d];
      dk[pos] = key[q];
      dv[pos] = sv[i];
    }
    __syncthreads();
    if (t < 256u) {
      uint32_t add = 0;
      for (uint32_t y = 0; y < CS_WAVES; ++y) add += s_cnt[y][t];
      s_off[t] += add;
    }
    __syncthreads();
  }
  return true;
}

__global__ void __launch_bounds__(CS_THREADS) k_rs_pass(KP P, const uint4* stg, uint32_t n_host, CSort C, uint32_t p,
                                                        const unsigned long long* sk, const unsigned long long* sv,
                                                        unsigned long long* dk, unsigned long long* dv) {
  const uint32_t n = cs_n(P, stg, n_host);
  if (n > CS_SMALL) (void)rs_pass_tile(P, n, C, p, sk, sv, dk, dv);
}

// Slots opened per tile of the sorted batch (C.stat is free once the passes are done: tile
// counts in stat[0 .. nt), their exclusive scan in stat[maxt .. maxt + nt), k_excl_scan)
__device__ __forceinline__ void rs_slots_tile(const KP& P, uint32_t n, const CSort& C, const unsigned long long* k,
                                              uint32_t tile) {
  __shared__ uint32_t s_lds[CS_WAVES];
  if (tile * CS_TILE >= n) return;
  __syncthreads();  // (a fused loop's previous tile has read s_lds)
  const uint32_t i0 = tile * CS_TILE + CS_PER * threadIdx.x;
  uint32_t cnt = 0;
  for (uint32_t q = 0; q < CS_PER; ++q) {
    const uint32_t i = i0 + q;
    if (i < n && slot_start(P, i, i ? k[i - 1] : 0ull, k[i])) ++cnt;
  }
  uint32_t tot;
  cs_block_scan(cnt, &tot, s_lds);
  if (threadIdx.x == 0) C.stat[tile] = tot;
}

__global__ void __launch_bounds__(CS_THREADS) k_rs_slots(KP P, const uint4* stg, uint32_t n_host, CSort C,
                                                         const unsigned long long* k) {
  const uint32_t n = cs_n(P, stg, n_host);
  if (n > CS_SMALL) rs_slots_tile(P, n, C, k, blockIdx.x);
}

__device__ __forceinline__ void rs_commit_tile(const KP& P, uint32_t n, const CSort& C, const unsigned long long* k,
                                               const unsigned long long* v, uint32_t tile) {
  __shared__ uint32_t s_lds[CS_WAVES];
  if (tile * CS_TILE >= n) return;
  __syncthreads();  // (a fused loop's previous tile has read s_lds)
  commit_block(P, P.ctl->gcount, P.ctl->ccount, n, tile * CS_TILE, C.stat[C.maxt + tile],
               [&](uint32_t i) { return k[i]; }, [&](uint32_t i) { return v[i]; }, s_lds);
}

__global__ void __launch_bounds__(CS_THREADS) k_rs_commit(KP P, const uint4* stg, uint32_t n_host, CSort C,
                                                          const unsigned long long* k, const unsigned long long* v) {
  const uint32_t n = cs_n(P, stg, n_host);
  if (n > CS_SMALL) rs_commit_tile(P, n, C, k, v, blockIdx.x);
}

__device__ __forceinline__ void rs_fin_one(const KP& P, const uint4* stg, uint32_t n, const CSort& C) {
  const uint32_t nt = (n + CS_TILE - 1u) / CS_TILE;
  P.ctl->g_prev = P.ctl->gcount;
  P.ctl->gcount += C.stat[C.maxt + nt - 1u] + C.stat[nt - 1u];
  P.ctl->c_prev = P.ctl->ccount;
  P.ctl->ccount += n;
  if (stg) P.ctl->stg_count = 0u;
  atomicAdd(&P.stat_shards[ST_COMMIT_RADIX], 1ull);  // (one thread: shard 0)
}

__global__ void k_rs_fin(KP P, const uint4* stg, uint32_t n_host, CSort C) {
  const uint32_t n = cs_n(P, stg, n_host);
  if (n > CS_SMALL) rs_fin_one(P, stg, n, C);
}

// Does a possibly-live ring slot hold a batch of several gossips? (swim_set_loss)
__global__ void k_multi_live(KP P, uint32_t* out) {
  const uint32_t lo = P.ctl->glo, hi = P.ctl->gcount;
  const uint32_t n = hi - lo > P.GC ? P.GC : hi - lo;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint2 r = P.g_cref[gmod(P, lo + i)];
    if (r.y - r.x > 1u) atomicOr(out, 1u);
  }
}

// Gossips per bitmap word (wsum) and per slot (scnt) of the words the last commit wrote slots into,
// or (all) of every word that may be live (batch slots start: the words committed before them)
__device__ __forceinline__ void commit_wsum_body(const KP& P, uint32_t all) {
  const uint32_t g1 = P.ctl->gcount;
  const uint32_t g0 = all ? (g1 - P.ctl->glo > P.GC ? g1 - P.GC : P.ctl->glo) : P.ctl->g_prev;
  const uint32_t w0 = g0 >> 5, w1 = (g1 + 31u) >> 5;
  const uint32_t* cref = reinterpret_cast<const uint32_t*>(P.g_cref);
  for (uint32_t w = w0 + blockIdx.x * blockDim.x + threadIdx.x; w < w1; w += gridDim.x * blockDim.x) {
    uint32_t sum = 0;
    const uint32_t ws = wmod(P, w);
    for (uint32_t b = 0; b < 32u; ++b) {
      const uint32_t id = (w << 5) + b;
      uint32_t c = 0;
      if ((int32_t)(g1 - id) > 0) {  // created (the word's slots from earlier commits count)
        const uint32_t s = gmod(P, id);
        c = cref[2u * s + 1u] - cref[2u * s];
      }
      sum += c;
      P.scnt[ws * 32u + b] = (uint16_t)(c < SCNT_SAT ? c : SCNT_SAT);
    }
    P.wsum[ws] = sum;
  }
}

__global__ void k_commit_wsum(KP P, uint32_t all) { commit_wsum_body(P, all); }

// ---- record dictionary, after every commit: claim, entries, free ----
// A block for each subject of the commit's records that has none: the CAS winner pops a free
// block (or takes a new one); when none is left the subject is marked with this commit's
// no-block tag (its records take the apply kernel's slow path) and is not claimed again until a
// later commit, so a commit makes at most one failed claim per subject: the high-water mark passes
// DICT_SIDS by at most the commit's subjects (< 2^21), and k_dict_entries clamps it back, so it can
// never wrap onto blocks in use. (A compare-and-swap loop that never passed DICT_SIDS serialized
// thousands of claims of one storm commit: C3 18.2 -> 20.6 ms/period.) No thread waits on another.
__device__ __forceinline__ void dict_claim_body(const KP& P) {
  const uint32_t c0 = P.ctl->c_prev, n = P.ctl->ccount - c0, nfree = P.ctl->d_nfree;
  const uint32_t tag = DICT_NOBLK | (c0 & DICT_TAG_MASK);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t subj = P.c_sr[(c0 + i) & P.cmask].x;
    if (subj >= P.N) continue;
    const uint32_t cur = P.sid_of[subj];
    // a block, a claim in progress, or a claim of this commit that found none
    if (cur < P.dsids || cur == DICT_LOCK || cur == tag) continue;
    if (atomicCAS(&P.sid_of[subj], cur, DICT_LOCK) != cur) continue;  // NONE or an older commit's tag
    const uint32_t k = atomicAdd(&P.ctl->d_taken, 1u);
    uint32_t sid = NONE;
    if (k < nfree) {
      sid = P.d_free[nfree - 1u - k];
    } else {  // (one claim per subject and commit: k_dict_entries clamps the mark back to dsids)
      const uint32_t hw = atomicAdd(&P.ctl->d_hw, 1u);
      if (hw < P.dsids) sid = hw;
    }
    if (sid != NONE) P.d_subj[sid] = subj;
    P.sid_of[subj] = sid != NONE ? sid : tag;
  }
}

// Each record's entry in its subject's block: an entry holding the same record, else the first
// empty one (claimed by CAS); a full block or no block: ID_NONE, remembered in d_none_last.
__device__ __forceinline__ void dict_entries_body(const KP& P) {
  const uint32_t c0 = P.ctl->c_prev, n = P.ctl->ccount - c0;
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // the blocks k_dict_claim popped leave the stack
    const uint32_t t = P.ctl->d_taken, f = P.ctl->d_nfree;
    P.ctl->d_nfree = f - min(t, f);
    P.ctl->d_taken = 0u;
    if (P.ctl->d_hw > P.dsids) P.ctl->d_hw = P.dsids;  // failed claims of the last commit
  }
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t x = c0 + i;
    const uint2 sr = P.c_sr[x & P.cmask];
    uint32_t id = ID_NONE;
    if (sr.x >= P.N) {
      id = ID_USER;
    } else {
      const uint32_t sid = P.sid_of[sr.x];
      if (sid < P.dsids) {
        // (16-bit ids: the two top ids of an 8,192-block dictionary are the sentinels, never entries)
        const uint32_t ways = (P.cid16 && sid * DICT_WAYS + DICT_WAYS > ID16_USER) ? ID16_USER - sid * DICT_WAYS : DICT_WAYS;
        for (uint32_t k = 0; k < ways; ++k) {
          uint32_t* e = &P.d_rec[sid * DICT_WAYS + k];
          uint32_t v = *e;
          if (v == 0u) v = atomicCAS(e, 0u, sr.y);
          if (v == 0u || v == sr.y) {
            id = sid * DICT_WAYS + k;
            break;
          }
        }
      }
    }
    if (P.cid16)
      P.c_id16[x & P.cmask] = (uint16_t)(id == ID_USER ? ID16_USER : (id == ID_NONE ? ID16_NONE : id));
    else
      P.c_id[x & P.cmask] = id;
    if (id < P.dsids * DICT_WAYS)
      atomicMax(&P.d_last[id], x + 1u);
    else if (id == ID_NONE) {
      atomicMax(&P.ctl->d_none_last, x + 1u);
      atomicMax(const_cast<uint32_t*>(&P.none_last[sr.x]), x + 1u);
    }
  }
}

// Entries no live record names are emptied; a block left empty goes back on the stack (its
// subject gets a block again with its next record).
__device__ __forceinline__ void dict_free_body(const KP& P) {
  const uint32_t hw = min(P.ctl->d_hw, P.dsids), c_lo = live_rec_lo(P);
  for (uint32_t sid = blockIdx.x * blockDim.x + threadIdx.x; sid < hw; sid += gridDim.x * blockDim.x) {
    const uint32_t subj = P.d_subj[sid];
    if (subj == NONE) continue;
    bool live = false, emptied = false;
    for (uint32_t k = 0; k < DICT_WAYS; ++k) {
      const uint32_t id = sid * DICT_WAYS + k;
      if (P.d_rec[id] == 0u) continue;
      if ((int32_t)(P.d_last[id] - c_lo) > 0) {
        live = true;
      } else {
        P.d_rec[id] = 0u;
        emptied = true;
      }
    }
    if (emptied && P.dmark) {  // an entry may take another record: the block's merge marks lapse
      uint32_t g = P.d_gen[sid] + 1u;
      if ((g & GEN_MASK) == 0u) {  // the marks' 24 generation bits wrap: no stale mark may match
        ++g;
        for (uint32_t r = 0; r < P.nloc; ++r) P.dmark[(size_t)r * P.dsids + sid] = 0u;
      }
      P.d_gen[sid] = g;
    }
    if (!live) {
      P.d_subj[sid] = NONE;
      P.sid_of[subj] = NONE;
      P.d_free[atomicAdd(&P.ctl->d_nfree, 1u)] = sid;
    }
  }
}

// Slot entry bitmaps of this commit's long ranges: a workgroup per new slot whose range holds at
// least as many records as the dictionary's bitmap has words in use (below that, walking the ids
// costs a receiver fewer LDS operations than ORing the bitmap). Records without an entry (a user
// gossip, a full block) leave the range without one: a receiver walks those ranges.
__global__ void __launch_bounds__(256) k_slot_bm(KP P) {
  extern __shared__ uint32_t s_rb[];  // dsids / 4 words
  __shared__ uint32_t s_flag;
  const uint32_t g0 = P.ctl->g_prev, g1 = P.ctl->gcount, nbw = P.dsids / 4u;
  const uint32_t bw = (min(P.ctl->d_hw, P.dsids) * DICT_WAYS + 31u) >> 5;
  const uint32_t dids = P.dsids * DICT_WAYS, dlim = P.cid16 ? min(dids, ID16_USER) : dids;
  for (uint32_t g = g0 + blockIdx.x; (int32_t)(g1 - g) > 0; g += gridDim.x) {
    const uint32_t sl = gmod(P, g);
    const uint2 cr = P.g_cref[sl];
    if (cr.y - cr.x < bw || cr.y - cr.x < 64u) continue;  // (uniform)
    for (uint32_t t = threadIdx.x; t < nbw; t += blockDim.x) s_rb[t] = 0u;
    if (threadIdx.x == 0) s_flag = 0u;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < cr.y - cr.x; i += blockDim.x) {
      const uint32_t x = cr.x + i;
      const uint32_t id = P.cid16 ? (uint32_t)P.c_id16[x & P.cmask] : P.c_id[x & P.cmask];
      const uint32_t idn = P.cid16 ? (id >= ID16_USER ? NONE : id) : id;
      if (idn < dlim)
        atomicOr(&s_rb[idn >> 5], 1u << (idn & 31u));
      else
        s_flag = 1u;
    }
    __syncthreads();
    if (s_flag == 0u) {
      __shared__ uint32_t s_rbi;
      if (threadIdx.x == 0) s_rbi = atomicAdd(&P.ctl->rb_next, 1u) % P.rb_cap;
      __syncthreads();
      const uint32_t rb = s_rbi;
      uint32_t* dst = P.rb_bits + (size_t)rb * nbw;
      for (uint32_t t = threadIdx.x; t < nbw; t += blockDim.x) dst[t] = s_rb[t];
      if (threadIdx.x == 0) {
        P.rb_tag[rb] = cr.x;
        P.g_rb[sl] = rb;
      }
    } else if (threadIdx.x == 0) {
      P.g_rb[sl] = NONE;
    }
    __syncthreads();
  }
}

// The entry ids of this commit's short slots (16-bit ids): a slot whose range holds at most SID_INLINE
// records carries them in g_sid, so a receiver's apply reads them with the range (g_sid beside g_cref)
// instead of after it (c_id16 at the range: one dependent load fewer per single gossip received). A
// record's id never changes while its slot is live (k_dict_entries writes it once, at the commit).
// C3 apply 6.45 -> 6.09 / 6.14 ms per period (13.90 -> 13.51 / 13.59 per period), C2 3.60 -> 3.53, C4's
// schedule at 65,536 (c4d65) 19.53 -> 19.03 / 19.01
// (8 ids per slot in 16 B measured slower: C3 13.82 against 13.54 / 13.68, c4d65 19.19 against 19.01 / 19.00)
constexpr uint32_t SID_INLINE = 4;
__device__ __forceinline__ void slot_ids_body(const KP& P) {
  const uint32_t g0 = P.ctl->g_prev, g1 = P.ctl->gcount;
  for (uint32_t g = g0 + blockIdx.x * blockDim.x + threadIdx.x; (int32_t)(g1 - g) > 0; g += gridDim.x * blockDim.x) {
    const uint32_t sl = gmod(P, g);
    const uint2 cr = P.g_cref[sl];
    const uint32_t len = cr.y - cr.x;
    if (len == 0u || len > SID_INLINE) continue;
    uint32_t v[4] = {0u, 0u, 0u, 0u};
    for (uint32_t k = 0; k < len; ++k) v[k] = P.c_id16[(cr.x + k) & P.cmask];
    P.g_sid[sl] = make_uint2(v[0] | (v[1] << 16), v[2] | (v[3] << 16));
  }
}

// (launches after a commit: the batch slots' word counts ride the claim, the short slots' entry ids the
// free; neither depends on the other's step)
__global__ void k_dict_claim(KP P, uint32_t wsum) {
  if (wsum) commit_wsum_body(P, 0u);
  dict_claim_body(P);
}
__global__ void k_dict_entries(KP P) { dict_entries_body(P); }
__global__ void k_dict_free(KP P, uint32_t sids) {
  dict_free_body(P);
  if (sids) slot_ids_body(P);
}


// Exclusive prefix sum of n words in one workgroup (sharded exchange offsets)
__device__ __forceinline__ void excl_scan_block(const uint32_t* in, uint32_t* out, uint32_t n) {
  __shared__ uint32_t s_lds4[CS_WAVES];
  const uint32_t per = (n + CS_THREADS - 1u) / CS_THREADS;
  const uint32_t a = min(n, threadIdx.x * per), e = min(n, a + per);
  uint32_t sum = 0;
  for (uint32_t i = a; i < e; ++i) sum += in[i];
  uint32_t tot;
  uint32_t run = cs_block_scan(sum, &tot, s_lds4);
  for (uint32_t i = a; i < e; ++i) {
    const uint32_t v = in[i];
    out[i] = run;
    run += v;
  }
}

__global__ void __launch_bounds__(CS_THREADS) k_excl_scan(const uint32_t* in, uint32_t* out, uint32_t n) {
  excl_scan_block(in, out, n);
}

// The radix chain in one launch (k_rs_hist, a k_rs_pass per digit, k_rs_slots, the tile scan,
// k_rs_commit, k_rs_fin, with a grid barrier between steps) on a grid of at most CS_FUSE
// workgroups, each walking tiles at a grid stride (the passes take tiles in start order from their
// counters, as k_rs_pass does): every workgroup of such a grid is resident at once, so the barrier
// cannot wait on one that was never scheduled. The host takes it for phases whose bound allows at
// most CS_FUSE tiles (a gossip round: nloc / 4,096), where a batch the LDS sort took returns at
// once: one launch instead of eleven, most of a quiet round's commit.
constexpr uint32_t CS_FUSE = 32;
// (the workgroup barrier completes every wave's stores to the XCD's L2; thread 0's agent-scope
// fences then write that L2 back before the arrival and invalidate it after the wait: one L2
// write-back / invalidate per workgroup and barrier, not per wave, which on 8 XCDs costs microseconds)
__device__ __forceinline__ void cs_grid_sync(const KP& P, uint32_t* bar, uint32_t& target) {
  __syncthreads();
  target += gridDim.x;
  if (threadIdx.x == 0) {
    __threadfence();
    atomicAdd(bar, 1u);
    uint32_t spins = 0;
    while (__hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (++spins > (1u << 24)) {  // a workgroup never arrived: fail loudly, never hang
        atomicOr(&P.ctl->overflow, OV_BUG);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    __threadfence();  // the other workgroups' stores visible after it (no stale L1 / L2 lines)
  }
  __syncthreads();
}

__global__ void __launch_bounds__(CS_THREADS) k_rs_fused(KP P, const uint4* stg, uint32_t n_host, CSort C) {
  const uint32_t n = cs_n(P, stg, n_host);
  if (n <= CS_SMALL) return;  // (uniform over the grid: no workgroup enters a barrier)
  uint32_t* bar = C.ctr + CS_MAXPASS;  // reset with the tile counters by k_commit
  uint32_t target = 0;
  for (uint32_t tile = blockIdx.x; tile * CS_TILE < n; tile += gridDim.x) rs_hist_tile(P, stg, n, C, tile);
  cs_grid_sync(P, bar, target);
  for (uint32_t p = 0; p < C.npass; ++p) {
    const bool even = (p & 1u) == 0u;
    while (rs_pass_tile(P, n, C, p, even ? C.k0 : C.k1, even ? C.v0 : C.v1, even ? C.k1 : C.k0, even ? C.v1 : C.v0)) {
    }
    cs_grid_sync(P, bar, target);
  }
  const bool in0 = (C.npass & 1u) == 0u;
  const unsigned long long* ks = in0 ? C.k0 : C.k1;
  for (uint32_t tile = blockIdx.x; tile * CS_TILE < n; tile += gridDim.x) rs_slots_tile(P, n, C, ks, tile);
  cs_grid_sync(P, bar, target);
  if (blockIdx.x == 0) excl_scan_block(C.stat, C.stat + C.maxt, C.maxt);
  cs_grid_sync(P, bar, target);
  for (uint32_t tile = blockIdx.x; tile * CS_TILE < n; tile += gridDim.x)
    rs_commit_tile(P, n, C, ks, in0 ? C.v0 : C.v1, tile);
  cs_grid_sync(P, bar, target);
  if (blockIdx.x == 0 && threadIdx.x == 0) rs_fin_one(P, stg, n, C);
}

// ---------------------------------------------------------------------------------------
// Phase 0: failure detector.
// ---------------------------------------------------------------------------------------
struct Probe {
  uint32_t j, nA, nB, stB, preq, direct;  // outcome: nA SUSPECT events, then nB events of status stB
};

// doPing / doPingReq (FailureDetectorImpl.java:126-209) of alive observer i with others > 0:
// selectPingMember advances i's cursor (written back only when `commit`), then the outcome of the
// direct ping or the ping-req round.
__device__ __forceinline__ Probe fd_probe(const KP& P, uint32_t i, bool commit) {
  Probe pr = {NONE, 0u, 0u, SWIM_SUSPECT, 0u, 0u};
  const uint32_t N = P.N;
  const uint32_t half = perm_half_bits(N);
  // selectPingMember (FailureDetectorImpl.java:340-349)
  uint32_t ep = P.fd_epoch[i], cur = P.fd_cursor[i];
  PermKey key = perm_key(P.seed, K_FD_PERM, i, ep);
  uint32_t j = NONE;
  for (uint32_t guard = 0; guard < 2u * N + 2u; ++guard) {
    if (cur >= N) {
      cur = 0;
      ++ep;
      key = perm_key(P.seed, K_FD_PERM, i, ep);
    }
    const uint32_t x = perm_apply(cur++, N, half, key);
    if (x != i && cell_get(P, i, x) != 0u) {
      j = x;
      break;
    }
  }
  if (commit) {
    P.fd_epoch[i] = ep;
    P.fd_cursor[i] = cur;
  }
  if (j == NONE) {  // member count says >0 but the row holds nobody: invariant broken
    atomicOr(&P.ctl->overflow, OV_BUG);
    j = (i + 1) % N;
  }
  pr.j = j;
  // onPing at the process on j's address answers DEST_GONE unless it is j itself (FDI:226-252),
  // which computeMemberStatus turns into DEAD (FDI:370-391)
  const uint32_t acked = (P.rerouted && route(P, j) != j) ? SWIM_DEAD : SWIM_ALIVE;
  // the direct round trip counts if it is back within pingTimeout (FDI:145 .timeout); a later ack
  // competes with the ping-req relays below
  const bool ping_in = delivered(P, K_PING, i, j, 0, P.tick);
  const uint32_t t_direct = P.delay_on ? msg_delay(P, K_PING, i, j, 0, P.tick) + msg_delay(P, K_ACK, j, i, 0, P.tick) : 0u;
  if (ping_in && delivered(P, K_ACK, j, i, 0, P.tick) && (!P.delay_on || t_direct < P.pto)) {
    pr.direct = 1;
    pr.nB = 1;
    pr.stB = acked;
    return pr;
  }
  // selectPingReqMembers (FailureDetectorImpl.java:351-363)
  uint32_t proxies[MAXK];
  uint32_t np = 0;
  if (P.kreq > 0u) {
    const PermKey pk = perm_key(P.seed, K_PROXY_PERM, i, P.period);
    for (uint32_t pos = 0; pos < N && np < P.kreq; ++pos) {
      const uint32_t x = perm_apply(pos, N, half, pk);
      if (x != i && x != j && cell_get(P, i, x) != 0u) proxies[np++] = x;
    }
  }
  if (!P.time_left_pos || np == 0) {
    pr.nB = 1;  // FailureDetectorImpl.java:163-165
    return pr;
  }
  pr.preq = 1;
  // the ack that reaches i's transport first (ms after the direct ping was sent): a proxy's
  // forwarded ack (PING_REQs leave at the direct timeout and wait pingInterval - pingTimeout,
  // FDI:152-183), or the direct ping's own late ack, which carries the same correlation id
  uint32_t first = NONE, t_first = NONE;
  for (uint32_t q = 0; q < np; ++q) {
    const uint32_t p = proxies[q];
    if (!out_ok(P, K_PING_REQ, i, p, j, P.tick)) {
      ++pr.nA;  // NetworkEmulator send error -> immediate SUSPECT
      continue;
    }
    ++pr.nB;
    if ((first == NONE || P.delay_on) && in_ok(P, p, i) && delivered(P, K_PROXY_PING, p, j, i, P.tick) &&
        delivered(P, K_PROXY_ACK, j, p, i, P.tick) && out_ok(P, K_FWD_ACK, p, i, j, P.tick)) {
      const uint32_t hops = P.delay_on ? msg_delay(P, K_PING_REQ, i, p, j, P.tick) + msg_delay(P, K_PROXY_PING, p, j, i, P.tick) +
                                             msg_delay(P, K_PROXY_ACK, j, p, i, P.tick) + msg_delay(P, K_FWD_ACK, p, i, j, P.tick)
                                       : 0u;
      if (hops < P.pint - P.pto && P.pto + hops < t_first) {  // earliest; ties: selection order
        first = p;
        t_first = P.pto + hops;
      }
    }
  }
  if (P.delay_on && pr.nB && ping_in && t_direct >= P.pto && t_direct < P.pint && t_direct <= t_first &&
      out_ok(P, K_ACK, j, i, 0, P.tick))
    first = j;  // the late direct ack wins ties
  // cid-only matching (TransportImpl.java:236-238): that ack completes every pending
  // subscription, then i's inbound filter on its sender decides (NetworkEmulatorTransport.java:64-68)
  pr.stB = (first != NONE && in_ok(P, i, first)) ? acked : SWIM_SUSPECT;
  return pr;
}

__device__ __forceinline__ uint32_t block_excl_scan1024(uint32_t v, uint32_t* total, uint32_t* lds16);

// N x K mode, before the FD phase: an untracked target whose record this probe turns SUSPECT
// (the only way a subject's record first leaves the baseline: every later change — gossip,
// SYNC, timeout, refutation — concerns a subject some record already changed) needs a column.
// A requested subject is listed once (track_req flags it, track_list holds it).
__device__ __forceinline__ void track_request(const KP& P, uint32_t j) {
  if (P.colmap[j] != NONE || atomicExch(&P.track_req[j], 1u) != 0u) return;
  const uint32_t o = atomicAdd(&P.ctl->ntrack, 1u);
  if (o < P.tcap)
    P.track_list[o] = j;
  else
    atomicOr(&P.ctl->overflow, OV_TRACK);  // more first changes in one phase than columns exist
}

__global__ void __launch_bounds__(256) k_fd_track(KP P) {
  SWIM_GUARD(P);
  const uint32_t i = P.row0 + blockIdx.x * blockDim.x + threadIdx.x;
  if (i < P.row0 + P.nloc && P.alive[i] && P.cnt[i] > 0u) {
    const Probe pr = fd_probe(P, i, false);
    if (pr.nA + pr.nB > 0u && (pr.nA > 0u || pr.stB == SWIM_SUSPECT)) track_request(P, pr.j);
  }
}

// Sharded: every shard's requests (its observers' probes) travel to every shard, so all of them
// allocate the same columns (a SYNC row is a row of columns; k_sync_pack)
__global__ void k_track_pack(KP P) {
  const uint32_t n = min(P.ctl->ntrack, P.tcap);
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) P.xsend[i] = P.track_list[i];
}

// the gathered lists (block q of `stride` words, cnt[q] entries) replace the local one
__global__ void k_track_unpack(KP P, const uint32_t* cnt, uint32_t stride) {
  __shared__ uint32_t s_n;
  if (threadIdx.x == 0) s_n = 0u;
  __syncthreads();
  for (uint32_t q = 0; q < P.world; ++q) {
    const uint32_t base = s_n;
    for (uint32_t i = threadIdx.x; i < cnt[q]; i += blockDim.x) {
      const uint32_t j = P.xrecv[(size_t)q * stride + i];
      P.track_req[j] = 1u;
      if (base + i < P.tcap) P.track_list[base + i] = j;
    }
    __syncthreads();
    if (threadIdx.x == 0) s_n = base + cnt[q];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (s_n > P.tcap) atomicOr(&P.ctl->overflow, OV_TRACK);
    P.ctl->ntrack = min(s_n, P.tcap);
  }
}

// One workgroup: the listed subjects get the next free columns in subject order (deterministic,
// the same on every shard), the columns pre-filled with BASELINE cells, the subject's presence
// materialised (every alive observer of this shard but itself holds it), no deadline.
constexpr uint32_t TRACK_SORT = 4096;  // subjects one FD phase may start tracking (LDS sort)
__global__ void __launch_bounds__(1024) k_track_alloc(KP P) {
  SWIM_GUARD(P);
  __shared__ uint32_t s_j[TRACK_SORT];
  __shared__ uint32_t s_lds[16];
  const uint32_t t = threadIdx.x;
  const uint32_t n = min(P.ctl->ntrack, P.tcap);
  if (n == 0u) return;
  if (n > TRACK_SORT) {
    if (t == 0) atomicOr(&P.ctl->overflow, OV_TRACK);
    return;
  }
  uint32_t m = 1;
  while (m < n) m <<= 1;
  for (uint32_t i = t; i < m; i += blockDim.x) s_j[i] = i < n ? P.track_list[i] : NONE;
  __syncthreads();
  for (uint32_t k = 2; k <= m; k <<= 1)
    for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
      for (uint32_t i = t; i < m; i += blockDim.x) {
        const uint32_t l = i ^ jj;
        if (l > i) {
          const uint32_t a = s_j[i], b = s_j[l];
          if ((a > b) == ((i & k) == 0)) {
            s_j[i] = b;
            s_j[l] = a;
          }
        }
      }
      __syncthreads();
    }
  const uint32_t c0 = P.ctl->ncols;
  const uint32_t alive_local = P.ctl->alive_count;  // alive observers of this shard
  uint32_t col = c0;
  for (uint32_t b0 = 0; b0 < n; b0 += blockDim.x) {  // new = first of its value, still untracked
    const uint32_t i = b0 + t;
    const uint32_t j = i < n ? s_j[i] : NONE;
    const bool fresh = i < n && (i == 0u || s_j[i - 1u] != j) && P.colmap[j] == NONE;
    uint32_t tot;
    const uint32_t off = block_excl_scan1024(fresh ? 1u : 0u, &tot, s_lds);
    if (i < n) P.track_req[j] = 0u;
    if (fresh) {
      const uint32_t c = col + off;
      if (c >= P.W) {
        atomicOr(&P.ctl->overflow, OV_TRACK);
      } else {
        P.colsubj[c] = j;
        P.pres[j] = alive_local - ((P.alive[j] && is_local(P, j)) ? 1u : 0u);
        P.colmap[j] = c;
      }
    }
    col += tot;
  }
  __syncthreads();
  if (t == 0) {
    P.ctl->ncols = col;
    P.ctl->ntrack = 0u;
  }
}

// the allocated columns in subject order (SYNC merges assign gossip sequence numbers in it)
__global__ void __launch_bounds__(256) k_colorder(KP P) {
  SWIM_GUARD(P);
  const uint32_t n = P.ctl->ncols < P.W ? P.ctl->ncols : P.W;
  for (uint32_t c = threadIdx.x; c < n; c += blockDim.x) {
    const uint32_t sj = P.colsubj[c];
    uint32_t rank = 0;
    for (uint32_t d = 0; d < n; ++d) rank += P.colsubj[d] < sj ? 1u : 0u;
    P.colorder[rank] = c;
  }
}

// N x K: give subject j a column now (swim_leave: the member's own record changes)
__global__ void k_track_one(KP P, uint32_t j) {
  if (threadIdx.x == 0) track_request(P, j);
}

// ---------------------------------------------------------------------------------------
// Phase 0: failure detector, one thread per observer.
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_fd(KP P) {
  SWIM_GUARD(P);
  const uint32_t i = P.row0 + blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t probes = 0, direct = 0, preq = 0, sev = 0, aev = 0, dev = 0, created = 0;
  Tally T;
  if (i < P.row0 + P.nloc && P.alive[i] && P.cnt[i] > 0u) {
    const Probe pr = fd_probe(P, i, true);
    const uint32_t j = pr.j;
    probes = 1;
    direct = pr.direct;
    preq = pr.preq;
    // publishPingResult -> onFailureDetectorEvent, sequentially (MembershipProtocolImpl.java:376-404)
    const uint32_t snap = P.cnt[i];
    for (uint32_t e = 0; e < pr.nA + pr.nB; ++e) {
      const uint32_t st = e < pr.nA ? (uint32_t)SWIM_SUSPECT : pr.stB;
      if (P.trace & SWIM_TRACE_FD) push_event(P, i, j, SWIM_EV_FD, e, st);  // FailureDetector.listen()
      if (st == SWIM_ALIVE)
        ++aev;
      else if (st == SWIM_DEAD)
        ++dev;
      else
        ++sev;
      const uint32_t r0 = cell_get(P, i, j);
      if (r0 == 0u || rec_code(r0) == st) continue;
      if (st == SWIM_ALIVE) {
        P.sync_fd[i] = j;
        continue;
      }
      // SUSPECT with the record's incarnation, or DEAD (a DEST_GONE ack: never spread, MPI:571-587)
      const uint32_t rec = apply_record(P, i, j, st == SWIM_DEAD ? SWIM_DEAD : SWIM_PACK(rec_inc(r0), SWIM_SUSPECT),
                                        SWIM_R_FAILURE_DETECTOR_EVENT, 0u, snap, T);
      if (rec) {
        emit_gossip(P, i, j, rec, P.gseq[i]++);
        ++created;
      }
    }
  }
  add_stat(P, ST_FD_PROBES, probes);
  add_stat(P, ST_FD_DIRECT_OK, direct);
  add_stat(P, ST_FD_PING_REQ, preq);
  add_stat(P, ST_FD_SUSPECT_EV, sev);
  add_stat(P, ST_FD_ALIVE_EV, aev);
  add_stat(P, ST_FD_DEAD_EV, dev);
  add_stat(P, ST_GOSSIPS_CREATED, created);
  flush_tally(P, T);
}

// ---------------------------------------------------------------------------------------
// Gossip round.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t range_mask(uint32_t id0, uint32_t lo, uint32_t hi) {
  // bits b of the word whose id id0 + b lies in [lo, hi)
  uint32_t m = 0xFFFFFFFFu;
  if (lo > id0) m = lo - id0 >= 32u ? 0u : m << (lo - id0);
  if (hi < id0 + 32u) m &= hi <= id0 ? 0u : (0xFFFFFFFFu >> (32u - (hi - id0)));
  return m;
}

// Four infection rounds per dword (byte b = word bit 4q + b). Byte-wise (r - d) mod 2^8: the high
// bit of every byte is set before the subtraction so no borrow crosses a byte, then fixed up.
__device__ __forceinline__ uint32_t bytes_sub(uint32_t r, uint32_t d) {
  const uint32_t R = (r & 0xFFu) * 0x01010101u, H = 0x80808080u;
  return ((R | H) - (d & ~H)) ^ ((R ^ ~d) & H);
}

// 4-bit mask: bit b set iff byte b of a > t (t < 2^15). Bytes go to 16-bit lanes, where
// v + 0x8000 - (t + 1) reaches bit 15 iff v > t and never carries into the next lane.
__device__ __forceinline__ uint32_t bytes_gt(uint32_t a, uint32_t t) {
  const uint32_t K = (0x8000u - (t + 1u)) * 0x00010001u;
  const uint32_t gl = ((a & 0x00FF00FFu) + K) & 0x80008000u;         // bytes 0, 2
  const uint32_t gh = (((a >> 8) & 0x00FF00FFu) + K) & 0x80008000u;  // bytes 1, 3
  return ((gl >> 15) & 1u) | ((gh >> 14) & 2u) | ((gl >> 29) & 4u) | ((gh >> 28) & 8u);
}

// 4-bit mask -> byte mask (0xFF per set bit): the four shifted copies do not overlap
__device__ __forceinline__ uint32_t nibble_bytes(uint32_t n) { return ((n * 0x00204081u) & 0x01010101u) * 0xFFu; }

// receiver p gets sender entry e this round (a local member id, or XREC | received record)
__device__ __forceinline__ void register_sender(const KP& P, uint32_t p, uint32_t e) {
  const uint32_t slot = atomicAdd(&P.in_cnt[p], 1u);
  if (slot < INCAP) {
    P.in_list[(size_t)p * INCAP + slot] = e;
  } else {  // rare: a receiver picked by more than INCAP senders
    const uint32_t o = atomicAdd(&P.ctl->n_inov, 1u);
    P.in_ov[2 * o] = p;
    P.in_ov[2 * o + 1] = e;
  }
}

__device__ __forceinline__ uint32_t block_excl_scan1024(uint32_t v, uint32_t* total, uint32_t* lds16) {
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  uint32_t wt;
  const uint32_t x = wave_excl_scan(v, &wt) + v;  // the wave's inclusive scan (DPP)
  if (lane == 63u) lds16[w] = x;
  __syncthreads();
  uint32_t base = 0, tot = 0;
  for (uint32_t k = 0; k < blockDim.x / 64u; ++k) {
    const uint32_t t = lds16[k];
    if (k < w) base += t;
    tot += t;
  }
  __syncthreads();
  *total = tot;
  return base + x - v;
}

// ---- GossipState.infectedFrom (GossipState.java:17; GossipProtocolImpl.java:181,248) -------
// A member never sends gossip g to a peer it received g from during its current GossipState of
// g. Storing every (member, gossip, sender) triple is out of reach in a storm (~150 senders per
// held gossip), so the device keeps exactly the part that can matter:
//   * every member's in-history: the senders that delivered to it in the last hzn rounds;
//   * for a delivery whose receiver may select its sender as a gossip peer within hzn rounds
//     (may_select, conservative), a record of the delivered gossips;
//   * when a member does select such a peer, its window for that peer is pruned by the records
//     (k_gossip_pairfill, k_gossip_pairprune); a selected peer in the in-history without a record (a prediction
//     that failed) raises OV_IFROM instead of silently diverging.
// hzn = gossipPeriodsToSpread(N) + 1: a record made in round t can only suppress sends in rounds
// t+1 .. t+1+spread, the last rounds the receiver can still have those gossips in its window.
// 0: s is out of p's reach within the horizon; 1: within it; 2: near enough that the present
// members ahead of it decide (pos / wrap: s's position in the shuffle the cursor will reach)
__device__ __forceinline__ uint32_t may_select_pre(const KP& P, uint32_t p, uint32_t s, uint32_t* pos_out,
                                                   bool* wrap_out) {
  const uint32_t others = P.cnt[p];
  if (others < P.f + 64u) return 1u;  // small views: "select all" is never far away
  const uint32_t N = P.N;
  const uint64_t kappa = (2ull * N + others) / (others + 1ull);  // >= 2 positions per present member
  const uint64_t reach = (uint64_t)(P.hzn + 1u) * P.f * kappa + 64u;
  if (reach >= N) return 1u;
  const uint32_t half = perm_half_bits(N);
  const uint32_t ep = P.g_epoch[p], cur = P.g_cursor[p];
  uint32_t pos = perm_inverse(s, N, half, perm_key(P.seed, K_GOSSIP_PERM, p, ep));
  bool wrap = false;
  if (!(pos >= cur && pos - cur < reach)) {
    if (cur + reach <= N) return 0u;
    // the cursor may wrap into the next shuffle within the horizon
    pos = perm_inverse(s, N, half, perm_key(P.seed, K_GOSSIP_PERM, p, ep + 1u));
    if (pos >= cur + reach - N) return 0u;
    wrap = true;
  }
  *pos_out = pos;
  *wrap_out = wrap;
  return 2u;
}

// Exact refinement: selectGossipMembers takes the first f present members from the cursor each
// round, so s comes up once the present members ahead of it are used up. Members removed in
// the meantime only bring it closer: a quarter of margin (a misprediction raises OV_IFROM).
// `stride` threads starting at `first` share the count (a wave: 64; one thread: 1).
__device__ __forceinline__ uint32_t may_select_ahead(const KP& P, uint32_t p, uint32_t pos, bool wrap, uint32_t first,
                                                     uint32_t stride) {
  const uint32_t N = P.N, half = perm_half_bits(N);
  const uint32_t ep = P.g_epoch[p], cur = P.g_cursor[p];
  const PermKey k0 = perm_key(P.seed, K_GOSSIP_PERM, p, ep);
  uint32_t ahead = 0;
  const uint32_t end0 = wrap ? N : pos;
  for (uint32_t x = cur + first; x < end0; x += stride) {
    const uint32_t m = perm_apply(x, N, half, k0);
    ahead += (m != p && cell_get(P, p, m) != 0u) ? 1u : 0u;
  }
  if (wrap) {
    const PermKey k1 = perm_key(P.seed, K_GOSSIP_PERM, p, ep + 1u);
    for (uint32_t x = first; x < pos; x += stride) {
      const uint32_t m = perm_apply(x, N, half, k1);
      ahead += (m != p && cell_get(P, p, m) != 0u) ? 1u : 0u;
    }
  }
  return ahead;
}

__device__ __forceinline__ bool may_select_within(const KP& P, uint32_t ahead) {
  return ahead < (P.f * P.hzn * 5u) / 4u + 16u;
}

// one thread's decision (k_gossip_need)
__device__ __forceinline__ bool may_select(const KP& P, uint32_t p, uint32_t s) {
  uint32_t pos = 0;
  bool wrap = false;
  const uint32_t pre = may_select_pre(P, p, s, &pos, &wrap);
  if (pre != 2u) return pre == 1u;
  return may_select_within(P, may_select_ahead(P, p, pos, wrap, 0u, 1u));
}

__device__ __forceinline__ uint32_t bytes_sub(uint32_t r, uint32_t d);
__device__ __forceinline__ uint32_t bytes_gt(uint32_t a, uint32_t t);

// bits of word ws whose current GossipState at member m began no later than round t (a record
// of round t about them still applies): infection round inf, state created in round inf - 1
// (or committed for round inf), so (t + 1 - inf) mod 2^8 <= 255 - hzn (swim_create checks that
// sweepmax + hzn < 256, so the two cases cannot alias)
__device__ __forceinline__ uint32_t state_since(const KP& P, uint32_t m, uint32_t ws, uint32_t t, uint32_t need) {
  uint4 d0, d1;
  if (P.hd4)  // (escapes of the slots asked about that m still holds)
    hd_load32<true>(P, lrow(P, m), ws, d0, d1, need & P.hb[lrow(P, m) * (P.GC >> 5) + ws]);
  else
    hd_load32<false>(P, lrow(P, m), ws, d0, d1);
  const uint32_t d32[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
  uint32_t late = 0;
#pragma unroll
  for (uint32_t q = 0; q < 8u; ++q) late |= bytes_gt(bytes_sub(t + 1u, d32[q]), 255u - P.hzn) << (4u * q);
  return ~late;
}

// One workgroup, once per round, before any member acts. Advances the oldest-live pointer (a
// gossip is dead once every holder has swept it: the last holder got it by wlast) and lists the
// ACTIVE bitmap words: those where some holder's send window (age <= spread) may be non-empty or
// some holder's sweep (age > sweep, GossipProtocolImpl.java:281-304) may fire this round. Every
// holder's infection round of a slot lies in [g_create, wlast], so a word whose whole age range
// is past every window and short of every sweep is idle for all members and is never touched.
// Spread/sweep bounds use the min/max bit_length(others+1) over alive members (bl_hist).
__global__ void __launch_bounds__(1024) k_gossip_prep(KP P) {
  __shared__ uint32_t s_lo, s_hi, s_blo, s_bhi, s_first;
  __shared__ uint32_t s_part[16];
  Ctl* c = P.ctl;
  if (threadIdx.x == 0) c->sp_n = 0u;  // the last round's spill slots were cleared by its k_finalize
  if (c->overflow) {  // the run has failed (reported at the next swim_sync): list nothing, touch nothing
    if (threadIdx.x == 0) {
      c->n_act = 0;
      c->n_alist = c->n_inov = c->sp_cnt = c->rp_cnt = c->pw_used = 0;
      c->scan_lo = c->scan_hi = c->gcount;
    }
    return;
  }
  if (threadIdx.x == 0) s_first = NONE;
  __syncthreads();
  {  // the first word (from glo) that may still be held: wlast bounds every slot's infection round
    const uint32_t hi0 = c->gcount, lo0 = c->glo;
    const uint32_t lo1 = hi0 - lo0 > P.GC ? hi0 - P.GC : lo0;
    for (uint32_t wi = (lo1 >> 5) + threadIdx.x; wi < ((hi0 + 31u) >> 5); wi += blockDim.x)
      if (P.wlast[wmod(P, wi)] + P.sweepmax >= P.round) {
        atomicMin(&s_first, wi);
        break;  // later words of this thread are larger
      }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t hi = c->gcount;
    uint32_t lo = c->glo;
    if (hi - lo > P.GC) lo = hi - P.GC;
    // a full ring (k_commit has raised OV_GOSSIP): keep the listed words within one lap of
    // the ring, so no list position reaches past a W32-word row of wb / nb
    const uint32_t lo_w = (((hi + 31u) >> 5) - (P.GC >> 5)) << 5;
    if (((hi + 31u) >> 5) - (lo >> 5) > (P.GC >> 5)) lo = lo_w;
    const uint32_t first = s_first == NONE ? hi : (s_first << 5);
    if (first > lo) lo = first < hi ? first : hi;
    c->glo = lo;
    c->n_alist = 0;
    c->n_inov = 0;
    c->sp_cnt = 0;
    c->rp_cnt = 0;
    c->pw_used = 0;
    c->rs_rec[P.round & 255u] = c->rec_cnt;
    c->rs_body[P.round & 255u] = c->body_cnt;
    c->scan_lo = lo;
    c->scan_hi = hi;
    uint32_t blo = 32, bhi = 0;
    if (P.blx) {  // sharded: bounds over every shard's alive members (all-reduced)
      bhi = P.blx[0];
      blo = 32u - P.blx[1];
    } else {
      for (uint32_t b = 0; b < 32u; ++b)
        if (c->bl_hist[b]) {
          blo = b < blo ? b : blo;
          bhi = b;
        }
    }
    if (blo > bhi) blo = bhi = 1;  // nobody alive: nothing will be scanned anyway
    s_lo = lo;
    s_hi = hi;
    s_blo = blo;
    s_bhi = bhi;
  }
  __syncthreads();
  const uint32_t lo = s_lo, hi = s_hi;
  const uint32_t w_lo = lo >> 5, w_end = (hi + 31u) >> 5;
  const int32_t r = (int32_t)P.round;
  const int32_t spread_lo = (int32_t)(P.rm * s_blo), spread_hi = (int32_t)(P.rm * s_bhi);
  const int32_t sweep_lo = 2 * (spread_lo + 1), sweep_hi = 2 * (spread_hi + 1);
  const uint32_t W32 = P.GC >> 5;
  // Words are listed by aligned quads: a quad with any active word contributes all four (the
  // idle ones with class NONE/NONE, which every consumer skips), so list position 4q..4q+3 maps
  // to four consecutive, 16-B-aligned holdings words and k_gossip_select reads them with one
  // 16-B load. When the padded span would not fit the list (a live range of ~GC ids), only the
  // active words are listed and the consumers fall back to per-word loads.
  const uint32_t w_beg = w_lo & ~3u, q_end = (w_end + 3u) & ~3u;
  const bool pad = q_end - w_beg <= W32;
  uint32_t base = 0;
  for (uint32_t t0 = w_beg; t0 < q_end; t0 += 4u * blockDim.x) {
    const uint32_t wq = t0 + 4u * threadIdx.x;
    uint32_t e[4], onm = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4u; ++j) {
      const uint32_t wi = wq + j;
      uint32_t wc = WC_NONE, sc = WC_NONE;
      if (wi >= w_lo && wi < w_end) {
        const uint32_t ws = wmod(P, wi);
        const uint32_t id0 = (wi << 5) > lo ? (wi << 5) : lo;
        const int32_t inf_lo = (int32_t)P.g_create[gmod(P, id0)];
        const int32_t inf_hi = (int32_t)P.wlast[ws];
        const int32_t amin = r - inf_hi, amax = r - inf_lo;  // holders' ages lie in [amin, amax]
        wc = amin > spread_hi ? WC_NONE : (amax <= spread_lo ? WC_ALL : WC_MIXED);
        sc = amax <= sweep_lo ? WC_NONE : (amin > sweep_hi ? WC_ALL : WC_MIXED);
      }
      if (wc != WC_NONE || sc != WC_NONE) onm |= 1u << j;
      e[j] = (wi - w_beg) | (wc << 26) | (sc << 28);
    }
    const uint32_t cnt = pad ? (onm ? 4u : 0u) : (uint32_t)__popc(onm);
    uint32_t total;
    const uint32_t off = block_excl_scan1024(cnt, &total, s_part);
    if (pad) {
      if (onm) {
        *reinterpret_cast<uint4*>(P.act + base + off) = make_uint4(e[0], e[1], e[2], e[3]);
#pragma unroll
        for (uint32_t j = 0; j < 4u; ++j)  // word -> list position, for infectedFrom records
          P.actpos[wmod(P, wq + j)] = make_uint2(P.round, base + off + j);
      }
    } else {
      uint32_t o = base + off;
#pragma unroll
      for (uint32_t j = 0; j < 4u; ++j)
        if ((onm >> j) & 1u) {
          P.actpos[wmod(P, wq + j)] = make_uint2(P.round, o);
          P.act[o++] = e[j];
        }
    }
    base += total;
  }
  if (threadIdx.x == 0) {
    c->n_act = base;
    c->w_beg = w_beg;
    c->wbeg_hist[P.round & 255u] = w_beg;
  }
}

// ---- quiet periods ("Quiet periods") ----
// After a period's FD commit: may any member still hold a gossip at the period's first round r0?
// k_gossip_prep's own test (a word is held while wlast + sweepmax >= round) over the whole live
// range. When none is, every gossip round of the period is a no-op for every kernel of the round:
// nothing is listed (select returns at once, GossipProtocolImpl.java:144-146 "gossips non-empty"),
// nobody registers with a peer, so nothing is pulled, recorded, applied, created or committed; wlast
// and the ring only grow through those kernels, so the answer holds for every round of the period.
// out[0] = 1: the rounds run (a word may be held, or the run has failed and prep must see it).
__global__ void __launch_bounds__(1024) k_quiet_check(KP P, uint32_t r0, uint32_t* out) {
  __shared__ uint32_t s_busy;
  const Ctl* c = P.ctl;
  if (threadIdx.x == 0) s_busy = c->overflow ? 1u : 0u;
  __syncthreads();
  const uint32_t hi0 = c->gcount, lo0 = c->glo;
  const uint32_t lo1 = hi0 - lo0 > P.GC ? hi0 - P.GC : lo0;
  bool busy = false;
  for (uint32_t wi = (lo1 >> 5) + threadIdx.x; wi < ((hi0 + 31u) >> 5); wi += blockDim.x)
    if (P.wlast[wmod(P, wi)] + P.sweepmax >= r0) {
      busy = true;
      break;
    }
  if (busy) s_busy = 1u;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = s_busy;
}

// What the G skipped rounds r0 .. r0 + G - 1 of a quiet period leave behind, written at once: the
// per-round bookkeeping of k_gossip_prep listing nothing (the oldest-live pointer at the ring's end,
// the record-pool fills and list starts of each round), select's empty peer counts, the
// in-history heads k_gossip_inhist files per round, pull's cleared registrations and each round's
// empty commit (k_commit of no gossips: g_prev / c_prev at the counts). The host then runs
// k_dict_free once, as the first round's commit would have (the rounds after it free nothing more).
__global__ void __launch_bounds__(256) k_quiet_rounds(KP P, uint32_t r0, uint32_t G) {
  Ctl* c = P.ctl;
  const uint32_t hi = c->gcount;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const uint32_t w_beg = (hi >> 5) & ~3u;
    c->glo = hi;
    c->sp_n = 0u;
    c->n_act = 0u;
    c->w_beg = w_beg;
    c->n_alist = c->n_inov = c->sp_cnt = c->rp_cnt = c->pw_used = 0u;
    c->scan_lo = c->scan_hi = hi;
    for (uint32_t q = 0; q < G; ++q) {
      const uint32_t r = (r0 + q) & 255u;
      c->rs_rec[r] = c->rec_cnt;
      c->rs_body[r] = c->body_cnt;
      c->wbeg_hist[r] = w_beg;
    }
    c->g_prev = hi;
    c->c_prev = c->ccount;
  }
  const uint32_t m = P.row0 + blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= P.row0 + P.nloc) return;
  P.npeers[m] = 0u;
  P.in_cnt[m] = 0u;
  const uint32_t ihh = P.ih_head[m];
  uint32_t* rh = P.ih_rhead + lrow(P, m) * 256u;
  for (uint32_t q = 0; q < G; ++q) rh[(r0 + q) & 255u] = ihh;
  if (m == P.dbg_watch) {
    for (uint32_t q = 0; q < G; ++q) {
      uint32_t* L = P.dbg_log + ((r0 + q) & 255u) * 8u;
      L[0] = r0 + q;
      L[1] = L[2] = L[3] = 0u;
      L[4] = L[5] = L[6] = NONE;
    }
  }
}

// sweepGossips of a leaving member's own DEAD gossip completes its spread() (GPI:299-302)
__device__ __forceinline__ void leave_swept(const KP& P, uint32_t m, uint32_t ws, uint32_t clear) {
  const uint32_t sl = P.leave_slot[m];
  if (sl != NONE && (sl >> 5) == ws && ((clear >> (sl & 31u)) & 1u)) P.stopf[m] = 1;
}

// One wave per member m, on the start-of-round state (before any delivery of round r):
// doSpreadGossip's "gossips non-empty" test (GossipProtocolImpl.java:144-146, the held count),
// the peer choice selectGossipMembers (:253-274), the send window (:242-251) and the sweep
// sweepGossips (:281-304) of entries with r > infectionPeriod + sweep, over the ACTIVE words only.
// Swept entries are cleared before round-r deliveries so receivers see them absent; a gossip
// swept in round r still counts as held at its start. Window words go to wb, indexed by position
// in the active list. A word's infection rounds (64 B) are read only when its class is MIXED;
// ALL/NONE words are decided by the class. A member with a non-empty window registers with each
// chosen peer (in_cnt), so delivery can run receiver-side (k_gossip_pull).
// one list quad per lane per step at 6 waves per SIMD (80 VGPRs, 44 B of scratch): with the MIXED
// entries flattened across the wave, more waves in flight beat more loads per wave (C3 select 63.9
// -> 55.3 ms per 20 periods, C4's schedule 94.9 -> 87.9)
#define SWIM_SEL_BATCH 1
#define SWIM_SEL_WAVES 6
constexpr uint32_t SEL_BATCH = SWIM_SEL_BATCH;  // list quads per lane per step in k_gossip_select

// The lane that owns item q of a wave-wide flattened list: the last lane j with off_j <= q (off =
// the lanes' exclusive offsets, non-decreasing; every lane calls it, each with its own q).
__device__ __forceinline__ uint32_t wave_owner(uint32_t off, uint32_t q) {
  uint32_t lo = 0;
#pragma unroll
  for (uint32_t step = 32; step > 0; step >>= 1) {
    const uint32_t o = __shfl(off, (int)(lo + step), 64);
    if (o <= q) lo += step;
  }
  return lo;
}

// position of the k-th (0-based) set bit of m, k < popcount(m)
__device__ __forceinline__ uint32_t kth_set_bit(uint32_t m, uint32_t k);

// wave_owner for a window of 64 items: lane x gets the owner of item q0 + x, where lane L owns items
// [off_L, off_L + cnt_L) (off = the exclusive scan of cnt). A lane whose item does not exist gets an
// arbitrary owner (callers test q < total). (A ballot / VALU variant of it measured no faster, §6.5.)
__device__ __forceinline__ uint32_t wave_owner_at(uint32_t off, uint32_t cnt, uint32_t q0) {
  (void)cnt;
  return wave_owner(off, q0 + (threadIdx.x & 63u));
}

__device__ __forceinline__ uint32_t kth_set_bit(uint32_t m, uint32_t k) {
  uint32_t pos = 0;
#pragma unroll
  for (uint32_t w = 16; w > 0; w >>= 1) {
    const uint32_t c = (uint32_t)__popc(m & ((1u << w) - 1u));
    if (k >= c) {
      k -= c;
      m >>= w;
      pos += w;
    }
  }
  return pos;
}

// One wave per member. (The workgroup's 4 waves sharing one member's holdings pass, as the pull does
// on small shards, measured slower on C2's 4,096 members: select 0.41 -> 0.46 ms per period, §6.5.)
template <bool HD4>
__device__ __forceinline__ void select_body(const KP& P) {
  SWIM_GUARD(P);
  __shared__ uint32_t s_peers[4][MAXF];
  __shared__ uint32_t s_nrec[4][MAXF];          // infectedFrom records found per chosen peer
  __shared__ uint32_t s_rec[4][MAXF][MAXREC];
  __shared__ uint32_t s_lk[4][64];  // the MIXED pass's lack bits, by owner lane
  __shared__ uint2 s_mw[4][4 * SEL_BATCH][64];  // {list entry, holdings word} of this step's MIXED entries
  // this step's window words by (entry, lane): a lane stores its quads' words to wb as 16-B stores
  // (one 4-B store per MIXED position, from whichever lane finished it, cost ~20 B of HBM writes each)
  __shared__ uint32_t s_win[4][4 * SEL_BATCH][64];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t w = threadIdx.x >> 6;
  const uint32_t m = P.row0 + blockIdx.x * 4u + w;
  const uint32_t N = P.N;
  const uint32_t r = P.round;
  const uint32_t lo = P.ctl->scan_lo, hi = P.ctl->scan_hi;
  if (lo >= hi) {  // no live gossip anywhere (a quiet round): nothing is held, sent or swept
    if (lane == 0 && m < P.row0 + P.nloc) P.npeers[m] = 0u;
    if (m == P.dbg_watch && lane == 0) {
      uint32_t* L = P.dbg_log + (r & 255u) * 8u;
      L[0] = r;
      L[1] = L[2] = L[3] = 0u;
      L[4] = L[5] = L[6] = NONE;
    }
    return;
  }
#ifdef SWIM_SEL_PROF  // per-wave phase wall clock (100 MHz), summed: dbg_log u64 [8..11]
  unsigned long long tp = wall_clock64();
#define SEL_MARK(q)                                                                        \
  if (lane == 0) {                                                                         \
    const unsigned long long tn = wall_clock64();                                          \
    atomicAdd(reinterpret_cast<unsigned long long*>(P.dbg_log) + 8 + (q), tn - tp);        \
    tp = tn;                                                                               \
  }
#else
#define SEL_MARK(q)
#endif
  const uint32_t n_act = P.ctl->n_act, w_beg = P.ctl->w_beg;
  const bool mine = m < P.row0 + P.nloc;
  const bool active = mine && P.alive[m] && lo < hi;
  const uint32_t W32 = P.GC >> 5;
  uint32_t others = 0, nclear = 0, hdw = 0, winw = 0, winbits = 0;
  bool win_l = false;
  const bool any = active && P.held[m] > 0u;  // wave-uniform
  if (any) {
    others = P.cnt[m];
    const uint32_t sweep = sweep_rounds(P, others);
    const uint32_t spread = spread_rounds(P, others);
    uint32_t* hbr = P.hb + lrow(P, m) * W32;
    uint32_t* wbr = P.wb + lrow(P, m) * W32;
    uint16_t* mmr = P.mm + lrow(P, m) * W32;
    const bool lack_ok = (n_act + 31u) / 32u <= P.nsumw;  // the list fits the bitmap (as nsum)
    // SEL_BATCH aligned quads of list entries per lane per step: one 16-B list load and (for a
    // quad of consecutive aligned words, the padded layout of k_gossip_prep) one 16-B holdings
    // load each, all issued together (bytes in flight). Words whose class the member's own age
    // bounds settle are finished in a fully unrolled pass (no dynamically indexed register
    // arrays, so nothing goes to scratch); the few left MIXED are finished one by one from a mask.
    for (uint32_t k0 = 0; k0 < n_act; k0 += 256u * SEL_BATCH) {
      uint32_t ev[4 * SEL_BATCH], wv[4 * SEL_BATCH];
#pragma unroll
      for (uint32_t j = 0; j < SEL_BATCH; ++j) {
        const uint32_t kq = k0 + 256u * j + 4u * lane;
        const uint4 a = kq < n_act ? *reinterpret_cast<const uint4*>(P.act + kq) : make_uint4(0u, 0u, 0u, 0u);
        ev[4 * j] = a.x;
        ev[4 * j + 1] = a.y;
        ev[4 * j + 2] = a.z;
        ev[4 * j + 3] = a.w;
      }
#pragma unroll
      for (uint32_t j = 0; j < SEL_BATCH; ++j) {
        const uint32_t kq = k0 + 256u * j + 4u * lane;
        const uint32_t o0 = ev[4 * j] & ACT_OFF_MASK;
        const uint32_t ws0 = wmod(P, w_beg + o0);
        const bool quad = kq + 3u < n_act && (ws0 & 3u) == 0u && (ev[4 * j + 3] & ACT_OFF_MASK) == o0 + 3u;
        if (quad) {
          const uint4 h = *reinterpret_cast<const uint4*>(hbr + ws0);
          wv[4 * j] = h.x;
          wv[4 * j + 1] = h.y;
          wv[4 * j + 2] = h.z;
          wv[4 * j + 3] = h.w;
        } else {
#pragma unroll
          for (uint32_t i = 0; i < 4u; ++i)
            wv[4 * j + i] = kq + i < n_act ? hbr[wmod(P, w_beg + (ev[4 * j + i] & ACT_OFF_MASK))] : 0u;
        }
      }
      uint32_t mixm = 0;  // entries whose infection rounds must be read
      uint32_t lackm = 0;  // entries (sent words) in which the member lacks a live gossip
      uint32_t wbm = 0;  // entries at globally MIXED list positions: their window words go to wb
#pragma unroll 1
      for (uint32_t jq = 0; jq < SEL_BATCH; ++jq) {
        // quad jq's values by select chains (no dynamically indexed register arrays: no scratch)
        uint32_t eq[4], hq[4];
#pragma unroll
        for (uint32_t i = 0; i < 4u; ++i) {
          eq[i] = ev[i];
          hq[i] = wv[i];
#pragma unroll
          for (uint32_t t = 1; t < SEL_BATCH; ++t)
            if (jq == t) {
              eq[i] = ev[4 * t + i];
              hq[i] = wv[4 * t + i];
            }
        }
#pragma unroll
        for (uint32_t i = 0; i < 4u; ++i) {
        const uint32_t j = 4u * jq + i;
        const uint32_t k = k0 + 256u * jq + 4u * lane + i;
        const uint32_t e = eq[i], word = hq[i];
        const uint32_t wi = w_beg + (e & ACT_OFF_MASK);
        const uint32_t wc = (e >> 26) & 3u, sc = (e >> 28) & 3u;
        const uint32_t ws = wmod(P, wi);
        const uint32_t live = k < n_act ? range_mask(wi << 5, lo, hi) : 0u;
        const uint32_t held = word & live;
        uint32_t clear = 0, win = 0;
        s_win[w][j][lane] = 0u;
        if (k < n_act && wc == WC_MIXED) wbm |= 1u << j;
        if (held) {
          uint32_t wcm = wc, scm = sc;
          if (wcm == WC_MIXED || scm == WC_MIXED) {
            // this member's own age range in the word: [r - newest, r - oldest] (mod 2^8)
            const uint32_t mmv = mmr[ws];
            const uint32_t amin = (r - (mmv >> 8)) & 0xFFu, amax = (r - mmv) & 0xFFu;
            if (wcm == WC_MIXED) wcm = amin > spread ? WC_NONE : (amax <= spread ? WC_ALL : WC_MIXED);
            if (scm == WC_MIXED) scm = amax <= sweep ? WC_NONE : (amin > sweep ? WC_ALL : WC_MIXED);
          }
          if (wcm == WC_MIXED || scm == WC_MIXED) {
            mixm |= 1u << j;
            s_mw[w][j][lane] = make_uint2(e, word);  // for the pass below: no list or holdings re-read
            continue;
          }
          if (wcm == WC_ALL) win = held;
          if (scm == WC_ALL) clear = held;
          if (clear) {
            hbr[ws] = word & ~clear;
            nclear += (uint32_t)__popc(clear);
            if (P.leaving[m]) leave_swept(P, m, ws, clear);
          }
        }
        if (k < n_act && wc != WC_NONE) {
          if ((held & ~clear) != live) lackm |= 1u << j;  // a sender may bring it something here
          // a globally ALL word's window is the member's holdings after the sweep, which receivers
          // read directly (k_gossip_pull runs before any holdings change); only MIXED words need wb
          if (wc == WC_MIXED) {
            ++winw;
            s_win[w][j][lane] = win;
          }
          win_l |= win != 0u;
          winbits += slot_gossips(P, ws, win);  // GossipRequests: one per gossip
        }
        }
      }
      auto hd_ld = [&](uint32_t e_, uint4& a_, uint4& b_) {
        const uint32_t wi_ = w_beg + (e_ & ACT_OFF_MASK), ws_ = wmod(P, wi_);
        // (hd4: escapes of the held live slots only; the holdings word is cache-resident)
        hd_load32<HD4>(P, lrow(P, m), ws_, a_, b_, HD4 ? hbr[ws_] & range_mask(wi_ << 5, lo, hi) : 0xFFFFFFFFu);
      };
      // a MIXED entry (list entry e, holdings word, list position k) from its 32 infection rounds:
      // sweep, window, age bounds, wb; true when the member lacks a live gossip of the word
      auto finish_mixed = [&](uint32_t e, uint32_t word, uint32_t j, uint32_t o, uint4 d0, uint4 d1) -> bool {
        const uint32_t wi = w_beg + (e & ACT_OFF_MASK);
        const uint32_t wc = (e >> 26) & 3u;
        const uint32_t ws = wmod(P, wi);
        const uint32_t held = word & range_mask(wi << 5, lo, hi);
        // age = r - infectionPeriod, exact mod 2^8 (every held entry received before round r)
        ++hdw;
        const uint32_t d32[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
        // four ages per dword at once (byte-wise r - round, then 16-bit-lane threshold tests)
        uint32_t over_sweep = 0, over_spread = 0;
        uint32_t ages[8];
#pragma unroll
        for (uint32_t q = 0; q < 8u; ++q) {
          const uint32_t a = bytes_sub(r, d32[q]);
          ages[q] = a;
          over_sweep |= bytes_gt(a, sweep) << (4u * q);
          over_spread |= bytes_gt(a, spread) << (4u * q);
        }
        const uint32_t clear = held & over_sweep;  // sweepGossips
        const uint32_t win = held & ~over_spread;
        const bool lack = wc != WC_NONE && (held & ~clear) != range_mask(wi << 5, lo, hi);
        uint32_t oldest_kept = 0;
        const uint32_t kept = held & ~clear;
        if (clear && kept) {
#pragma unroll
          for (uint32_t q = 0; q < 8u; ++q) {
            const uint32_t a = ages[q] & nibble_bytes((kept >> (4u * q)) & 0xFu);
            oldest_kept = max(oldest_kept, max(max(a & 0xFFu, (a >> 8) & 0xFFu), max((a >> 16) & 0xFFu, a >> 24)));
          }
        }
        if (clear && (held & ~clear)) reinterpret_cast<uint8_t*>(mmr)[2u * ws] = (uint8_t)(r - oldest_kept);  // oldest
        if (clear) {
          hbr[ws] = word & ~clear;
          nclear += (uint32_t)__popc(clear);
          if (P.leaving[m]) leave_swept(P, m, ws, clear);
        }
        if (wc != WC_NONE) {
          if (wc == WC_MIXED) {
            ++winw;
            s_win[w][j][o] = win;
          }
          win_l |= win != 0u;
          winbits += slot_gossips(P, ws, win);  // GossipRequests: one per gossip
        }
        return lack;
      };
      {  // the wave's MIXED entries flattened, one per lane per step: a lane's own entries cluster
         // where the list holds the storm's newest words, and walked per lane the wave waited for
         // the lane with the most (their list entry and holdings word are in s_mw, LDS; C3 select
         // 67.0 -> 64.0 ms per 20 periods)
        s_lk[w][lane] = 0u;
        uint32_t tot;
        const uint32_t off = wave_excl_scan((uint32_t)__popc(mixm), &tot);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        for (uint32_t q0 = 0; q0 < tot; q0 += 64u) {
          const uint32_t q = q0 + lane;
          const uint32_t o = wave_owner_at(off, (uint32_t)__popc(mixm), q0);
          const uint32_t mo = __shfl(mixm, (int)o, 64), oo = __shfl(off, (int)o, 64);
          if (q < tot) {
            const uint32_t j = kth_set_bit(mo, q - oo);
            const uint2 mw = s_mw[w][j][o];
            uint4 d0, d1;
            hd_ld(mw.x, d0, d1);
            if (finish_mixed(mw.x, mw.y, j, o, d0, d1))
              atomicOr(&s_lk[w][o], 1u << j);
          }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        lackm |= s_lk[w][lane];
      }
#pragma unroll
      for (uint32_t jq = 0; jq < SEL_BATCH; ++jq)  // the window words of the lane's quads (positions < n_act <= W32)
        if ((wbm >> (4u * jq)) & 0xFu)
          *reinterpret_cast<uint4*>(wbr + DBG_IDX(k0 + 256u * jq + 4u * lane, W32 - 3u, "select wb4")) =
              make_uint4(s_win[w][4u * jq][lane], s_win[w][4u * jq + 1u][lane], s_win[w][4u * jq + 2u][lane],
                         s_win[w][4u * jq + 3u][lane]);
      if (lack_ok) {  // positions k0 + 256 jq + 4 lane + i: eight lanes fill one bitmap word
#pragma unroll
        for (uint32_t jq = 0; jq < SEL_BATCH; ++jq) {
          uint32_t v = ((lackm >> (4u * jq)) & 0xFu) << (4u * (lane & 7u));
          v |= __shfl_xor(v, 1, 64);
          v |= __shfl_xor(v, 2, 64);
          v |= __shfl_xor(v, 4, 64);
          const uint32_t wq = (k0 + 256u * jq) / 32u + lane / 8u;
          if ((lane & 7u) == 0u && 32u * wq < n_act) P.lack[lrow(P, m) * P.nsumw + wq] = v;
        }
      }
    }
    if (lack_ok && lane == 0) P.lack_round[m] = r;
  }
  SEL_MARK(0);
  uint32_t np = 0;
  if (any) {
    // selectGossipMembers, wave-cooperative: lanes test 64 consecutive positions of the
    // keyed shuffle, ballot, take the first members in position order.
    if (others < P.f) {
      for (uint32_t base = 0; base < N; base += 64u) {
        const uint32_t x = base + lane;
        const bool ok = x < N && x != m && cell_get(P, m, x) != 0u;
        const unsigned long long b = __ballot(ok);
        if (ok) {
          const uint32_t rank = np + (uint32_t)__popcll(b & ((1ull << lane) - 1ull));
          if (rank < (uint32_t)MAXF) s_peers[w][rank] = x;
        }
        np += (uint32_t)__popcll(b);
      }
      if (np > (uint32_t)MAXF) np = MAXF;
    } else {
      const uint32_t half = perm_half_bits(N);
      uint32_t ep = P.g_epoch[m], cur = P.g_cursor[m];
      for (int attempt = 0; attempt < 2; ++attempt) {
        const PermKey key = perm_key(P.seed, K_GOSSIP_PERM, m, ep);
        np = 0;
        uint32_t pos = cur;
        while (pos < N && np < P.f) {
          const uint32_t p = pos + lane;
          uint32_t x = 0;
          bool ok = false;
          if (p < N) {
            x = perm_apply(p, N, half, key);
            ok = x != m && cell_get(P, m, x) != 0u;
          }
          const unsigned long long b = __ballot(ok);
          const uint32_t need = P.f - np;
          const uint32_t have = (uint32_t)__popcll(b);
          if (have >= need) {
            unsigned long long bb = b;  // position of the need-th set bit
            for (uint32_t t = 1; t < need; ++t) bb &= bb - 1ull;
            const uint32_t last = (uint32_t)__builtin_ctzll(bb);
            if (ok && lane <= last) s_peers[w][np + (uint32_t)__popcll(b & ((1ull << lane) - 1ull))] = x;
            np = P.f;
            pos = pos + last + 1u;
            break;
          }
          if (ok) s_peers[w][np + (uint32_t)__popcll(b & ((1ull << lane) - 1ull))] = x;
          np += have;
          pos += 64u;
        }
        if (np == P.f) {
          cur = pos;
          break;
        }
        ++ep;  // reshuffle (GossipProtocolImpl.java:259-262)
        cur = 0;
      }
      if (lane == 0) {
        P.g_epoch[m] = ep;
        P.g_cursor[m] = cur;
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    if (lane < np) P.peers[(size_t)m * P.f + lane] = s_peers[w][lane];
  }
  SEL_MARK(1);
  // spreadGossipsTo is a no-op for an empty window: only non-empty windows reach receivers
  const bool reg = __any(win_l) && np > 0u;
  // GossipRequest messages: every window gossip to every alive peer (GPI:225-239), counted here
  // because receivers that already hold a whole word never look at the senders' windows
  const uint32_t alive_peers = (uint32_t)__popcll(__ballot(reg && lane < np && route(P, s_peers[w][lane]) != NONE));
  winbits = wave_sum(winbits);
  uint32_t entry = m;  // what peer `lane` registers: m, or a pruned pair
  if (reg) {
    // GossipState.isInfected (GPI:248): the peers that delivered to m within the horizon, from
    // m's in-history (newest first, rounds ascending in append order)
    if (lane < MAXF) s_nrec[w][lane] = 0u;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    // the entries appended since round r - hzn (the per-round head history; a stale head is
    // older, so the window only grows): their senders (4 B each), the whole entry on a match
    const uint32_t head = P.ih_head[m];
    uint32_t first = head > IHCAP ? head - IHCAP : 0u;
    if (r >= P.hzn) {
      const uint32_t h0 = P.ih_rhead[lrow(P, m) * 256u + ((r - P.hzn) & 255u)];
      if (h0 > first && h0 <= head) first = h0;
    }
    const uint4* ring = P.ih + lrow(P, m) * IHCAP;
    const uint32_t* snd = P.ih_snd + lrow(P, m) * IHCAP;
    for (uint32_t j = first + lane; j < head; j += 64u) {
      const uint32_t x = snd[j & (IHCAP - 1u)];
      for (uint32_t q = 0; q < np; ++q)
        if (s_peers[w][q] == x) {
          const uint4 e = ring[j & (IHCAP - 1u)];
          if (e.y + P.hzn < r) break;  // too old to suppress anything
          if (e.z == NONE) {  // a delivery predicted never to be sent back: cannot stay exact
            ifrom_overflow(P, IF_MISPREDICT);
          } else {
            const uint32_t c = atomicAdd(&s_nrec[w][q], 1u);
            if (c < MAXREC)
              s_rec[w][q][c] = e.z;
            else
              ifrom_overflow(P, IF_MAXREC);
          }
        }
    }
    if (P.dq) {  // delayed messages from a chosen peer that arrived within the horizon (§3.16)
      uint32_t q0, q1;
      dq_window(P, m, &q0, &q1);
      const uint4* dq = P.dq + lrow(P, m) * P.dqcap;
      for (uint32_t j = q0 + lane; j < q1; j += 64u) {
        const uint4 e = dq[j & (P.dqcap - 1u)];
        if ((e.w & DQ_ARRIVED) && e.z < r && e.z + P.hzn >= r)
          for (uint32_t q = 0; q < np; ++q)
            if (s_peers[w][q] == e.x) atomicOr(&s_nrec[w][q], DQ_PAIR);
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    if (lane < np && s_nrec[w][lane]) {  // this pair's window gets pruned (k_gossip_pairprune / _pairdelay)
      const uint32_t nrc = s_nrec[w][lane] & (DQ_PAIR - 1u);
      const uint32_t nr = nrc < MAXREC ? nrc : MAXREC;
      const uint32_t sp = atomicAdd(&P.ctl->sp_cnt, 1u);
      const uint32_t n4 = (n_act + 3u) & ~3u;  // act-indexed window, padded to quads for k_gossip_pull
      const uint32_t off = atomicAdd(&P.ctl->pw_used, n4);
      if (sp < P.spcap && off + n4 <= P.pwcap && off + n4 >= off) {
        P.sp_list[sp] = make_uint4(m, s_peers[w][lane], nr, off);
        P.sp_dq[sp] = (s_nrec[w][lane] & DQ_PAIR) ? 1u : 0u;
        for (uint32_t c = 0; c < nr; ++c) P.sp_recs[(size_t)sp * MAXREC + c] = s_rec[w][lane][c];
        entry = SPAIR | sp;
      } else {
        ifrom_overflow(P, IF_PAIRS);
      }
    }
  }
  SEL_MARK(2);
  if (reg && lane < np) {
    uint32_t p = s_peers[w][lane];
    if (P.rerouted && route(P, p) != NONE) p = route(P, p);  // the process at p's address receives it
    if (is_local(P, p)) {
      register_sender(P, p, entry);
    } else {  // the window travels to p's shard (k_gossip_pack / k_gossip_unpack)
      const uint32_t dst = p / P.nloc;
      const uint32_t o = atomicAdd(&P.ctl->xg_cnt[dst], 1u);
      uint32_t* e = P.xg_pend + 2 * ((size_t)dst * P.nloc * P.f + o);
      e[0] = entry;
      e[1] = p;
    }
  }
  SEL_MARK(3);
  nclear = wave_sum(nclear);
  if (any && lane == 0 && nclear) P.held[m] -= nclear;
  if (mine && lane == 0) P.npeers[m] = reg ? np : 0u;
  add_stat(P, ST_G_SCANNED, (any && lane == 0) ? n_act : 0u);
  add_stat(P, ST_GOSSIP_SENDS, (reg && lane == 0) ? winbits * alive_peers : 0u);
  if (reg && lane == 0) P.dbg_send[2 * m] += (unsigned long long)winbits * alive_peers;
  if (m == P.dbg_watch && lane == 0) {
    uint32_t* L = P.dbg_log + (r & 255u) * 8u;
    L[0] = r;
    L[1] = reg ? winbits : 0u;
    L[2] = reg ? alive_peers : 0u;
    L[3] = np;
    for (uint32_t q = 0; q < 3u; ++q) L[4 + q] = q < np ? s_peers[w][q] : NONE;
  }
  add_stat(P, ST_G_HDREAD, hdw);
  add_stat(P, ST_G_WINW, winw);
}
__global__ void __launch_bounds__(256, SWIM_SEL_WAVES) k_gossip_select(KP P) { select_body<false>(P); }
__global__ void __launch_bounds__(256, SWIM_SEL_WAVES) k_gossip_select_h4(KP P) { select_body<true>(P); }
// small shards: a workgroup per member

__device__ __forceinline__ uint32_t remote_window(const KP& P, uint32_t i, uint32_t k);

// member m's start-of-round send window at active-list position k, as k_gossip_pull reads it
__device__ __forceinline__ uint32_t own_window(const KP& P, uint32_t m, uint32_t k, uint32_t w_beg, uint32_t lo,
                                               uint32_t hi) {
  const uint32_t ea = P.act[k];
  const uint32_t wc = (ea >> 26) & 3u;
  if (wc == WC_NONE) return 0u;
  const uint32_t W32 = P.GC >> 5;
  const uint32_t wi = w_beg + (ea & ACT_OFF_MASK);
  if (wc == WC_ALL) return P.hb[lrow(P, m) * W32 + (wmod(P, wi))] & range_mask(wi << 5, lo, hi);
  return P.wb[lrow(P, m) * W32 + k];
}

// Pruned pairs (sender m, peer x) of this round: m's window minus every gossip x delivered to m
// (a record of round t) during m's current GossipState of it (selectGossipsToSend's
// !isInfected filter, GossipProtocolImpl.java:245-250). k_gossip_pairfill copies m's window into
// the pair's pw slot, k_gossip_pairprune clears the recorded gossips; k_gossip_pull (or the shard
// exchange) then reads pw instead of wb/hb. Work is split in PCHUNK-position pieces, one wave each.
__global__ void __launch_bounds__(256) k_gossip_pairfill(KP P) {
  SWIM_GUARD(P);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t n = P.ctl->sp_cnt < P.spcap ? P.ctl->sp_cnt : P.spcap;
  const uint32_t n_act = P.ctl->n_act, w_beg = P.ctl->w_beg, lo = P.ctl->scan_lo, hi = P.ctl->scan_hi;
  const uint32_t n4 = (n_act + 3u) & ~3u;
  const uint32_t nch = (n4 + PCHUNK - 1u) / PCHUNK;
  for (uint32_t u = blockIdx.x * 4u + (threadIdx.x >> 6); u < n * nch; u += gridDim.x * 4u) {
    const uint4 sp = P.sp_list[u / nch];
    const uint32_t k1 = min(n4, (u % nch + 1u) * PCHUNK);
    for (uint32_t k = (u % nch) * PCHUNK + lane; k < k1; k += 64u)
      P.pw[sp.w + k] = k < n_act ? own_window(P, sp.x, k, w_beg, lo, hi) : 0u;
  }
}

// A wave per (pair, chunk) walking the pair's records, their headers loaded one per lane in one round
// of loads (a wave per (pair, record slot, chunk), most of them past the pair's records, measured
// slower: C2 3.75 -> 3.62 ms per period, C3 and C4's schedule -0.7 %)
__global__ void __launch_bounds__(256) k_gossip_pairprune(KP P) {
  SWIM_GUARD(P);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t n = P.ctl->sp_cnt < P.spcap ? P.ctl->sp_cnt : P.spcap;
  const uint32_t n_act = P.ctl->n_act, w_beg = P.ctl->w_beg;
  const uint32_t nch = (P.astride + PCHUNK - 1u) / PCHUNK;  // chunks of the longest record
  uint32_t removed_alive = 0;
  for (uint32_t u = blockIdx.x * 4u + (threadIdx.x >> 6); u < n * nch; u += gridDim.x * 4u) {
    const uint32_t i = u / nch, c = u % nch;
    const uint4 sp = P.sp_list[i];
    const uint32_t nr = min(sp.z, (uint32_t)MAXREC);
    uint4 hdr_l = make_uint4(0u, 0u, 0u, 0u);
    uint32_t len_l = 0u;
    if (lane < nr) {
      const uint32_t rec = P.sp_recs[(size_t)i * MAXREC + lane];
      hdr_l = P.rec_hdr[rec & (P.rcap - 1u)];
      len_l = P.rec_len[rec & (P.rcap - 1u)];
    }
    uint32_t removed = 0;
    for (uint32_t j = 0; j < nr; ++j) {  // the pair's records
      const uint32_t t = (uint32_t)__shfl((int)hdr_l.z, (int)j, 64), body = (uint32_t)__shfl((int)hdr_l.w, (int)j, 64);
      const uint32_t len = (uint32_t)__shfl((int)len_l, (int)j, 64);
      if (c * PCHUNK >= len) continue;
      const uint32_t wbt = P.ctl->wbeg_hist[t & 255u];
      const uint32_t* act_t = P.act_ring + (size_t)(t & 255u) * P.astride;
      const uint32_t q1 = min(len, (c + 1u) * PCHUNK);
      for (uint32_t q = c * PCHUNK + lane; q < q1; q += 64u) {
        const uint32_t bits = P.rec_body[(body + q) & (P.bcap - 1u)];
        if (!bits) continue;
        const uint32_t wi = wbt + (act_t[q] & ACT_OFF_MASK);
        if (wi < w_beg) continue;  // every holder has swept the word
        const uint2 ap = P.actpos[wmod(P, wi)];  // listed this round, as this very word?
        if (ap.x != P.round || ap.y >= n_act) continue;
        const uint32_t ea = P.act[ap.y];
        if ((ea & ACT_OFF_MASK) != wi - w_beg || ((ea >> 26) & 3u) == WC_NONE) continue;  // nobody's window
        const uint32_t supp = bits & state_since(P, sp.x, wmod(P, wi), t, bits);
        if (supp) removed += slot_gossips(P, wmod(P, wi), atomicAnd(&P.pw[sp.w + ap.y], ~supp) & supp);
      }
    }
    if (route(P, sp.y) != NONE) {  // the send counter covers alive peers only
      removed_alive += removed;
      if (removed) atomicAdd(&P.dbg_send[2 * sp.x + 1], (unsigned long long)removed);
      if (removed && sp.x == P.dbg_watch) atomicAdd(&P.dbg_log[(P.round & 255u) * 8u + 7u], removed);
    }
  }
  add_stat(P, ST_GOSSIP_SUPP, removed_alive);
  add_stat(P, ST_IF_PAIRS, (blockIdx.x == 0 && threadIdx.x == 0) ? n : 0u);
}

// Pruned pairs whose peer also delivered delayed messages to the sender: every
// such message that arrived within the horizon, during the sender's current GossipState of its
// gossip, takes that gossip out of the pair's window (GossipProtocolImpl.java:181,245-250). One
// wave per pair scans the sender's delayed-message ring.
__global__ void __launch_bounds__(256) k_gossip_pairdelay(KP P) {
  SWIM_GUARD(P);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t n = P.ctl->sp_cnt < P.spcap ? P.ctl->sp_cnt : P.spcap;
  const uint32_t n_act = P.ctl->n_act, w_beg = P.ctl->w_beg, r = P.round;
  uint32_t removed_alive = 0;
  for (uint32_t i = blockIdx.x * 4u + (threadIdx.x >> 6); i < n; i += gridDim.x * 4u) {
    if (!P.sp_dq[i]) continue;  // (uniform per wave)
    const uint4 sp = P.sp_list[i];  // {sender, peer, records, window offset}
    uint32_t q0, q1;
    dq_window(P, sp.x, &q0, &q1);
    const uint4* dq = P.dq + lrow(P, sp.x) * P.dqcap;
    uint32_t removed = 0;
    for (uint32_t j = q0 + lane; j < q1; j += 64u) {
      const uint4 e = dq[j & (P.dqcap - 1u)];  // {peer that sent it, ring slot, arrival round, flags}
      if (e.x != sp.y || !(e.w & DQ_ARRIVED) || e.z >= r || e.z + P.hzn < r) continue;
      const uint32_t ws = wmod(P, e.y >> 5);
      const uint2 ap = P.actpos[ws];  // listed this round, as this very word?
      if (ap.x != r || ap.y >= n_act) continue;
      const uint32_t ea = P.act[ap.y];
      if ((wmod(P, w_beg + (ea & ACT_OFF_MASK))) != ws || ((ea >> 26) & 3u) == WC_NONE) continue;
      const uint32_t supp = (1u << (e.y & 31u)) & state_since(P, sp.x, ws, e.z, 1u << (e.y & 31u));
      if (supp) removed += slot_gossips(P, ws, atomicAnd(&P.pw[sp.w + ap.y], ~supp) & supp);
    }
    if (route(P, sp.y) != NONE) {  // the send counter covers alive peers only
      removed_alive += removed;
      if (removed) atomicAdd(&P.dbg_send[2 * sp.x + 1], (unsigned long long)removed);
    }
  }
  add_stat(P, ST_GOSSIP_SUPP, removed_alive);
}

#define SWIM_REC_ILP 2
constexpr uint32_t REC_ILP = SWIM_REC_ILP;  // k_gossip_record's loss / delay draws per step of a lane
#define SWIM_REC_GRID 1024
constexpr uint32_t REC_GRID = SWIM_REC_GRID;  // k_gossip_record's workgroups (4 waves each, walking the records' chunks)

// word k of a delivery record: what sender entry `sreg` delivered to p this round at active
// position k (its window for p, minus lost messages: the same loss draws as k_gossip_pull).
// (Drawing lazily at pruning time instead was measured slower: a record is pruned against
// several times within its horizon, C2 5.7 vs 5.1 ms/period.)
__device__ __forceinline__ uint32_t delivered_word(const KP& P, uint32_t sreg, uint32_t sid, uint32_t p, uint32_t k,
                                                   uint32_t w_beg, uint32_t lo, uint32_t hi) {
  const uint32_t ea = P.act[k];
  if (((ea >> 26) & 3u) == WC_NONE) return 0u;
  uint32_t v;
  if (sreg & XREC)
    v = remote_window(P, sreg & ~XREC, k);
  else if (sreg & SPAIR)
    v = P.pw[P.sp_list[sreg & ~SPAIR].w + k];
  else
    v = own_window(P, sreg, k, w_beg, lo, hi);
  if (v && (P.loss_mode == 1u || P.delay_on)) {  // this round's deliveries only: not lost, not delayed
    const uint32_t wi = w_beg + (ea & ACT_OFF_MASK);
    const uint32_t* gh = P.g_hash + (wmod(P, wi)) * 32u;
    uint32_t need = v;
    v = 0u;
    while (need) {  // REC_ILP messages per step: their id-hash loads in flight together
      uint32_t bb[REC_ILP], hh[REC_ILP];
#pragma unroll
      for (uint32_t k = 0; k < REC_ILP; ++k) {
        bb[k] = need ? (uint32_t)__builtin_ctz(need) : 32u;
        need &= need - 1u;
      }
#pragma unroll
      for (uint32_t k = 0; k < REC_ILP; ++k) hh[k] = bb[k] < 32u ? gh[bb[k]] : 0u;
#pragma unroll
      for (uint32_t k = 0; k < REC_ILP; ++k) {
        if (bb[k] >= 32u) continue;
        const u32x4 d = draw4(P.seed, K_GOSSIP, sid, p, hh[k], P.tick);
        if (P.loss_mode == 1u && d.x < P.loss_thr) continue;
        if (P.delay_on && delay_of_draw(P, d.y) >= P.gint) continue;
        v |= 1u << bb[k];
      }
    }
  }
  return v;
}

// Recorded deliveries of this round (chosen in k_gossip_inhist): the receiver's
// addToInfected(sender) for every gossip delivered (GossipProtocolImpl.java:181), one word per
// position of this round's active list (kept in act_ring for the record's lifetime). Runs before
// k_gossip_apply changes any holdings; PCHUNK positions per wave.
__global__ void __launch_bounds__(256) k_gossip_record(KP P) {
  SWIM_GUARD(P);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t n = P.ctl->rp_cnt < P.spcap ? P.ctl->rp_cnt : P.spcap;
  const uint32_t n_act = P.ctl->n_act, w_beg = P.ctl->w_beg, lo = P.ctl->scan_lo, hi = P.ctl->scan_hi;
  const uint32_t nch = (n_act + PCHUNK - 1u) / PCHUNK;
  for (uint32_t u = blockIdx.x * 4u + (threadIdx.x >> 6); u < n * nch; u += gridDim.x * 4u) {
    const uint4 rp = P.rp_list[u / nch];  // {in_list entry, receiver, record, sender id}
    const uint32_t off = P.rec_hdr[rp.z & (P.rcap - 1u)].w;
    const uint32_t k1 = min(n_act, (u % nch + 1u) * PCHUNK);
    for (uint32_t k = (u % nch) * PCHUNK + lane; k < k1; k += 64u)
      P.rec_body[(off + k) & (P.bcap - 1u)] = delivered_word(P, rp.x, rp.w, rp.y, k, w_beg, lo, hi);
  }
}

// One wave per receiver p, after every member's selection of the round: each sender whose
// messages can reach p joins p's in-history (round, record); a delivery p may answer with gossips
// of its own within the horizon (may_select on p's post-selection cursor) gets a record, which
// k_gossip_record fills after k_gossip_pull (GossipState.addToInfected, GPI:181).
__global__ void __launch_bounds__(256) k_gossip_inhist(KP P) {
  SWIM_GUARD(P);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t p = P.row0 + blockIdx.x * 4u + (threadIdx.x >> 6);
  if (p >= P.row0 + P.nloc) return;  // whole wave
  if (lane == 0) P.ih_rhead[lrow(P, p) * 256u + (P.round & 255u)] = P.ih_head[p];  // k_gossip_select's window
  const uint32_t deg = P.in_cnt[p];
  if (!deg || !P.alive[p] || P.loss_mode == 2u) return;  // nothing can be delivered
  const uint32_t r = P.round, n_act = P.ctl->n_act;
  uint32_t ihh = P.ih_head[p];
  uint4* ring = P.ih + lrow(P, p) * IHCAP;
  const uint32_t n_ov = deg > INCAP ? P.ctl->n_inov : 0u;
  uint32_t ov_pos = 0;
  uint32_t nrec = 0;
  for (uint32_t done = 0; done < deg;) {
    uint32_t sreg = 0, cdeg = 0;
    if (done == 0) {
      cdeg = deg < INCAP ? deg : INCAP;
      if (lane < cdeg) sreg = P.in_list[(size_t)p * INCAP + lane];
    } else {
      while (cdeg == 0 && ov_pos < n_ov) {  // receivers picked by more than INCAP senders (rare)
        const uint32_t o = ov_pos + lane;
        const bool mine = o < n_ov && P.in_ov[2 * o] == p;
        const unsigned long long b = __ballot(mine);
        if (mine) sreg = P.in_ov[2 * o + 1];  // lanes of a chunk need not be dense here
        cdeg = (uint32_t)__popcll(b);
        if (cdeg) {
          const uint32_t rank = (uint32_t)__popcll(b & ((1ull << lane) - 1ull));
          uint32_t v = 0;
          for (uint32_t t = 0; t < 64u; ++t) {
            const uint32_t x = __shfl(sreg, (int)t, 64), rk = __shfl(rank, (int)t, 64);
            if (((b >> t) & 1ull) && lane == rk) v = x;
          }
          sreg = v;
        }
        ov_pos += 64u;
      }
      if (cdeg == 0) break;
    }
    done += cdeg;
    uint32_t sid = 0;
    if (lane < cdeg) {
      if (sreg & XREC)
        sid = P.rpairs[2 * (sreg & ~XREC)];
      else if (sreg & SPAIR)
        sid = P.sp_list[sreg & ~SPAIR].x;
      else
        sid = sreg;
    }
    const bool ok_l = lane < cdeg && link_open(P, sid, p);
    const unsigned long long reach = __ballot(ok_l);
    uint32_t rec = NONE;
    // may_select per lane; the refinements (a count over up to ~10^3 shuffle positions) by the
    // whole wave, one sender at a time, instead of one long serial loop per lane
    uint32_t mpos = 0;
    bool mwrap = false;
    uint32_t ms = ok_l ? may_select_pre(P, p, sid, &mpos, &mwrap) : 0u;
    for (unsigned long long need = __ballot(ms == 2u); need; need &= need - 1ull) {
      const int q = __builtin_ctzll(need);
      const uint32_t pq = __shfl(mpos, q, 64);
      const bool wq = __shfl((uint32_t)mwrap, q, 64) != 0u;
      const uint32_t ahead = wave_sum(may_select_ahead(P, p, pq, wq, lane, 64u));
      if (lane == (uint32_t)q) ms = may_select_within(P, ahead) ? 1u : 0u;
    }
    if (ok_l && ms == 1u) {
      rec = atomicAdd(&P.ctl->rec_cnt, 1u);
      const uint32_t o = atomicAdd(&P.ctl->rp_cnt, 1u);
      const uint32_t body = atomicAdd(&P.ctl->body_cnt, n_act);
      // the records still inside the horizon start at rs_rec / rs_body of round r - hzn
      if (rec + 1u - P.ctl->rs_rec[(r - P.hzn) & 255u] > P.rcap ||
          body + n_act - P.ctl->rs_body[(r - P.hzn) & 255u] > P.bcap || o >= P.spcap) {
        ifrom_overflow(P, IF_RECORDS);
      } else {
        P.rec_hdr[rec & (P.rcap - 1u)] = make_uint4(sid, p, r, body);
        P.rec_len[rec & (P.rcap - 1u)] = n_act;
        P.rp_list[o] = make_uint4(sreg, p, rec, sid);
        ++nrec;
      }
    }
    if (ok_l) {
      const uint32_t pos = ihh + (uint32_t)__popcll(reach & ((1ull << lane) - 1ull));
      uint4* slot = ring + (pos & (IHCAP - 1u));
      if (pos >= IHCAP && (*slot).y + P.hzn >= r) ifrom_overflow(P, IF_INHIST);
      *slot = make_uint4(sid, r, rec, 0u);
      P.ih_snd[lrow(P, p) * IHCAP + (pos & (IHCAP - 1u))] = sid;
    }
    ihh += (uint32_t)__popcll(reach);
  }
  if (lane == 0) P.ih_head[p] = ihh;
  add_stat(P, ST_IF_RECORDS, nrec);
}

// One wave per receiver p: spreadGossipsTo (GossipProtocolImpl.java:215-251) seen from the
// receiving side. Every sender that picked p sends each gossip of its start-of-round window as
// one GossipRequest (:225-239); p adopts a gossip iff it does not hold it (onGossipReq :171-183).
// So p's first receipts of the round are (U over senders of window & delivered) & ~holds, computed
// in registers per active word: no atomics, every copy delivered in a round has the same effect.
// NetworkEmulator.evaluateLoss draws one value per (sender, receiver, gossip) message and is drawn
// only for gossips p still lacks. Receipts are OR-ed into nb (zero outside a round's receivers);
// receivers with any join alist. Senders come in chunks of <= 64 (in_list, then in_ov).
// a delayed GossipRequest sender -> p of ring slot `slot`, handled in round `arrive` (DESIGN.md
// §3.16): into p's ring (written by p's own pull wave only). The slot's word stays live and listed
// until then: its wlast (the newest infection round any holder may have) is raised to `arrive`,
// which only widens the word's age classes (MIXED instead of ALL / NONE: still exact).
__device__ __forceinline__ void dq_push(const KP& P, uint32_t p, uint32_t sender, uint32_t slot, uint32_t arrive) {
  const uint32_t pos = atomicAdd(&P.dq_head[p], 1u);
  uint4* e = P.dq + lrow(P, p) * P.dqcap + (pos & (P.dqcap - 1u));
  if (pos >= P.dqcap && (*e).z + P.hzn >= P.round) ifrom_overflow(P, IF_DELAYQ);  // in flight / in the horizon
  *e = make_uint4(sender, slot, arrive, 0u);
  const uint32_t ws = slot >> 5;
  if (P.wlast[ws] < arrive) atomicMax(&P.wlast[ws], arrive);
}

#define SWIM_PULL_WAVES 1
// DQ: this handle has delayed-message rings. The delay paths get an instance of
// their own, so the common one keeps its registers (4 waves per SIMD instead of 3).
#define SWIM_PULL_LOSS_ILP 2
constexpr uint32_t PULL_LOSS_ILP = SWIM_PULL_LOSS_ILP;  // loss draws per step of a lane (id-hash loads in flight)
#define SWIM_PULL_SILP 2
constexpr uint32_t PULL_SILP = SWIM_PULL_SILP;  // senders whose window loads a lane issues together


// DQ: message delays are or were on (dq ring); LOSS: the instance the host launches while a
// probabilistic loss is set, whose draws keep several id-hash loads in flight (more registers: the
// common instance keeps the one-at-a-time loop and 4 waves per SIMD).
// SPLIT = 1: one wave per receiver, 4 per workgroup. SPLIT = 4 (small shards, where one wave per
// receiver leaves the SIMDs a few waves each): the workgroup's 4 waves share one receiver, each
// walking every fourth quad of the active list; receipts meet in the LDS summary, the receiver's
// totals are taken after a workgroup barrier (every branch on the receiver is workgroup-uniform).
#ifndef SWIM_PULL_SPLIT_N
#define SWIM_PULL_SPLIT_N 16384
#endif
constexpr uint32_t PULL_SPLIT_N = SWIM_PULL_SPLIT_N;  // shards of at most this many rows (and 16 per CU, swim_handle::split_rows) pull 4 waves per receiver
template <bool DQ, bool LOSS, uint32_t SPLIT = 1u>
__device__ __forceinline__ void pull_body(const KP& P) {
  static_assert(SPLIT == 1u || (SPLIT == 4u && !DQ), "pull_body: one wave per receiver, or a workgroup (no delays)");
  SWIM_GUARD(P);
  __shared__ uint32_t s_sum[4 / SPLIT][NSUM];  // which active words got receipts (bit k of the list)
  __shared__ uint32_t s_snd[4][64];  // the current chunk of sender entries (read in divergent loops)
  __shared__ uint32_t s_sid[4][64];  // ... and their member ids
  __shared__ uint32_t s_pwo[4][64];  // ... and, for pruned pairs, their window offset in pw
  __shared__ uint32_t s_rcpt[4 / SPLIT];  // SPLIT > 1: the receiver's receipts over its waves
  // the lossy instance with a wave per receiver (shards of more than 4,096 rows: C4's) draws flattened
  // across the wave (deliver_flat): C4's schedule at 65,536 pull 7.85 -> 7.40 ms per period; the split
  // instance of small shards keeps each lane's own draws (C2's pull 0.77 -> 0.83 flattened, §6.6)
  constexpr bool FLAT = LOSS && !DQ && SPLIT == 1u;
  __shared__ uint32_t s_u[FLAT ? 4 : 1][FLAT ? 256 : 1];  // FLAT: the delivered bits of a sender's pass, by (lane, word)
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t part = (threadIdx.x >> 6) % SPLIT;  // this wave's share of the receiver's list quads
  const uint32_t p = P.row0 + blockIdx.x * (4u / SPLIT) + (threadIdx.x >> 6) / SPLIT;
  if (p >= P.row0 + P.nloc) return;  // whole wave (SPLIT > 1: the whole workgroup)
  const uint32_t n_act = P.ctl->n_act, w_beg = P.ctl->w_beg;
  const uint32_t W32 = P.GC >> 5;
  const uint32_t deg = P.in_cnt[p];
  uint32_t probes = 0, receipts = 0, words = 0;
  const uint32_t lo = P.ctl->scan_lo, hi = P.ctl->scan_hi;
  uint32_t* sum = s_sum[(threadIdx.x >> 6) / SPLIT];
  const uint32_t nsw = (n_act + 31u) >> 5;
  if ((deg || DQ) && P.alive[p] && n_act) {  // a stopped transport loses every message
    // (SPLIT > 1: deg, liveness and the list length are the receiver's, so every wave of the
    // workgroup takes this branch or none does, and its barriers are uniform)
    uint32_t* hbr = P.hb + lrow(P, p) * W32;
    uint32_t* nbr = P.nb + lrow(P, p) * W32;
    if (DQ && lane == 0)  // where this round's pushes start (dq_window)
      P.dq_rhead[lrow(P, p) * 256u + (P.round & 255u)] = P.dq_head[p];
    // (with delays every message needs its draw, held gossip or not: no skipping)
    const uint32_t* lackr =
        (!(DQ && P.delay_on) && nsw <= P.nsumw && P.lack_round[p] == P.round) ? P.lack + lrow(P, p) * P.nsumw : nullptr;
    if (nsw <= P.nsumw)
      for (uint32_t t = SPLIT > 1u ? threadIdx.x : lane; t < nsw; t += 64u * SPLIT) sum[t] = 0u;
    if (SPLIT > 1u) {
      if (threadIdx.x == 0) s_rcpt[0] = 0u;
      __syncthreads();
    }
    const uint32_t n_ov = deg > INCAP ? P.ctl->n_inov : 0u;
    uint32_t ov_pos = 0;
    for (uint32_t done = 0; done < deg;) {
      const bool first_chunk = done == 0;  // later chunks only add gossips earlier ones did not bring
      // next chunk of senders: lane q holds sender q
      uint32_t sreg = 0, cdeg = 0;
      if (done == 0) {
        cdeg = deg < INCAP ? deg : INCAP;
        if (lane < cdeg) sreg = P.in_list[DBG_IDX((size_t)p * INCAP + lane, (size_t)P.N * INCAP, "pull in_list")];
      } else {
        while (cdeg == 0 && ov_pos < n_ov) {
          const uint32_t o = ov_pos + lane;
          const bool mine = o < n_ov && P.in_ov[DBG_IDX(2ull * o, 2ull * P.N * P.f, "pull in_ov")] == p;
          const unsigned long long b = __ballot(mine);
          const uint32_t rank = (uint32_t)__popcll(b & ((1ull << lane) - 1ull));
          const uint32_t snd = mine ? P.in_ov[2 * o + 1] : 0u;
          // gather: lane `rank` of the chunk takes sender `snd`
          for (uint32_t t = 0; t < 64u; ++t) {
            const uint32_t v = __shfl(snd, (int)t, 64);
            const uint32_t rk = __shfl(rank, (int)t, 64);
            if (((b >> t) & 1ull) && lane == rk) sreg = v;
          }
          cdeg = (uint32_t)__popcll(b);
          ov_pos += 64u;
        }
        if (cdeg == 0) break;  // invariant: in_cnt counts every registration
      }
      done += cdeg;
      // an entry is a local sender's member id, or XREC | index of a pair received from the
      // sender's shard (its window words arrive sparse, see k_gossip_need)
      uint32_t sid = 0, pwo = 0;
      if (lane < cdeg) {
        if (sreg & XREC) {
          sid = P.rpairs[2 * (sreg & ~XREC)];
        } else if (sreg & SPAIR) {
          const uint4 sp = P.sp_list[DBG_IDX(sreg & ~SPAIR, P.spcap, "pull sp_list")];
          sid = sp.x;
          pwo = sp.w;
        } else {
          sid = sreg;
        }
      }
      const bool ok_l = lane < cdeg && P.loss_mode != 2u && link_open(P, sid, p);
      const unsigned long long reach = __ballot(ok_l);
      uint32_t* snd = s_snd[threadIdx.x >> 6];
      snd[lane] = sreg;
      s_sid[threadIdx.x >> 6][lane] = sid;
      s_pwo[threadIdx.x >> 6][lane] = pwo;
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      // lane takes an aligned quad of list entries (k_gossip_prep pads the list into quads of
      // consecutive aligned words): the receiver's holdings, its receipts so far and each
      // sender's window words then come in 16-B loads; other quads fall back to per-word loads
      // one aligned quad of list entries (k_gossip_prep pads the list into quads of consecutive
      // aligned words): the receiver's holdings, its receipts so far and each sender's window words
      // come in 16-B loads; other quads fall back to per-word loads. classify: which of the quad's
      // words can still bring the receiver something (todo); deliver: the senders' windows, the
      // loss draws, the receipts.
      auto classify = [&](uint32_t kq, const uint4& a, uint32_t (&wcv)[4], uint32_t (&wsv)[4], uint32_t (&live)[4],
                          uint32_t (&hw)[4], uint32_t& todo, uint32_t& anyall, uint32_t& anymix, bool& quad,
                          uint32_t& ws0) {
        const uint32_t ea[4] = {a.x, a.y, a.z, a.w};
        const uint32_t o0 = a.x & ACT_OFF_MASK;
        ws0 = wmod(P, w_beg + o0);
        quad = kq + 3u < n_act && (ws0 & 3u) == 0u && (a.w & ACT_OFF_MASK) == o0 + 3u;
        uint4 h4 = make_uint4(0u, 0u, 0u, 0u);
        if (quad) h4 = *reinterpret_cast<const uint4*>(hbr + ws0);
        const uint32_t ha[4] = {h4.x, h4.y, h4.z, h4.w};
        todo = 0;
        anyall = 0;
        anymix = 0;
#pragma unroll
        for (uint32_t i = 0; i < 4u; ++i) {
          const bool in = kq + i < n_act;
          wcv[i] = in ? (ea[i] >> 26) & 3u : WC_NONE;
          const uint32_t wi = w_beg + (ea[i] & ACT_OFF_MASK);
          wsv[i] = wmod(P, wi);
          live[i] = range_mask(wi << 5, lo, hi);
          hw[i] = quad ? ha[i] : (wcv[i] != WC_NONE ? hbr[wsv[i]] : 0u);
          if (wcv[i] == WC_NONE) continue;
          ++words;
          if (!(DQ && P.delay_on) && (hw[i] & live[i]) == live[i]) continue;  // holds every live gossip of the word
          todo |= 1u << i;
          anyall |= wcv[i] == WC_ALL ? 1u : 0u;
          anymix |= wcv[i] == WC_MIXED ? 1u : 0u;
        }
      };
      auto deliver = [&](uint32_t kq, const uint32_t (&wcv)[4], const uint32_t (&wsv)[4], const uint32_t (&live)[4],
                         const uint32_t (&hw)[4], uint32_t todo, uint32_t anyall, uint32_t anymix, bool quad,
                         uint32_t ws0) {
        uint32_t u[4] = {0u, 0u, 0u, 0u}, prev[4] = {0u, 0u, 0u, 0u};
        if (!first_chunk) {  // later chunks only add gossips earlier ones did not bring
          const uint4 p4 = *reinterpret_cast<const uint4*>(nbr + DBG_IDX(kq, W32 - 3u, "pull nbr4"));
          prev[0] = p4.x;
          prev[1] = p4.y;
          prev[2] = p4.z;
          prev[3] = p4.w;
        }
        for (uint32_t q0 = 0; q0 < cdeg; q0 += PULL_SILP) {
          uint32_t wv[PULL_SILP][4], mv[PULL_SILP];
#pragma unroll
          for (uint32_t j = 0; j < PULL_SILP; ++j) {  // the window loads of PULL_SILP senders, issued together
            const bool has = q0 + j < cdeg;
            const uint32_t en = has ? snd[q0 + j] : 0u;
            mv[j] = has ? s_sid[threadIdx.x >> 6][q0 + j] : 0u;
            uint4 wa = make_uint4(0u, 0u, 0u, 0u), wm = make_uint4(0u, 0u, 0u, 0u);
            if (has && (en & SPAIR)) {  // pruned pair: its window was written to pw
              wm = *reinterpret_cast<const uint4*>(
                  P.pw + DBG_IDX((size_t)s_pwo[threadIdx.x >> 6][q0 + j] + kq, P.pwcap - 3u, "pull pw"));  // act-indexed, padded to quads
            } else if (has && !(en & XREC) && quad) {
              if (anyall) wa = *reinterpret_cast<const uint4*>(P.hb + DBG_IDX(lrow(P, en) * W32 + ws0, (size_t)P.nloc * W32 - 3u, "pull hb4"));
              if (anymix) wm = *reinterpret_cast<const uint4*>(P.wb + DBG_IDX(lrow(P, en) * W32 + DBG_IDX(kq, W32 - 3u, "pull wb4 kq"), (size_t)P.nloc * W32 - 3u, "pull wb4"));
            }
            const uint32_t waa[4] = {wa.x, wa.y, wa.z, wa.w}, wma[4] = {wm.x, wm.y, wm.z, wm.w};
#pragma unroll
            for (uint32_t i = 0; i < 4u; ++i) {
              uint32_t v = 0u;
              if (has && ((todo >> i) & 1u)) {
                if (en & XREC)
                  v = remote_window(P, en & ~XREC, kq + i);
                else if (en & SPAIR)
                  v = wma[i];
                else if (quad)
                  v = wcv[i] == WC_ALL ? waa[i] & live[i] : wma[i];
                else
                  v = wcv[i] == WC_ALL ? P.hb[DBG_IDX(lrow(P, en) * W32 + wsv[i], (size_t)P.nloc * W32, "pull hb")] & live[i]
                                       : P.wb[DBG_IDX(lrow(P, en) * W32 + DBG_IDX(kq + i, W32, "pull wb kq"), (size_t)P.nloc * W32, "pull wb")];
              }
              wv[j][i] = v;
            }
          }
#pragma unroll
          for (uint32_t j = 0; j < PULL_SILP; ++j)
#pragma unroll
            for (uint32_t i = 0; i < 4u; ++i) {
              const uint32_t win = wv[j][i];
              if (!win) continue;
              ++probes;
              if (!((reach >> (q0 + j)) & 1ull)) continue;
              uint32_t cand = win & ~hw[i] & ~u[i] & ~prev[i];
              if (DQ && P.delay_on) {  // evaluateLoss + evaluateDelay per message, held gossip or not (§3.16)
                cand = 0u;
                for (uint32_t need = win; need; need &= need - 1u) {
                  const uint32_t b = (uint32_t)__builtin_ctz(need);
                  const u32x4 d = draw4(P.seed, K_GOSSIP, mv[j], p, P.g_hash[wsv[i] * 32u + b], P.tick);
                  if (P.loss_mode == 1u && d.x < P.loss_thr) continue;
                  const uint32_t dr = delay_of_draw(P, d.y) / P.gint;
                  if (dr == 0u)
                    cand |= 1u << b;
                  else
                    dq_push(P, p, mv[j], wsv[i] * 32u + b, P.round + dr);
                }
                cand &= ~hw[i] & ~u[i] & ~prev[i];
              } else if (!LOSS && cand && P.loss_mode == 1u) {  // (the host launches the LOSS instance then)
                uint32_t need = cand;
                cand = 0u;
                while (need) {
                  const uint32_t b = (uint32_t)__builtin_ctz(need);
                  need &= need - 1u;
                  if (draw1(P.seed, K_GOSSIP, mv[j], p, P.g_hash[wsv[i] * 32u + b], P.tick) >= P.loss_thr)
                    cand |= 1u << b;
                }
              } else if (LOSS && cand && P.loss_mode == 1u) {  // NetworkEmulator.evaluateLoss per message
                // two candidates at a time: their id-hash loads in flight together, then their draws
                // (one dependent hash load per candidate was the lossy storm's pull chain)
                uint32_t need = cand;
                cand = 0u;
                while (need) {
                  uint32_t bb[PULL_LOSS_ILP], hh[PULL_LOSS_ILP];
#pragma unroll
                  for (uint32_t k = 0; k < PULL_LOSS_ILP; ++k) {
                    bb[k] = need ? (uint32_t)__builtin_ctz(need) : 32u;
                    need &= need - 1u;
                  }
#pragma unroll
                  for (uint32_t k = 0; k < PULL_LOSS_ILP; ++k) hh[k] = bb[k] < 32u ? P.g_hash[wsv[i] * 32u + bb[k]] : 0u;
#pragma unroll
                  for (uint32_t k = 0; k < PULL_LOSS_ILP; ++k)
                    if (bb[k] < 32u && draw1(P.seed, K_GOSSIP, mv[j], p, hh[k], P.tick) >= P.loss_thr) cand |= 1u << bb[k];
                }
              }
              u[i] |= cand;
            }
        }
        uint32_t sbits = 0;
#pragma unroll
        for (uint32_t i = 0; i < 4u; ++i)
          if (u[i]) {  // holdings are updated by k_gossip_apply, after every receiver has pulled
            nbr[DBG_IDX(kq + i, W32, "pull nbr")] = prev[i] | u[i];
            receipts += (uint32_t)__popc(u[i]);
            sbits |= 1u << ((kq + i) & 31u);
          }
        if (sbits && nsw <= P.nsumw) atomicOr(&sum[kq >> 5], sbits);
      };
      // FLAT (the lossy instance): the loss draws of a sender's messages flattened across the wave, one
      // (word, gossip) per lane per step, instead of each lane drawing its own quad's candidates in a loop
      // (the wave waited for the lane with the most). Every lane takes part in every step (wave-uniform
      // loops; a lane without a quad to visit contributes no draws); a sender's delivered bits meet in LDS
      // (s_u) and return to the quads' lanes before the next sender, whose candidates exclude them, as in
      // deliver (the same draws: NetworkEmulator.evaluateLoss per message, one per gossip until delivered).
      auto deliver_flat = [&](uint32_t kq, const uint32_t (&wcv)[4], const uint32_t (&wsv)[4], const uint32_t (&live)[4],
                              const uint32_t (&hw)[4], uint32_t todo, uint32_t anyall, uint32_t anymix, bool quad,
                              uint32_t ws0) {
        uint32_t* su = s_u[FLAT ? (threadIdx.x >> 6) : 0];
        uint32_t u[4] = {0u, 0u, 0u, 0u}, prev[4] = {0u, 0u, 0u, 0u};
        if (!first_chunk && todo) {
          const uint4 p4 = *reinterpret_cast<const uint4*>(nbr + DBG_IDX(kq, W32 - 3u, "pull nbr4"));
          prev[0] = p4.x;
          prev[1] = p4.y;
          prev[2] = p4.z;
          prev[3] = p4.w;
        }
        for (uint32_t q0 = 0; q0 < cdeg; ++q0) {  // (wave-uniform)
          const uint32_t en = snd[q0], sid = s_sid[threadIdx.x >> 6][q0];
          const bool rch = ((reach >> q0) & 1ull) != 0ull;
          uint4 wa = make_uint4(0u, 0u, 0u, 0u), wm = make_uint4(0u, 0u, 0u, 0u);
          if (todo && (en & SPAIR)) {
            wm = *reinterpret_cast<const uint4*>(P.pw + DBG_IDX((size_t)s_pwo[threadIdx.x >> 6][q0] + kq, P.pwcap - 3u, "pull pw"));
          } else if (todo && !(en & XREC) && quad) {
            if (anyall) wa = *reinterpret_cast<const uint4*>(P.hb + DBG_IDX(lrow(P, en) * W32 + ws0, (size_t)P.nloc * W32 - 3u, "pull hb4"));
            if (anymix) wm = *reinterpret_cast<const uint4*>(P.wb + DBG_IDX(lrow(P, en) * W32 + DBG_IDX(kq, W32 - 3u, "pull wb4 kq"), (size_t)P.nloc * W32 - 3u, "pull wb4"));
          }
          const uint32_t waa[4] = {wa.x, wa.y, wa.z, wa.w}, wma[4] = {wm.x, wm.y, wm.z, wm.w};
          uint32_t cm[4], cnt = 0u;
#pragma unroll
          for (uint32_t i = 0; i < 4u; ++i) {
            uint32_t v = 0u;
            if ((todo >> i) & 1u) {
              if (en & XREC)
                v = remote_window(P, en & ~XREC, kq + i);
              else if (en & SPAIR)
                v = wma[i];
              else if (quad)
                v = wcv[i] == WC_ALL ? waa[i] & live[i] : wma[i];
              else
                v = wcv[i] == WC_ALL ? P.hb[DBG_IDX(lrow(P, en) * W32 + wsv[i], (size_t)P.nloc * W32, "pull hb")] & live[i]
                                     : P.wb[DBG_IDX(lrow(P, en) * W32 + DBG_IDX(kq + i, W32, "pull wb kq"), (size_t)P.nloc * W32, "pull wb")];
            }
            if (v) ++probes;
            cm[i] = rch ? v & ~hw[i] & ~u[i] & ~prev[i] : 0u;
            cnt += (uint32_t)__popc(cm[i]);
          }
          if (P.loss_mode == 1u) {
            uint32_t tot;
            const uint32_t off = wave_excl_scan(cnt, &tot);
            if (tot) {  // (wave-uniform)
#pragma unroll
              for (uint32_t i = 0; i < 4u; ++i) su[4u * lane + i] = 0u;
              __builtin_amdgcn_wave_barrier();
              __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
              for (uint32_t e0 = 0; e0 < tot; e0 += 64u) {
                const uint32_t q = e0 + lane;
                const uint32_t o = wave_owner(off, q);  // (every lane shuffles)
                const uint32_t c0 = __shfl(cm[0], (int)o, 64), c1 = __shfl(cm[1], (int)o, 64);
                const uint32_t c2 = __shfl(cm[2], (int)o, 64), c3 = __shfl(cm[3], (int)o, 64);
                const uint32_t w0 = __shfl(wsv[0], (int)o, 64), w1 = __shfl(wsv[1], (int)o, 64);
                const uint32_t w2 = __shfl(wsv[2], (int)o, 64), w3 = __shfl(wsv[3], (int)o, 64);
                const uint32_t oo = __shfl(off, (int)o, 64);
                if (q < tot) {
                  uint32_t k = q - oo, i = 0u, c = c0, ws = w0;
                  const uint32_t n0 = (uint32_t)__popc(c0), n1 = (uint32_t)__popc(c1), n2 = (uint32_t)__popc(c2);
                  if (k >= n0) {
                    k -= n0, i = 1u, c = c1, ws = w1;
                    if (k >= n1) {
                      k -= n1, i = 2u, c = c2, ws = w2;
                      if (k >= n2) k -= n2, i = 3u, c = c3, ws = w3;
                    }
                  }
                  const uint32_t b = kth_set_bit(c, k);
                  if (draw1(P.seed, K_GOSSIP, sid, p, P.g_hash[ws * 32u + b], P.tick) >= P.loss_thr)
                    atomicOr(&su[4u * o + i], 1u << b);
                }
              }
              __builtin_amdgcn_wave_barrier();
              __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
              for (uint32_t i = 0; i < 4u; ++i) cm[i] = su[4u * lane + i];
              __builtin_amdgcn_wave_barrier();  // (su is cleared by the next pass)
            }
          }
#pragma unroll
          for (uint32_t i = 0; i < 4u; ++i) u[i] |= cm[i];
        }
        uint32_t sbits = 0;
#pragma unroll
        for (uint32_t i = 0; i < 4u; ++i)
          if (u[i]) {
            nbr[DBG_IDX(kq + i, W32, "pull nbr")] = prev[i] | u[i];
            receipts += (uint32_t)__popc(u[i]);
            sbits |= 1u << ((kq + i) & 31u);
          }
        if (sbits && nsw <= P.nsumw) atomicOr(&sum[kq >> 5], sbits);
      };
      if constexpr (FLAT) {
        for (uint32_t kq0 = 256u * part; kq0 < n_act; kq0 += 256u * SPLIT) {  // (wave-uniform)
          const uint32_t kq = kq0 + 4u * lane;
          uint32_t todo = 0u, anyall = 0u, anymix = 0u, ws0 = 0u;
          uint32_t wcv[4] = {WC_NONE, WC_NONE, WC_NONE, WC_NONE}, wsv[4] = {0u, 0u, 0u, 0u};
          uint32_t live[4] = {0u, 0u, 0u, 0u}, hw[4] = {0u, 0u, 0u, 0u};
          bool quad = false;
          if (kq < n_act) {
            const uint32_t lw = lackr ? lackr[kq >> 5] : 0xFFFFFFFFu;
            const uint4 a = *reinterpret_cast<const uint4*>(P.act + kq);
            if ((lw >> (kq & 31u)) & 0xFu) classify(kq, a, wcv, wsv, live, hw, todo, anyall, anymix, quad, ws0);
          }
          if (__any(todo != 0u)) deliver_flat(kq, wcv, wsv, live, hw, todo, anyall, anymix, quad, ws0);
        }
      } else
      for (uint32_t kq = 4u * lane + 256u * part; kq < n_act; kq += 256u * SPLIT) {
        // the receiver's own select pass marked the sent words it lacks something in: skip the
        // rest without reading the holdings (most of them once a storm has spread; compacting the
        // marked quads first measured no faster: the visits are latency-bound). The list quad is
        // loaded beside its lack word, not after it: one round trip per visited quad (C4's schedule
        // pull 8.02 -> 7.82 ms per period; loading the next step's pair ahead too measured slower, §6.5)
        const uint32_t lw = lackr ? lackr[kq >> 5] : 0xFFFFFFFFu;
        const uint4 a = *reinterpret_cast<const uint4*>(P.act + kq);
        if (!((lw >> (kq & 31u)) & 0xFu)) continue;
        uint32_t todo, anyall, anymix, ws0;
        uint32_t wcv[4], wsv[4], live[4], hw[4];
        bool quad;
        classify(kq, a, wcv, wsv, live, hw, todo, anyall, anymix, quad, ws0);
        if (!todo) continue;
        deliver(kq, wcv, wsv, live, hw, todo, anyall, anymix, quad, ws0);
      }

      __builtin_amdgcn_wave_barrier();  // s_snd is rewritten by the next chunk
    }
    if (DQ) {  // delayed messages arriving this round (after the senders' plain nb stores)
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      uint32_t q0, q1;
      dq_window(P, p, &q0, &q1);
      uint4* dq = P.dq + lrow(P, p) * P.dqcap;
      for (uint32_t j = q0 + lane; j < q1; j += 64u) {
        const uint4 e = dq[j & (P.dqcap - 1u)];
        if (e.z != P.round || (e.w & DQ_ARRIVED)) continue;
        dq[j & (P.dqcap - 1u)].w = e.w | DQ_ARRIVED;  // counts for infectedFrom from now on (k_gossip_select)
        const uint32_t ws = wmod(P, e.y >> 5), bit = 1u << (e.y & 31u);
        if (hbr[ws] & bit) continue;  // held (after this round's sweep): no new GossipState
        const uint2 ap = P.actpos[ws];
        if (ap.x != P.round || ap.y >= n_act) {  // the slot's word is kept listed until then (wlast)
          atomicOr(&P.ctl->overflow, OV_BUG);
          continue;
        }
        const uint32_t old = atomicOr(&nbr[ap.y], bit);
        if (!(old & bit)) {
          ++receipts;
          if (nsw <= P.nsumw) atomicOr(&sum[ap.y >> 5], 1u << (ap.y & 31u));
        }
      }
    }
    uint32_t total = wave_sum(receipts);
    if (SPLIT > 1u) {  // the receiver's waves: receipts and summary bits meet in LDS
      if (lane == 0 && total) atomicAdd(&s_rcpt[0], total);
      __syncthreads();
      total = s_rcpt[0];
    }
    if (lane == 0 && part == 0u && total) {
      const uint32_t idx = atomicAdd(&P.ctl->n_alist, 1u);
      P.alist[DBG_IDX(2ull * idx, 2ull * P.N, "pull alist")] = p;
      P.alist[2 * idx + 1] = total;
    }
    if (total && nsw <= P.nsumw) {
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      for (uint32_t t = SPLIT > 1u ? threadIdx.x : lane; t < nsw; t += 64u * SPLIT) P.nsum[lrow(P, p) * P.nsumw + t] = sum[t];
    }
  }
  if (SPLIT > 1u) __syncthreads();  // (the receiver's every wave) all have read in_cnt
  if (lane == 0 && part == 0u) P.in_cnt[p] = 0u;  // ready for the next round
  add_stat(P, ST_G_PROBES, probes);  // (receipts are counted by k_gossip_apply, in gossips)
  add_stat(P, ST_G_PULLW, words);
}

__global__ void __launch_bounds__(256, SWIM_PULL_WAVES) k_gossip_pull(KP P) { pull_body<false, false>(P); }
// the lossy instance at 6 waves per SIMD (80 VGPRs, spilling): C4's schedule pull 170.8 -> 155.4 ms
// per 20 periods; the lossless one loses at any occupancy above its natural 4 (C3 58.2 -> 60.9)
#define SWIM_PULL_LOSS_WAVES 6
__global__ void __launch_bounds__(256, SWIM_PULL_LOSS_WAVES) k_gossip_pull_loss(KP P) {
  pull_body<false, true>(P);
}
__global__ void __launch_bounds__(256, SWIM_PULL_WAVES) k_gossip_pull_dq(KP P) { pull_body<true, true>(P); }
// small shards: a workgroup per receiver
__global__ void __launch_bounds__(256, SWIM_PULL_WAVES) k_gossip_pull_s4(KP P) { pull_body<false, false, 4u>(P); }
__global__ void __launch_bounds__(256, SWIM_PULL_LOSS_WAVES) k_gossip_pull_loss_s4(KP P) {
  pull_body<false, true, 4u>(P);
}

#ifndef SWIM_APPLY_HLOG
#define SWIM_APPLY_HLOG 14
#endif
#define SWIM_APPLY_THREADS 1024
#define SWIM_APPLY_PAIR 1
constexpr uint32_t HCAP_LOG = SWIM_APPLY_HLOG;
constexpr uint32_t HCAP = 1u << HCAP_LOG;  // per-receiver LDS hash slots: 128 KiB of keys + values
constexpr uint32_t HPROBE = 64;            // linear-probe bound; a key that finds no slot spills
constexpr uint32_t SPILL_CAP = 1024;       // spilled subjects per receiver and round (LDS list)
constexpr uint32_t PRES_WORDS = 2048;     // subject-presence bitmap for N <= 65,536
constexpr uint32_t APPLY_THREADS = SWIM_APPLY_THREADS;
// build-time tunables (-DSWIM_APPLY_HLOG / _THREADS): the table init starts at 64 slots, the
// block scan keeps one partial per wave (16 at most), and the kernel's LDS must fit gfx950's 160 KiB
static_assert(HCAP_LOG >= 6 && HCAP_LOG <= 14, "SWIM_APPLY_HLOG out of range");
static_assert(APPLY_THREADS % 64 == 0 && APPLY_THREADS <= 1024, "SWIM_APPLY_THREADS must be a multiple of 64, <= 1024");
static_assert(4 * (2 * HCAP + SPILL_CAP + (SWIM_APPLY_PAIR ? 2 : 1) * PRES_WORDS + 17) <= 160 * 1024,
              "k_gossip_apply LDS over 160 KiB");
// paired receivers split the workgroup into two 512-thread halves of 8 waves each
static_assert(!SWIM_APPLY_PAIR || APPLY_THREADS == 1024, "SWIM_APPLY_PAIR needs SWIM_APPLY_THREADS == 1024");

// exclusive scan over a whole 1,024-thread workgroup, or (pair) over each 512-thread half on its own
__device__ __forceinline__ uint32_t block_excl_scan_part(uint32_t v, uint32_t* total, uint32_t* lds16, bool pair,
                                                         uint32_t half) {
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  uint32_t wt;
  const uint32_t x = wave_excl_scan(v, &wt) + v;  // the wave's inclusive scan (DPP)
  if (lane == 63u) lds16[w] = x;
  __syncthreads();
  const uint32_t k0 = pair ? 8u * half : 0u, k1 = pair ? k0 + 8u : blockDim.x / 64u;
  uint32_t base = 0, tot = 0;
  for (uint32_t k = k0; k < k1; ++k) {
    const uint32_t t = lds16[k];
    if (k < w) base += t;
    tot += t;
  }
  __syncthreads();
  *total = tot;
  return base + x - v;
}

// Membership apply of a round's first receipts: onGossipReq's new-gossip branch
// (GossipProtocolImpl.java:175-180) and onMembershipGossip (MPI:407-414) with the lattice max of
// the records that reached a cell this round. Persistent workgroups take the
// receivers of alist (receiver, receipt count); for receiver p the receipts are nb, cleared on
// the way. They get infectionPeriod r+1 (one 32-B read-modify-write of the word's infection
// rounds). Ring slots of one commit are sorted by (subject, record), so one representative per
// run of one subject carries the run's lattice max; representatives are max-reduced per subject
// in an LDS hash sized to the receipt count. A subject that finds no slot within HPROBE probes
// goes to the spill table instead (consistently for the whole round) and onto an LDS list.
// Then one updateMembership per subject.
template <bool HD4>
__device__ __forceinline__ void apply_body(const KP& P) {
  SWIM_GUARD(P);
  // dynamic LDS sized for the cluster (apply_lds_words): small clusters get a smaller table and
  // two workgroups per CU; 2^apply_hlog table slots (keys, values), the spill list, and (N <=
  // 65,536) the subject-presence bitmap for row-order apply
  extern __shared__ uint32_t s_dyn[];
  const uint32_t hcap_log = P.apply_hlog, hcap = 1u << hcap_log;
  const uint32_t pres_words = P.N <= 32u * PRES_WORDS ? (P.N + 31u) / 32u : 0u;
  __shared__ uint32_t s_nsp[2];
  __shared__ uint32_t s_part[16];
  const uint32_t r = P.round;
  const uint32_t n_act = P.ctl->n_act, w_beg = P.ctl->w_beg, n_list = P.ctl->n_alist;
  const uint32_t W32 = P.GC >> 5;
  Tally T;
  uint32_t created = 0, nwords = 0, nruns = 0, nsubj = 0, nspills = 0, nrcpt = 0;
#ifdef SWIM_APPLY_PROF
  unsigned long long tp = wall_clock64();
#define APPLY_MARK(q)                                                                      \
  if (threadIdx.x == 0) {                                                                  \
    const unsigned long long tn = wall_clock64();                                          \
    atomicAdd(reinterpret_cast<unsigned long long*>(P.dbg_log) + (q), tn - tp);            \
    tp = tn;                                                                               \
  }
#else
#define APPLY_MARK(q)
#endif
  for (uint32_t li = blockIdx.x; li < n_list;) {
    // SWIM_APPLY_PAIR: two receivers at once when both fit half the table, one per half-block
    // (every barrier below is reached by both halves: same phases, same scan count)
    const uint32_t li2 = li + gridDim.x;
    // (8 x receipts <= table: each half's table has room for its compacted items too, so both
    // halves take the same compaction path and meet the same barriers)
    // (a half-table must hold the 64-slot minimum: tables of 128 slots and up)
    const bool pair = SWIM_APPLY_PAIR && hcap_log >= 7u && li2 < n_list && 8u * P.alist[2 * li + 1] <= hcap &&
                      8u * P.alist[2 * li2 + 1] <= hcap && (n_act + 31u) / 32u <= P.nsumw;  // uniform
    const uint32_t half = pair ? (threadIdx.x >> 9) : 0u;
    add_stat(P, ST_APPLY_PAIRS, (pair && threadIdx.x == 0u) ? 1u : 0u);
    const uint32_t tid = pair ? (threadIdx.x & 511u) : threadIdx.x, nthr = pair ? 512u : blockDim.x;
    const uint32_t mli = half ? li2 : li;
    li += pair ? 2u * gridDim.x : gridDim.x;
    const uint32_t hc_log = pair ? hcap_log - 1u : hcap_log;  // this receiver's table: 2^hc_log slots
    uint32_t* s_key = s_dyn + half * (hcap >> 1);
    uint32_t* s_val = s_dyn + hcap + half * (hcap >> 1);
    const uint32_t spill_cap = pair ? SPILL_CAP / 2u : SPILL_CAP;
    uint32_t* s_spl = s_dyn + 2u * hcap + half * (SPILL_CAP / 2u);
    uint32_t* s_pres = s_dyn + 2u * hcap + SPILL_CAP + half * pres_words;
    uint32_t& s_nspill = s_nsp[half];
    const uint32_t p = P.alist[2 * mli], total = P.alist[2 * mli + 1];
    uint32_t* nbr = P.nb + lrow(P, p) * W32;
    uint32_t lg = 6;  // table size >= 2x receipts, 64 .. 2^hc_log
    while (lg < hc_log && (1u << lg) < 2u * total) ++lg;
    const uint32_t hm = (1u << lg) - 1u;
    for (uint32_t t = tid; t <= hm; t += nthr) {
      s_key[t] = NONE;
      s_val[t] = 0u;
    }
    if (tid == 0) s_nspill = 0u;
    const bool pres = P.N <= 32u * PRES_WORDS;
    if (pres)
      for (uint32_t t = tid; t < (P.N + 31u) / 32u; t += nthr) s_pres[t] = 0u;
    __syncthreads();
    APPLY_MARK(0)
    // infection rounds, word liveness, and the lattice max per subject, over the words the
    // receipt summary lists (or every active word when the list is too long to summarize)
    const uint32_t nsw = (n_act + 31u) >> 5;
    const bool summ = nsw <= P.nsumw;
    const uint32_t* sumr = P.nsum + lrow(P, p) * P.nsumw;
    const uint32_t n_items = summ ? nsw * 32u : n_act;
    // per word with receipts: holdings, liveness, age bounds, infection rounds (32-B read-modify-
    // write), then one representative per subject run into the LDS table
    auto process = [&](uint32_t k, uint32_t ws, uint32_t bits, uint32_t prior, uint32_t rs, uint4 v0, uint4 v1) {
      ++nwords;
      nbr[k] = 0u;  // nb is all-zero between rounds
      if (P.wlast[ws] < r + 1u) atomicMax(&P.wlast[ws], r + 1u);
      const size_t mi = lrow(P, p) * W32 + ws;
      P.hb[mi] = prior | bits;  // onGossipReq: the receiver now holds them
      mm_received(P, mi, prior == 0u, r + 1u);  // (prior == 0: the word held nothing before)
      hd_receive<HD4>(P, lrow(P, p), ws, bits, prior, v0, v1, r + 1u);
      // records ascend within a run, so the run's highest receipt carries its lattice max
      rs |= 1u;
      uint32_t left = bits;
      while (left) {
        uint2 sr[4];  // four ring-record loads in flight per lane
        uint32_t nl = 0;
#pragma unroll
        for (uint32_t j = 0; j < 4u; ++j)
          if (left) {
            const uint32_t b = 31u - (uint32_t)__builtin_clz(left);
            const uint32_t below = b == 31u ? 0xFFFFFFFFu : ((2u << b) - 1u);
            const uint32_t a = 31u - (uint32_t)__builtin_clz(rs & below);  // start of b's run
            left &= (1u << a) - 1u;
            sr[j] = P.g_sr[ws * 32u + b];
            ++nl;
            ++nruns;
          }
#pragma unroll
        for (uint32_t j = 0; j < 4u; ++j) {
          if (j >= nl) break;
          if (sr[j].x >= P.N) {  // a user gossip: GossipProtocol.listen() (GossipProtocolImpl.java:176)
            push_event(P, p, sr[j].x - P.N, SWIM_EV_GOSSIP, SWIM_R_MEMBERSHIP_GOSSIP, sr[j].y);
            continue;
          }
          uint32_t h = (sr[j].x * 0x9E3779B1u) >> (32u - lg);
          bool placed = false;
          for (uint32_t q = 0; q < HPROBE; ++q) {
            const uint32_t prev = atomicCAS(&s_key[h], NONE, sr[j].x);
            if (prev == NONE || prev == sr[j].x) {
              atomicMax(&s_val[h], sr[j].y);
              if (prev == NONE && pres) atomicOr(&s_pres[sr[j].x >> 5], 1u << (sr[j].x & 31u));
              placed = true;
              break;
            }
            h = (h + 1u) & hm;
          }
          if (!placed) {  // slots only ever fill up, so this subject spills for the whole round
            const uint32_t c = col_of(P, sr[j].x);
            bool first = false;
            const uint32_t hs = c == NONE ? NONE : spill_put(P, p, c, sr[j].y, &first);
            if (c == NONE) atomicOr(&P.ctl->overflow, OV_TRACK);
            if (first) {
              const uint32_t o = atomicAdd(&s_nspill, 1u);
              if (o < spill_cap)
                s_spl[o] = hs;
              else
                atomicOr(&P.ctl->overflow, OV_SPILL);
            }
          }
        }
      }
    };
    const uint8_t* hdrow = P.hd + lrow(P, p) * P.GC;  // (8-bit rounds; hd4 merges nibbles in hd_receive)
    // The list positions with receipts, compacted from the summary into the table's unused tail:
    // the table has 2^lg >= 2 * total slots and a receipt word holds >= 1 receipt, so when
    // 2^lg < hcap the <= total positions fit in hcap - 2^lg >= 2^lg slots. Otherwise every summary
    // bit is an item and threads test their own.
    const bool compact = summ && lg < hc_log;
    uint32_t* s_items = s_key + (1u << lg);
    uint32_t n_comp = 0;
    if (compact) {
      for (uint32_t c0 = 0; c0 < nsw; c0 += nthr) {
        const uint32_t t = c0 + tid;
        uint32_t bits = t < nsw ? sumr[t] : 0u;
        uint32_t tot;
        uint32_t o = n_comp + block_excl_scan_part((uint32_t)__popc(bits), &tot, s_part, pair, half);
        while (bits) {
          s_items[o++] = 32u * t + (uint32_t)__builtin_ctz(bits);
          bits &= bits - 1u;
        }
        n_comp += tot;
      }
      __syncthreads();
    }
    APPLY_MARK(1)
    const uint32_t n_it = compact ? n_comp : n_items;
    for (uint32_t it0 = 0; it0 < n_it; it0 += 4u * nthr) {
      // four items per thread: their loads are issued together, stage by stage
      uint32_t kv[4], ev[4], bv[4], wsv[4], pv[4], rv[4];
      uint4 v0[4], v1[4];
#pragma unroll
      for (uint32_t j = 0; j < 4u; ++j) {
        const uint32_t it = it0 + j * nthr + tid;
        if (compact) {
          kv[j] = it < n_it ? s_items[it] : NONE;
        } else {
          // summary item = (summary word, bit): consecutive threads share one summary word
          const bool ok = it < n_items && (!summ || ((sumr[it >> 5] >> (it & 31u)) & 1u));
          kv[j] = ok ? it : NONE;
        }
      }
#pragma unroll
      for (uint32_t j = 0; j < 4u; ++j) ev[j] = kv[j] != NONE ? P.act[kv[j]] : 0u;
#pragma unroll
      for (uint32_t j = 0; j < 4u; ++j)
        bv[j] = (kv[j] != NONE && ((ev[j] >> 26) & 3u) != WC_NONE) ? nbr[kv[j]] : 0u;
#pragma unroll
      for (uint32_t j = 0; j < 4u; ++j) {
        wsv[j] = wmod(P, w_beg + (ev[j] & ACT_OFF_MASK));
        if (bv[j]) {
          pv[j] = P.hb[lrow(P, p) * W32 + wsv[j]];
          rv[j] = P.runw[wsv[j]];
          // the infection rounds of a 16-slot half are read only when it keeps some (see process)
          if (!HD4) {
            const uint4* dp = reinterpret_cast<const uint4*>(hdrow + (size_t)wsv[j] * 32u);
            if ((bv[j] & 0xFFFFu) && (pv[j] & 0xFFFFu)) v0[j] = dp[0];
            if ((bv[j] >> 16) && (pv[j] >> 16)) v1[j] = dp[1];
          }
        }
      }
#pragma unroll
      for (uint32_t j = 0; j < 4u; ++j)
        if (bv[j]) process(kv[j], wsv[j], bv[j], pv[j], rv[j], v0[j], v1[j]);
    }
    __syncthreads();
    APPLY_MARK(2)
    const uint32_t snap = P.cnt[p];
    auto apply = [&](uint32_t subj, uint32_t r1) {
      ++nsubj;
      const uint32_t rec = apply_record(P, p, subj, r1, SWIM_R_MEMBERSHIP_GOSSIP, 0u, snap, T);
      if (rec) {  // only onSelfMemberDetected spreads here (reason MEMBERSHIP_GOSSIP): one per round
        emit_gossip(P, p, subj, rec, P.gseq[p]++);
        ++created;
      }
    };
    if (pres) {  // one updateMembership per subject, in subject order: neighbouring threads touch
                 // neighbouring cells of the receiver's row (coalesced, line reuse)
      for (uint32_t t = tid; t < (P.N + 31u) / 32u; t += nthr) {
        uint32_t bits = s_pres[t];
        while (bits) {
          const uint32_t subj = 32u * t + (uint32_t)__builtin_ctz(bits);
          bits &= bits - 1u;
          uint32_t h = (subj * 0x9E3779B1u) >> (32u - lg);
          while (s_key[h] != subj) h = (h + 1u) & hm;  // present: placed within HPROBE probes
          apply(subj, s_val[h]);
        }
      }
    } else {
      for (uint32_t t = tid; t <= hm; t += nthr)  // one updateMembership per subject
        if (s_key[t] != NONE) apply(s_key[t], s_val[t]);
    }
    const uint32_t nsp = s_nspill < spill_cap ? s_nspill : spill_cap;
    if (nsp) __threadfence();
    for (uint32_t t = tid; t < nsp; t += nthr) {  // the spilled subjects' slots of the spill table
      const uint32_t hs = s_spl[t];
      apply(subj_of(P, spill_cell(P, hs)), atomicExch(&P.sp_val[hs], 0u));
    }
    if (tid == 0) atomicAdd(&P.held[p], total);
    nspills += tid == 0 ? nsp : 0u;
    nrcpt += tid == 0 ? total : 0u;  // one gossip per slot here (no batch slots)
    __syncthreads();  // the table is reused by the next receiver
    APPLY_MARK(3)
  }
  add_stat(P, ST_GOSSIPS_CREATED, created);
  add_stat(P, ST_APPLY_WORDS, nwords);
  add_stat(P, ST_APPLY_RUNS, nruns);
  add_stat(P, ST_APPLY_SUBJ, nsubj);
  add_stat(P, ST_APPLY_SPILL, nspills);
  add_stat(P, ST_GOSSIP_RECEIPTS, nrcpt);
  flush_tally(P, T);
}
__global__ void __launch_bounds__(APPLY_THREADS) k_gossip_apply(KP P) { apply_body<false>(P); }
__global__ void __launch_bounds__(APPLY_THREADS) k_gossip_apply_h4(KP P) { apply_body<true>(P); }

// ---- batch slots: k_gossip_apply for rings that hold gossip batches ----
// the highest received slot of every subject run (runw: run starts; a batch slot is a run of
// its own): the slot whose records carry the run's lattice max
__device__ __forceinline__ uint32_t run_tops(uint32_t bits, uint32_t rs) {
  rs |= 1u;
  uint32_t rm = 0;
  while (bits) {
    const uint32_t b = 31u - (uint32_t)__builtin_clz(bits);
    const uint32_t below = b == 31u ? 0xFFFFFFFFu : ((2u << b) - 1u);
    const uint32_t a = 31u - (uint32_t)__builtin_clz(rs & below);
    rm |= 1u << b;
    bits &= (1u << a) - 1u;
  }
  return rm;
}

// onGossipReq's new-gossip branch for one receipt word of receiver p: it holds the slots now
// (GossipProtocolImpl.java:175-178), with infectionPeriod r + 1, and the word's age bounds and
// liveness move with them (k_gossip_apply's `process`, without the record merge)
template <bool HD4>
__device__ __forceinline__ void receive_word(const KP& P, uint32_t p, uint32_t ws, uint32_t bits, uint32_t prior,
                                             uint4 v0, uint4 v1) {
  const uint32_t r = P.round, W32 = P.GC >> 5;
  if (P.wlast[ws] < r + 1u) atomicMax(&P.wlast[ws], r + 1u);
  const size_t mi = lrow(P, p) * W32 + ws;
  P.hb[mi] = prior | bits;
  mm_received(P, mi, prior == 0u, r + 1u);
  hd_receive<HD4>(P, lrow(P, p), ws, bits, prior, v0, v1, r + 1u);
}

// k_gossip_apply when the ring holds batch slots (P.batched): a received slot stands for all the
// gossips of its batch. One WAVE per receiver, AW_WAVES receivers per workgroup, no workgroup
// barriers. The records of every received run top are ORed into the wave's LDS bitmap over the
// record dictionary (one bit per entry); then per block (subject) with set bits
// the lattice max of its set entries is merged: updateMembership when it overrides the cell
// (MembershipRecord.isOverrides, the only records updateMembership acts on, MPI:489-496). A storm
// receiver gets ~10^4..10^5 records of ~10^3..10^4 subjects per round, mostly the same few records
// per subject again: an LDS hash of (subject, max) per receiver spent its time probing and
// spilling there (4.4 s per 100 C3 rounds); a bit per record costs one LDS OR.
// Records without an entry (dictionary out of blocks or ways) take the spill table (lattice max
// per cell; the claimed slots listed in LDS, the round's claimed slots scanned when the list overflows).
// While a subject has such a record live, its bitmap maxima go through the spill table as well, so a subject
// is merged exactly once per round.
#ifndef SWIM_APPLY_WSPILL
#define SWIM_APPLY_WSPILL 128
#endif
constexpr uint32_t AW_SPILL = SWIM_APPLY_WSPILL;  // spilled subjects a wave lists per receiver
constexpr uint32_t AW_WAVES = 4;                  // receivers in flight per workgroup
// 16-B entry-id loads in flight per lane on long ranges: 2 with 16-bit ids (8 per load), 4 with 32-bit
// ids (large dictionaries: the half/half partition at 16,384 44.6 -> 40.3 ms per period; C3, on 16-bit
// ids, 13.90 -> 14.11 at 4)
#define SWIM_AW_VILP 2
#define SWIM_AW_VILP32 4
#define SWIM_AW_QILP 2
constexpr uint32_t AW_QILP = SWIM_AW_QILP;        // 16-B entry-id loads in flight per lane (short ranges)
#define SWIM_AW_LONG 256
// the merge pass tests AW_MC groups of 512 bitmap words (their merge marks) before it flattens their
// blocks to merge together (fewer dependent rounds of loads per receiver than one group at a time)
#define SWIM_AW_MC 1
constexpr uint32_t AW_MC = SWIM_AW_MC;
// bitmap words whose merge marks and block generations one step of the merge pass loads together (4
// measured no faster: C3 13.74 / 13.74 against 13.69 / 13.81 ms per period, with 48 B of scratch, §6.6)
constexpr uint32_t AW_MW = 2;
static_assert(AW_MC >= 1u && AW_MC <= 4u, "SWIM_AW_MC: 1..4 groups of 512 bitmap words");
// record ranges of at least AW_LONG records are walked one at a time by the whole wave; shorter ones
// are flattened into one stream of 16-B quads across the wave
constexpr uint32_t AW_LONG = SWIM_AW_LONG;
// LDS words per wave: the entry bitmap (dsids / 4 words: DICT_WAYS bits per block), the spill list, misc
__host__ __device__ __forceinline__ uint32_t aw_words(uint32_t dsids) { return dsids / 4u + AW_SPILL + 4u; }
static_assert(AW_SPILL >= 1 && AW_SPILL <= 1024, "SWIM_APPLY_WSPILL out of range");

// A grid of as many workgroups as fit the chip, each wave walking the receiver list at a grid stride
// (a wave per possible receiver, the dispatcher handing out the list, measured slower: §6.5).
#define SWIM_AW_MINW 4  // (the LDS bitmap caps the 8,192-block dictionary at 4 waves per SIMD anyway:
                        // registers beyond 128 would only lower that)
// A wave per receiver. (The workgroup's 4 waves sharing one receiver and one LDS bitmap measured
// slower on C2's 4,096 members: apply 0.70 -> 1.13 ms per period, the workgroup barriers; §6.5.)
template <bool HD4, bool C16>
__device__ __forceinline__ void apply_b_body(const KP& P) {
  SWIM_GUARD(P);
  extern __shared__ uint32_t s_dyn[];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
  auto bsync = [] {  // the receiver's wave
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  };
  uint32_t* s_bm = s_dyn + wv * aw_words(P.dsids);  // entry bitmap: all-zero between receivers
  uint32_t* s_spl = s_bm + P.dsids / 4u;
  uint32_t* s_misc = s_spl + AW_SPILL;  // [0] spilled subjects
  const uint32_t n_act = P.ctl->n_act, w_beg = P.ctl->w_beg, n_list = P.ctl->n_alist;
  const uint32_t W32 = P.GC >> 5;
  const uint32_t bw = (min(P.ctl->d_hw, P.dsids) * DICT_WAYS + 31u) >> 5;  // bitmap words in use
  const uint32_t dids = P.dsids * DICT_WAYS;
  constexpr uint32_t IDG = C16 ? 8u : 4u;  // entry ids per 16-B load
  constexpr uint32_t AW_VILP = C16 ? SWIM_AW_VILP : SWIM_AW_VILP32;
  // ids at or above dlim are no entry (16 bits: the two sentinels top an 8,192-block dictionary)
  const uint32_t dlim = C16 ? min(dids, ID16_USER) : dids;
  // a live record has no dictionary entry: the subjects of such records merge through the spill table
  // (their entry records too), so every subject is merged exactly once per round
  const uint32_t c_lo = live_rec_lo(P);
  const bool any_none = (int32_t)(P.ctl->d_none_last - c_lo) > 0;
  Tally T;
  uint32_t created = 0, nwords = 0, nruns = 0, nsubj = 0, nspills = 0, nrecs = 0, nrcpt = 0, nskip = 0;
  auto wsync = [] {
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  };
#ifdef SWIM_APPLY_PROF  // per-wave phase wall clock (100 MHz), summed: dbg_log u64 [4..7]
  unsigned long long tp = wall_clock64();
#define APPLYB_MARK(q)                                                                     \
  if (lane == 0) {                                                                         \
    const unsigned long long tn = wall_clock64();                                          \
    atomicAdd(reinterpret_cast<unsigned long long*>(P.dbg_log) + 4 + (q), tn - tp);        \
    tp = tn;                                                                               \
  }
#else
#define APPLYB_MARK(q)
#endif
  for (uint32_t t = lane; t < bw; t += 64u) s_bm[t] = 0u;
#ifdef SWIM_APPLY_PROF
  unsigned long long t_w = 0, t_big = 0, t_short = 0, tq = 0;  // words / long ranges / short ranges
#define APPLYB_SUB(acc)                \
  {                                    \
    const unsigned long long tn = wall_clock64(); \
    acc += tn - tq;                    \
    tq = tn;                           \
  }
#else
#define APPLYB_SUB(acc)
#endif
  APPLYB_MARK(0);
  for (uint32_t li = blockIdx.x * nwv + wv; li < n_list; li += gridDim.x * nwv) {
    const uint32_t p = P.alist[2 * li], total = P.alist[2 * li + 1];
    uint32_t* nbr = P.nb + lrow(P, p) * W32;
    const uint32_t nsw = (n_act + 31u) >> 5;
    const bool summ = nsw <= P.nsumw;
    const uint32_t* sumr = P.nsum + lrow(P, p) * P.nsumw;
    const uint8_t* hdrow = P.hd + lrow(P, p) * P.GC;
    if (lane == 0) {
      s_misc[0] = 0u;
    }
    bsync();
    bool rowscan = false;  // the spill list overflowed: the round's claimed slots are scanned at the end
    uint32_t ent = 0, rc = 0;
    // lattice max into the receiver's spill-table cell; the key's claimer lists its slot
    auto spill = [&](uint32_t subj, uint32_t rec) {
      const uint32_t c = col_of(P, subj);
      if (c == NONE) {  // N x K: no column for a subject with a live gossip
        atomicOr(&P.ctl->overflow, OV_TRACK);
        return;
      }
      bool first = false;
      const uint32_t hs = spill_put(P, p, c, rec, &first);
      if (first) {
        const uint32_t o = atomicAdd(&s_misc[0], 1u);
        if (o < AW_SPILL)
          s_spl[o] = hs;
        else
          rowscan = true;
      }
    };
    // entry ids of the record ring: IDG per 16-B load (4 of 32 bits, or 8 of 16 bits)
    auto id_load = [&](uint32_t x) -> uint4 {
      return C16 ? *reinterpret_cast<const uint4*>(P.c_id16 + (x & P.cmask))
                 : *reinterpret_cast<const uint4*>(P.c_id + (x & P.cmask));
    };
    auto id_at = [&](const uint4& v, uint32_t k) -> uint32_t {
      const uint32_t w = (k / (IDG / 4u)) == 0u ? v.x : (k / (IDG / 4u)) == 1u ? v.y : (k / (IDG / 4u)) == 2u ? v.z : v.w;
      return C16 ? ((k & 1u) ? (w >> 16) : (w & 0xFFFFu)) : w;
    };
    // record-ring record x of a received run top (ids at or above dlim: a user gossip or no entry)
    auto record = [&](uint32_t x, uint32_t id) {
      if (id < dlim) {
        atomicOr(&s_bm[id >> 5], 1u << (id & 31u));
        return;
      }
      const uint2 sr = P.c_sr[x & P.cmask];
      if (sr.x >= P.N)  // a user gossip: GossipProtocol.listen() (GossipProtocolImpl.java:176)
        push_event(P, p, sr.x - P.N, SWIM_EV_GOSSIP, SWIM_R_MEMBERSHIP_GOSSIP, sr.y);
      else
        spill(sr.x, sr.y);
    };
    // one receipt word per lane (kv = its active-list position, or NONE): holdings, infection
    // rounds and age bounds, then the records of its run tops, flattened across the wave
    auto word = [&](uint32_t kv) {
#ifdef SWIM_APPLY_PROF
      tq = wall_clock64();
#endif
      const uint32_t e = kv != NONE ? P.act[kv] : 0u;
      const uint32_t b0 = kv != NONE ? nbr[kv] : 0u;  // issued beside the list entry, not after it
      const uint32_t bits = ((e >> 26) & 3u) != WC_NONE ? b0 : 0u;
      const uint32_t ws = wmod(P, w_beg + (e & ACT_OFF_MASK));
      uint32_t rm = 0u;
      if (bits) {
        const uint32_t prior = P.hb[lrow(P, p) * W32 + ws];
        const uint32_t rs = P.runw[ws];
        uint4 v0 = make_uint4(0u, 0u, 0u, 0u), v1 = v0;
        if (!HD4) {
          const uint4* dp = reinterpret_cast<const uint4*>(hdrow + (size_t)ws * 32u);
          if ((bits & 0xFFFFu) && (prior & 0xFFFFu)) v0 = dp[0];
          if ((bits >> 16) && (prior >> 16)) v1 = dp[1];
        }
        receive_word<HD4>(P, p, ws, bits, prior, v0, v1);
#ifdef SWIM_APPLY_PROF
        atomicAdd(reinterpret_cast<unsigned long long*>(P.dbg_log) + 14, bits == ~0u ? 1ull : 0ull);
        atomicAdd(reinterpret_cast<unsigned long long*>(P.dbg_log) + 15, 1ull);
#endif
        nbr[kv] = 0u;  // nb is all-zero between rounds
        ++nwords;
        rm = run_tops(bits, rs);
        rc += (uint32_t)(__popc(bits) - __popc(rm));  // slots inside runs: one gossip each
        nruns += (uint32_t)__popc(rm);
      }
      uint32_t tot;
      const uint32_t off = wave_excl_scan((uint32_t)__popc(rm), &tot);
      for (uint32_t q0 = 0; q0 < tot; q0 += 64u) {
        const uint32_t q = q0 + lane;
        const uint32_t o = wave_owner_at(off, (uint32_t)__popc(rm), q0);
        const uint32_t mo = __shfl(rm, (int)o, 64), wo = __shfl(ws, (int)o, 64), oo = __shfl(off, (int)o, 64);
        uint2 cr = make_uint2(0u, 0u), si = cr;
        const uint32_t slq = wo * 32u + kth_set_bit(mo, q - oo);  // the run top's ring slot
        if (q < tot) {
          cr = P.g_cref[slq];
          if (C16) si = P.g_sid[slq];  // (issued beside the range, not after it)
        }
        const uint32_t len = cr.y - cr.x;
        ent += len;
        // ranges of at most SID_INLINE records: their ids came with the range (k_slot_ids)
        const bool inl = C16 && len != 0u && len <= SID_INLINE;
        if (inl) {
#pragma unroll
          for (uint32_t k = 0; k < SID_INLINE; ++k)
            if (k < len) record(cr.x + k, ((k < 2u ? si.x : si.y) >> (16u * (k & 1u))) & 0xFFFFu);
        }
#ifdef SWIM_APPLY_PROF
        if (__any(len != 0u)) APPLYB_SUB(t_w);
#endif
#ifdef SWIM_APPLY_PROF  // receipt words received whole, and the records they carry: dbg_log u64 [12..16]
        {
          const bool fw = __shfl((uint32_t)(bits == ~0u), (int)o, 64) != 0u;
          const unsigned long long rf = wave_sum(fw && q < tot ? len : 0u), ra = wave_sum(q < tot ? len : 0u);
          const unsigned long long rl = wave_sum(q < tot && len >= 64u ? len : 0u);
          if (lane == 0) {
            atomicAdd(reinterpret_cast<unsigned long long*>(P.dbg_log) + 16, rl);
            atomicAdd(reinterpret_cast<unsigned long long*>(P.dbg_log) + 12, rf);
            atomicAdd(reinterpret_cast<unsigned long long*>(P.dbg_log) + 13, ra);
          }
        }
#endif
        // long ranges (batches): the whole wave walks each, 16-B loads of entry ids per lane (4 ids,
        // or 8 of 16 bits)
        unsigned long long big = __ballot(len >= AW_LONG);
        while (big) {
          const int L = __builtin_ctzll(big);
          big &= big - 1ull;
          const uint32_t b0 = __shfl(cr.x, L, 64), b1 = __shfl(cr.y, L, 64);
          if (b1 - b0 >= bw && P.rb_cap) {  // the range's entry bitmap, if its commit built one (k_slot_bm)
            const uint32_t sl = __shfl(slq, L, 64);
            uint32_t rb = P.g_rb[sl];
            if (rb != NONE && P.rb_tag[rb] != b0) rb = NONE;  // (taken by a newer range since)
            if (rb != NONE) {  // (uniform)
              const uint32_t nbw = P.dsids / 4u;
              const uint32_t* src = P.rb_bits + (size_t)rb * nbw;
              for (uint32_t t = 4u * lane; t < bw; t += 256u) {
                if (t + 3u < nbw) {
                  const uint4 v = *reinterpret_cast<const uint4*>(src + t);
                  s_bm[t] |= v.x;
                  s_bm[t + 1u] |= v.y;
                  s_bm[t + 2u] |= v.z;
                  s_bm[t + 3u] |= v.w;
                } else {
                  for (uint32_t k = 0; t + k < bw; ++k) s_bm[t + k] |= src[t + k];
                }
              }
              if (lane == 0) {
                unsigned long long* st = P.stat_shards + (blockIdx.x & (STAT_SHARDS - 1u)) * STAT_STRIDE;
                atomicAdd(&st[ST_APPLY_RBM], 1ull);
                atomicAdd(&st[ST_APPLY_RBREC], (unsigned long long)(b1 - b0));
              }
              continue;
            }
          }
          // aligned 16-B groups of entry ids from the group holding b0: IDG records per lane per load
          const uint32_t a0 = b0 & ~(IDG - 1u), span = b1 - a0;
          for (uint32_t x0 = 0; x0 < span; x0 += 64u * IDG * AW_VILP) {
            uint4 v[AW_VILP];
#pragma unroll
            for (uint32_t u = 0; u < AW_VILP; ++u) {
              const uint32_t d = x0 + 64u * IDG * u + IDG * lane;
              v[u] = d < span ? id_load(a0 + d) : make_uint4(0u, 0u, 0u, 0u);
            }
#pragma unroll
            for (uint32_t u = 0; u < AW_VILP; ++u) {
              const uint32_t x = a0 + x0 + 64u * IDG * u + IDG * lane;
#pragma unroll
              for (uint32_t k = 0; k < IDG; ++k)
                if ((x + k - b0) < (b1 - b0)) record(x + k, id_at(v[u], k));
            }
          }
        }
        APPLYB_SUB(t_big);
        // short ranges (single gossips, small batches): their aligned 16-B groups of entry ids
        // flattened across the lanes, one group per lane per load (one owner search per group). (Walking
        // ranges of at most one / two / three groups by their own lane instead, without the owner
        // search, measured slower: C3 apply 6.41 -> 6.47 / 6.60 / 6.98 ms per period, §6.6: the lanes'
        // ranges are uneven.)
        {
          const bool sh = len != 0u && len < AW_LONG && !inl;
          const uint32_t nq = sh ? ((cr.x & (IDG - 1u)) + len + IDG - 1u) / IDG : 0u;
          uint32_t qtot;
          const uint32_t qoff = wave_excl_scan(nq, &qtot);
          for (uint32_t e0 = 0; e0 < qtot; e0 += 64u * AW_QILP) {
            uint4 v[AW_QILP];
            uint32_t qb[AW_QILP], bx[AW_QILP], bl[AW_QILP];
#pragma unroll
            for (uint32_t u = 0; u < AW_QILP; ++u) {
              const uint32_t ee = e0 + 64u * u + lane;
              const uint32_t eo = wave_owner_at(qoff, nq, e0 + 64u * u);
              // (every lane shuffles: a lane past qtot may own nothing yet be another lane's source)
              bx[u] = __shfl(cr.x, (int)eo, 64);
              const uint32_t lo = __shfl(len, (int)eo, 64), oo = __shfl(qoff, (int)eo, 64);
              bl[u] = ee < qtot ? lo : 0u;
              qb[u] = (bx[u] & ~(IDG - 1u)) + IDG * (ee - oo);
              v[u] = ee < qtot ? id_load(qb[u]) : make_uint4(0u, 0u, 0u, 0u);
            }
#pragma unroll
            for (uint32_t u = 0; u < AW_QILP; ++u) {
#pragma unroll
              for (uint32_t k = 0; k < IDG; ++k)
                if ((qb[u] + k - bx[u]) < bl[u]) record(qb[u] + k, id_at(v[u], k));
            }
          }
        }
        APPLYB_SUB(t_short);
      }
    };
    if (!summ) {
      for (uint32_t it0 = 0; it0 < n_act; it0 += 64u) word(it0 + lane < n_act ? it0 + lane : NONE);
    } else {  // the summary's set bits, flattened across the wave
      for (uint32_t c0 = 0; c0 < nsw; c0 += 64u) {
        const uint32_t sb = c0 + lane < nsw ? sumr[c0 + lane] : 0u;
        uint32_t tot;
        const uint32_t off = wave_excl_scan((uint32_t)__popc(sb), &tot);
        for (uint32_t q0 = 0; q0 < tot; q0 += 64u) {
          const uint32_t q = q0 + lane;
          const uint32_t o = wave_owner_at(off, (uint32_t)__popc(sb), q0);
          const uint32_t bo = __shfl(sb, (int)o, 64), oo = __shfl(off, (int)o, 64);
          word(q < tot ? 32u * (c0 + o) + kth_set_bit(bo, q - oo) : NONE);
        }
      }
    }
    {
      const uint32_t E = wave_sum(ent), R = wave_sum(rc) + E;
      if (lane == 0) {
        nrcpt += R;
        nrecs += E;
      }
    }
    bsync();  // every record of the receiver is in the bitmap
    APPLYB_MARK(1);
    const uint32_t snap = P.cnt[p];
    uint32_t* mrow = P.dmark + lrow(P, p) * P.dsids;  // the receiver's merge marks
    auto apply = [&](uint32_t subj, uint32_t r1) {
      ++nsubj;
      const uint32_t rec = apply_record(P, p, subj, r1, SWIM_R_MEMBERSHIP_GOSSIP, 0u, snap, T);
      if (rec) {  // only onSelfMemberDetected spreads here (reason MEMBERSHIP_GOSSIP): one per round
        emit_gossip(P, p, subj, rec, P.gseq[p]++);
        ++created;
      }
    };
    // per block with set entries: the max of its set entries' records, merged once. The blocks
    // with set bits of 512 bitmap words are flattened across the wave (one block per lane: its
    // eight entry records in two 16-B loads beside its subject), then the words are cleared.
    static_assert(DICT_WAYS == 8, "a bitmap byte per block");
    // The merge marks are read with the bitmap words (a lane's word covers 4 blocks: their 4 marks
    // and generations are one 16-B load each, consecutive lanes consecutive lines), so the blocks whose set entries are all marked drop out before the per-block pass.
    const uint4* mrow4 = reinterpret_cast<const uint4*>(mrow);
    const uint4* gen4 = reinterpret_cast<const uint4*>(P.d_gen);
    // AW_MC groups of 512 bitmap words are tested, then their blocks to merge flattened together
    for (uint32_t t0 = 0; t0 < bw; t0 += 512u * AW_MC) {
      uint32_t bm[AW_MC];  // bit 4u + j of bm[ci]: word t0 + 512 ci + 64u + lane has set entries in its block j, not all marked
      uint32_t nzw = 0u;   // bit 8 ci + u: that word has set entries
#pragma unroll
      for (uint32_t ci = 0; ci < AW_MC; ++ci) {
      bm[ci] = 0u;
#pragma unroll
      for (uint32_t h2 = 0; h2 < 8u / AW_MW; ++h2) {  // (AW_MW words in flight per step: registers)
        uint32_t wv[AW_MW];
        uint4 mv[AW_MW], gv[AW_MW];
#pragma unroll
        for (uint32_t uu = 0; uu < AW_MW; ++uu) {
          const uint32_t t = t0 + 512u * ci + 64u * (AW_MW * h2 + uu) + lane;
          wv[uu] = t < bw ? s_bm[t] : 0u;
          mv[uu] = wv[uu] ? mrow4[t] : make_uint4(0u, 0u, 0u, 0u);
          gv[uu] = wv[uu] ? gen4[t] : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (uint32_t uu = 0; uu < AW_MW; ++uu) {
          const uint32_t u = AW_MW * h2 + uu;
          if (wv[uu]) nzw |= 1u << (8u * ci + u);
          const uint32_t mk[4] = {mv[uu].x, mv[uu].y, mv[uu].z, mv[uu].w};
          const uint32_t gg[4] = {gv[uu].x, gv[uu].y, gv[uu].z, gv[uu].w};
#pragma unroll
          for (uint32_t j = 0; j < 4u; ++j) {
            const uint32_t m = (wv[uu] >> (8u * j)) & 0xFFu;
            if (!m) continue;
            if ((mk[j] >> 8) == (gg[j] & GEN_MASK) && (m & ~mk[j] & 0xFFu) == 0u)
              ++nskip;  // every set entry already found not to override the present cell (MPI:489)
            else
              bm[ci] |= 1u << (4u * u + j);
          }
        }
      }
      }
      uint32_t cnt = 0u;
#pragma unroll
      for (uint32_t ci = 0; ci < AW_MC; ++ci) cnt += (uint32_t)__popc(bm[ci]);
      uint32_t tot;
      const uint32_t off = wave_excl_scan(cnt, &tot);
      for (uint32_t q0 = 0; q0 < tot; q0 += 64u) {
        const uint32_t q = q0 + lane;
        const uint32_t o = wave_owner_at(off, cnt, q0);
        const uint32_t oo = __shfl(off, (int)o, 64);
        // the owner's (q - oo)-th block: which of its AW_MC masks, then which bit
        uint32_t kk = q - oo, bo = 0u, cs = 0u;
        bool found = false;
#pragma unroll
        for (uint32_t ci = 0; ci < AW_MC; ++ci) {
          const uint32_t bc = __shfl(bm[ci], (int)o, 64);  // (every lane shuffles)
          const uint32_t c = (uint32_t)__popc(bc);
          if (!found) {
            if (kk < c) {
              bo = bc;
              cs = ci;
              found = true;
            } else {
              kk -= c;
            }
          }
        }
        if (q < tot) {
          const uint32_t b = kth_set_bit(bo, kk);
          const uint32_t t = t0 + 512u * cs + 64u * (b >> 2) + o, j = b & 3u;
          const uint32_t base = 32u * t + 8u * j;  // entry id of the block's way 0
          const uint32_t sid = base / DICT_WAYS;
          const uint32_t m = (s_bm[t] >> (8u * j)) & 0xFFu;
          uint32_t* mkp = mrow + sid;
          const uint32_t mk = *mkp, g = P.d_gen[sid] & GEN_MASK;  // (lines the scan just read)
          const uint4* dr = reinterpret_cast<const uint4*>(P.d_rec + base);
          const uint4 r0 = dr[0], r1 = dr[1];
          const uint32_t subj = P.d_subj[sid];
          const bool mvalid = (mk >> 8) == g;
          uint32_t best = max(max((m & 1u) ? r0.x : 0u, (m & 2u) ? r0.y : 0u),
                              max((m & 4u) ? r0.z : 0u, (m & 8u) ? r0.w : 0u));
          best = max(best, max(max((m & 16u) ? r1.x : 0u, (m & 32u) ? r1.y : 0u),
                               max((m & 64u) ? r1.z : 0u, (m & 128u) ? r1.w : 0u)));
          if (any_none && (int32_t)(P.none_last[subj] - c_lo) > 0) {
            spill(subj, best);
          } else {
            const uint32_t c = cell_get(P, p, subj);
            if (is_overrides(best, c) || (P.nxk && P.colmap[subj] == NONE)) {  // (the latter: OV_TRACK)
              apply(subj, best);
            } else {
              ++nsubj;
              // no set entry overrides the present cell: mark them (an absent cell is not
              // marked: a record that does not override it may override a re-added one)
              const uint32_t nm = (g << 8) | (((mvalid ? mk : 0u) | m) & 0xFFu);
              if (c != SWIM_ABSENT && nm != mk) *mkp = nm;
            }
          }
        }
      }
      wsync();  // every lane has read its blocks' bits
#pragma unroll
      for (uint32_t u = 0; u < 8u * AW_MC; ++u)
        if ((nzw >> u) & 1u) s_bm[t0 + 512u * (u >> 3) + 64u * (u & 7u) + lane] = 0u;
    }
    bsync();  // every merge of the receiver is done, its spill list complete
    APPLYB_MARK(2);
    const uint32_t nsp = min(s_misc[0], AW_SPILL);
    if (__any(rowscan)) {  // every spilled subject: this row's keys among the round's claimed slots
      __threadfence();
      const uint32_t nu = min(atomicAdd(&P.ctl->sp_n, 0u), P.spmask + 1u);
      const unsigned long long k0 = lrow(P, p) * (unsigned long long)P.W + 1ull, k1 = k0 + P.W;
      for (uint32_t t = lane; t < nu; t += 64u) {
        const uint32_t hs = P.sp_used[t];  // (another wave's entry may still be stale: keys filter it)
        const unsigned long long k = P.sp_key[hs];
        if (k < k0 || k >= k1) continue;
        const uint32_t v = atomicExch(&P.sp_val[hs], 0u);
        if (v) apply(subj_of(P, (uint32_t)(k - k0)), v);
      }
    } else {
      if (nsp) __threadfence();
      for (uint32_t t = lane; t < nsp; t += 64u) {
        const uint32_t hs = s_spl[t];
        apply(subj_of(P, spill_cell(P, hs)), atomicExch(&P.sp_val[hs], 0u));
      }
    }
    if (lane == 0) atomicAdd(&P.held[p], total);
    nspills += lane == 0 ? s_misc[0] : 0u;
    bsync();  // the spill counter is reset for the next receiver
    APPLYB_MARK(3);
  }
  add_stat(P, ST_GOSSIPS_CREATED, created);
  add_stat(P, ST_APPLY_WORDS, nwords);
  add_stat(P, ST_APPLY_RUNS, nruns);
  add_stat(P, ST_APPLY_SUBJ, nsubj);
  add_stat(P, ST_APPLY_SPILL, nspills);
  add_stat(P, ST_APPLY_RECS, nrecs);
  add_stat(P, ST_GOSSIP_RECEIPTS, nrcpt);
  add_stat(P, ST_APPLY_SKIP, nskip);
#ifdef SWIM_APPLY_PROF
  if (lane == 0) {
    atomicAdd(reinterpret_cast<unsigned long long*>(P.dbg_log) + 17, t_w);
    atomicAdd(reinterpret_cast<unsigned long long*>(P.dbg_log) + 18, t_big);
    atomicAdd(reinterpret_cast<unsigned long long*>(P.dbg_log) + 19, t_short);
  }
#endif
  flush_tally(P, T);
}
__global__ void __launch_bounds__(64 * AW_WAVES, SWIM_AW_MINW) k_gossip_apply_b(KP P) { apply_b_body<false, false>(P); }
__global__ void __launch_bounds__(64 * AW_WAVES, SWIM_AW_MINW) k_gossip_apply_b_h4(KP P) { apply_b_body<true, false>(P); }
__global__ void __launch_bounds__(64 * AW_WAVES, SWIM_AW_MINW) k_gossip_apply_b16(KP P) { apply_b_body<false, true>(P); }
__global__ void __launch_bounds__(64 * AW_WAVES, SWIM_AW_MINW) k_gossip_apply_b16_h4(KP P) { apply_b_body<true, true>(P); }
// small shards: a workgroup per receiver (16-bit ids: dictionaries of at most 8,192 blocks)

// hd4 handles, once a period: escape entries whose slot the row no longer holds with nibble 15
// (swept, or rewritten with a small offset) become tombstones, so the table holds only live escapes
__global__ void k_hx_sweep(KP P) {
  uint32_t live = 0;
  for (uint32_t h = blockIdx.x * blockDim.x + threadIdx.x; h <= P.hxmask; h += gridDim.x * blockDim.x) {
    const unsigned long long v = P.hx[h];
    if (v == HX_EMPTY || v == HX_TOMB) continue;
    const unsigned long long key = (v >> 8) - 1ull;
    const size_t row = (size_t)(key / P.GC);
    const uint32_t sl = (uint32_t)(key % P.GC);
    const bool held = (P.hb[row * (P.GC >> 5) + (sl >> 5)] >> (sl & 31u)) & 1u;
    const uint32_t nib = (P.hd[row * (P.GC / 2u) + (sl >> 1)] >> (4u * (sl & 1u))) & 0xFu;
    if (!held || nib != 15u)
      P.hx[h] = HX_TOMB;
    else
      ++live;
  }
  // the live entries (the table's load: SWIM_EOVERFLOW mask 256 once an insert probes 64 slots)
  uint32_t wl;
  (void)wave_excl_scan(live, &wl);
  if ((threadIdx.x & 63u) == 0u && wl) atomicAdd(&P.ctl->hx_live, wl);
}

// ---------------------------------------------------------------------------------------
// Cross-shard exchange (world > 1): pack before the host's collective, unpack after it.
// ---------------------------------------------------------------------------------------
// locate record g of the send layout: destination shards in rank order, `cnt` records each
__device__ __forceinline__ bool xrec_locate(const KP& P, const uint32_t* cnt, uint32_t g, uint32_t* dst,
                                            uint32_t* idx) {
  for (uint32_t q = 0; q < P.world; ++q) {
    if (g < cnt[q]) {
      *dst = q;
      *idx = g;
      return true;
    }
    g -= cnt[q];
  }
  return false;
}

// Cross-shard gossip delivery asks before it ships: (1) the sender shard sends its (sender,
// receiver) registrations; (2) the receiver shard answers, per pair, a bitmap over the round's
// active list of the words the receiver still lacks something in (exactly the words
// k_gossip_pull will look at); (3) the sender shard ships the window words of those positions
// only. After a storm, when everyone holds everything, (3) is empty.

// (1) registrations [sender, receiver], destination shards in rank order
__global__ void k_gossip_pack_pairs(KP P, uint32_t n_rec) {
  SWIM_GUARD(P);
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t dst, i;
  if (g < n_rec && xrec_locate(P, P.ctl->xg_cnt, g, &dst, &i)) {
    const uint32_t* e = P.xg_pend + 2 * ((size_t)dst * P.nloc * P.f + i);
    P.xsend[2 * g] = (e[0] & SPAIR) ? P.sp_list[e[0] & ~SPAIR].x : e[0];
    P.xsend[2 * g + 1] = e[1];
  }
}

__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t* total, uint32_t* lds4);

// block-wide exclusive scan of 4 consecutive values per thread (blockDim = 256)
__device__ __forceinline__ void scan4_256(const uint32_t v[4], uint32_t out[4], uint32_t* total, uint32_t* lds4) {
  const uint32_t loc = v[0] + v[1] + v[2] + v[3];
  const uint32_t base = block_excl_scan256(loc, total, lds4);
  out[0] = base;
  out[1] = base + v[0];
  out[2] = out[1] + v[1];
  out[3] = out[2] + v[2];
}

// (2) receiver shard: keep the received pairs, compute each pair's need bitmap (kept for the
// pull, and sent back), its per-word prefix counts and its total
__global__ void __launch_bounds__(256) k_gossip_need(KP P, uint32_t n_pairs, uint32_t nneed) {
  SWIM_GUARD(P);
  __shared__ uint32_t s_lds4[4];
  const uint32_t n_act = P.ctl->n_act, w_beg = P.ctl->w_beg, lo = P.ctl->scan_lo, hi = P.ctl->scan_hi;
  const uint32_t W32 = P.GC >> 5;
  for (uint32_t i = blockIdx.x; i < n_pairs; i += gridDim.x) {
    const uint32_t p = P.xrecv[2 * i + 1];
    if (threadIdx.x == 0) {
      P.rpairs[2 * i] = P.xrecv[2 * i];
      P.rpairs[2 * i + 1] = p;
    }
    const uint32_t* hbr = P.hb + lrow(P, p) * W32;
    // a delivery p will record (infectedFrom, k_gossip_record) needs the whole window; with message
    // delays every message of the window draws its loss and delay, held gossip or not (k_gossip_pull_dq)
    const bool all = P.alive[p] && P.loss_mode != 2u && link_open(P, P.xrecv[2 * i], p) &&
                     (P.delay_on || may_select(P, p, P.xrecv[2 * i]));
    uint32_t cnt[4], pre[4];
#pragma unroll
    for (uint32_t j = 0; j < 4u; ++j) {
      const uint32_t t = 4u * threadIdx.x + j;
      uint32_t bits = 0;
      if (t < nneed)
        for (uint32_t b = 0; b < 32u; ++b) {
          const uint32_t k = 32u * t + b;
          if (k >= n_act) break;
          const uint32_t e = P.act[k];
          if (((e >> 26) & 3u) == WC_NONE) continue;
          const uint32_t wi = w_beg + (e & ACT_OFF_MASK);
          const uint32_t live = range_mask(wi << 5, lo, hi);
          if (all || (hbr[wmod(P, wi)] & live) != live) bits |= 1u << b;
        }
      if (t < nneed) {
        P.rneed[(size_t)i * nneed + t] = bits;
        P.xsend[(size_t)i * nneed + t] = bits;
      }
      cnt[j] = (uint32_t)__popc(bits);
    }
    uint32_t total;
    scan4_256(cnt, pre, &total, s_lds4);
#pragma unroll
    for (uint32_t j = 0; j < 4u; ++j) {
      const uint32_t t = 4u * threadIdx.x + j;
      if (t < nneed) P.rpref[(size_t)i * nneed + t] = pre[j];
    }
    if (threadIdx.x == 0) P.rtot[i] = total;
  }
}

// (3a) sender shard: words each of its pairs must ship (the need bitmaps came back in send order)
__global__ void k_gossip_wcount(KP P, uint32_t n_pairs, uint32_t nneed) {
  SWIM_GUARD(P);
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < n_pairs) {
    uint32_t c = 0;
    for (uint32_t t = 0; t < nneed; ++t) c += (uint32_t)__popc(P.xrecv[(size_t)g * nneed + t]);
    P.wcnt[g] = c;
  }
}

// (3b) the needed window words of each pair, in need-bit order, at woff[g]
__global__ void __launch_bounds__(256) k_gossip_pack_sparse(KP P, uint32_t n_pairs, uint32_t nneed) {
  SWIM_GUARD(P);
  __shared__ uint32_t s_lds4[4];
  const uint32_t w_beg = P.ctl->w_beg, lo = P.ctl->scan_lo, hi = P.ctl->scan_hi;
  const uint32_t W32 = P.GC >> 5;
  for (uint32_t g = blockIdx.x; g < n_pairs; g += gridDim.x) {
    uint32_t dst, i;
    if (!xrec_locate(P, P.ctl->xg_cnt, g, &dst, &i)) break;
    const uint32_t ent = P.xg_pend[2 * ((size_t)dst * P.nloc * P.f + i)];
    const uint32_t m = (ent & SPAIR) ? P.sp_list[ent & ~SPAIR].x : ent;
    const uint32_t* pwr = (ent & SPAIR) ? P.pw + P.sp_list[ent & ~SPAIR].w : nullptr;  // pruned window
    const uint32_t* wbr = P.wb + lrow(P, m) * W32;
    const uint32_t* hbr = P.hb + lrow(P, m) * W32;
    uint32_t nv[4], cnt[4], pre[4];
#pragma unroll
    for (uint32_t j = 0; j < 4u; ++j) {
      const uint32_t t = 4u * threadIdx.x + j;
      nv[j] = t < nneed ? P.xrecv[(size_t)g * nneed + t] : 0u;
      cnt[j] = (uint32_t)__popc(nv[j]);
    }
    uint32_t total;
    scan4_256(cnt, pre, &total, s_lds4);
    uint32_t* out = P.xsend + P.woff[g];
#pragma unroll
    for (uint32_t j = 0; j < 4u; ++j) {
      uint32_t bits = nv[j], o = pre[j];
      while (bits) {  // the window as k_gossip_pull reads it
        const uint32_t b = (uint32_t)__builtin_ctz(bits);
        bits &= bits - 1u;
        const uint32_t k = 32u * (4u * threadIdx.x + j) + b;
        const uint32_t e = P.act[k];
        const uint32_t wc = (e >> 26) & 3u, wi = w_beg + (e & ACT_OFF_MASK);
        out[o++] = pwr ? pwr[k] : (wc == WC_ALL ? hbr[wmod(P, wi)] & range_mask(wi << 5, lo, hi) : wbr[k]);
      }
    }
  }
}

// received sparse windows join their receivers' sender lists
__global__ void k_gossip_unpack(KP P, uint32_t n_pairs) {
  SWIM_GUARD(P);
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < n_pairs) register_sender(P, P.rpairs[2 * g + 1], XREC | g);
}

// window word k of received pair i (0 where the receiver needed nothing: pull skips those)
__device__ __forceinline__ uint32_t remote_window(const KP& P, uint32_t i, uint32_t k) {
  const size_t nw = (size_t)i * P.nneed + (k >> 5);
  const uint32_t nb = P.rneed[nw], bit = 1u << (k & 31u);
  if (!(nb & bit)) return 0u;
  return P.xrecv[P.roff[i] + P.rpref[nw] + (uint32_t)__popc(nb & (bit - 1u))];
}

// SYNC request records [q, receiver, requester's table at phase start]
__global__ void __launch_bounds__(256) k_sync_pack(KP P, uint32_t n_rec) {
  SWIM_GUARD(P);
  for (uint32_t g = blockIdx.x; g < n_rec; g += gridDim.x) {
    uint32_t dst, i;
    if (!xrec_locate(P, P.ctl->xs_cnt, g, &dst, &i)) break;
    const uint32_t q = P.xs_pend[(size_t)dst * 2u * P.nloc + i];
    uint32_t* out = P.xsend + (size_t)g * sync_rec_words(P);  // a row of W cells (N x K: columns; tmode: touched)
    // a joiner's initial SYNC (JOIN_REQ | jsend index): [JOIN_REQ | joiner, seed, table]
    const uint2 js = (q & JOIN_REQ) ? P.jsend[q & ~JOIN_REQ] : make_uint2(q >> 1, 0u);
    if (threadIdx.x == 0) {
      out[0] = (q & JOIN_REQ) ? (JOIN_REQ | js.x) : q;
      out[1] = (q & JOIN_REQ) ? js.y : P.req_to[q];
    }
    const uint32_t* row = P.view + lrow(P, js.x) * P.W;
    if (tlisted(P))
      for (uint32_t c = threadIdx.x; c < P.ctl->ntouched; c += blockDim.x) out[2 + c] = row[P.tlist[c]];
    else
      for (uint32_t c = threadIdx.x; c < P.W; c += blockDim.x) out[2 + c] = row[c];
  }
}

// received SYNC requests join their receivers' buckets (k_scan / k_sync_scatter_remote)
__global__ void k_sync_unpack(KP P, uint32_t n_rec) {
  SWIM_GUARD(P);
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g == 0) P.ctl->xr_n = n_rec;
  if (g < n_rec) {
    const uint32_t* rec = P.xrecv + (size_t)g * sync_rec_words(P);
    if (!(rec[0] & JOIN_REQ)) P.rs_ref[rec[0]] = g;  // (a joiner's record is found by its seed's merge)
    recv_one(P, rec[1]);
  }
}

__global__ void k_sync_scatter_remote(KP P, uint32_t n_rec) {
  SWIM_GUARD(P);
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < n_rec) {
    const uint32_t* rec = P.xrecv + (size_t)g * sync_rec_words(P);
    const uint32_t to = rec[1];
    const uint32_t e = (rec[0] & JOIN_REQ) ? 4u * (rec[0] & ~JOIN_REQ) + 2u : 4u * (rec[0] >> 1) + (rec[0] & 1u);
    P.bucket[P.recv_off[to] + atomicAdd(&P.recv_fill[to], 1u)] = e;
  }
}

// requester side: where the SYNC_ACK of remote request q landed
__global__ void k_sync_ack_unpack(KP P, uint32_t n_rec) {
  SWIM_GUARD(P);
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < n_rec) {
    const uint32_t q = P.xrecv[(size_t)g * sync_rec_words(P)];
    if (q == NONE) return;  // a joiner's initial SYNC whose seed is not the one it takes the SYNC_ACK of
    if (q & JOIN_REQ)
      P.jack_ref[q & ~JOIN_REQ] = g;
    else
      P.ack_ref[q] = g;
  }
}

// The device half of a library-driven exchange's status row: the counts an exchange
// needs are in Ctl, so they go into the row the status all-gather carries instead of to the host first
// (one host stop per exchange, not two). row[XS_ERR]: an error this shard's state raises (every rank sees
// it and fails at the same exchange); row[XS_A0], row[XS_A1]: what the host needs afterwards;
// row[XS_CNT + q]: words to rank q (an all-gather: row[XS_CNT] alone).
enum XsKind : uint32_t { XS_NONE = 0, XS_COMMIT, XS_TRACK, XS_SEL, XS_WIN, XS_SYNC, XS_DONE };
constexpr uint32_t XS_ERR = 2, XS_A0 = 3, XS_A1 = 4, XS_CNT = 5;
struct XsArgs {
  uint32_t kind, world;
  uint32_t cap;      // COMMIT: stage capacity; TRACK: track capacity; WIN: send words; SYNC: sync_capacity
  uint32_t hdr;      // COMMIT: block header words (leaves)
  uint32_t nloc;     // COMMIT: stopped-member clamp (leaves), else 0
  uint32_t rl_dense; // SYNC: row cells without touched columns
  uint32_t tmode, N;
  uint64_t tail;     // COMMIT: words after the gossips and stopped members
  uint32_t bnd[SWIM_MAX_WORLD + 1];  // WIN: the out pairs' first index per peer shard
};
__global__ void k_xstatus(const Ctl* c, const uint32_t* woff, uint64_t* row, XsArgs a) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  uint64_t err = 0, a0 = 0, a1 = 0;
  for (uint32_t q = 0; q < a.world; ++q) row[XS_CNT + q] = 0;
  switch (a.kind) {
    case XS_COMMIT: {
      const uint32_t n = c->stg_count < a.cap ? c->stg_count : a.cap;  // beyond: OV_GOSSIP already raised
      const uint32_t ns = c->n_stop < a.nloc ? c->n_stop : a.nloc;
      err = c->overflow ? SWIM_EOVERFLOW : 0;
      a0 = n;
      a1 = ns;
      row[XS_CNT] = a.hdr + 4ull * n + ns + a.tail;
      break;
    }
    case XS_TRACK:
      row[XS_CNT] = c->ntrack < a.cap ? c->ntrack : a.cap;
      break;
    case XS_SEL:
      err = c->n_act > 32u * 1024u ? SWIM_EOVERFLOW : 0;
      a0 = c->n_act;
      for (uint32_t q = 0; q < a.world; ++q) {
        row[XS_CNT + q] = 2ull * c->xg_cnt[q];
        a1 += c->xg_cnt[q];
      }
      break;
    case XS_WIN: {
      const uint32_t n_out = a.bnd[a.world];
      err = woff[n_out] > a.cap ? SWIM_EOVERFLOW : 0;
      for (uint32_t q = 0; q < a.world; ++q) row[XS_CNT + q] = woff[a.bnd[q + 1]] - woff[a.bnd[q]];
      break;
    }
    case XS_SYNC: {
      const uint32_t rl = (a.tmode && c->ntouched < a.N) ? c->ntouched : a.rl_dense;
      for (uint32_t q = 0; q < a.world; ++q) {
        row[XS_CNT + q] = (uint64_t)c->xs_cnt[q] * (rl + 2u);
        a1 += c->xs_cnt[q];
      }
      err = a1 > a.cap ? SWIM_EOVERFLOW : 0;
      a0 = rl;
      a1 |= (uint64_t)a.cap << 32;  // (this rank's sync_capacity: every rank checks every rank's receipts)
      break;
    }
    case XS_DONE:
      err = c->overflow ? SWIM_EOVERFLOW : 0;
      break;
  }
  row[XS_ERR] = err;
  row[XS_A0] = a0;
  row[XS_A1] = a1;
}

// Every commit exchange also carries the shard's per-word gossip liveness (wlast) and its
// bit-length bounds after the words of its staged gossips: [gossips | wlast | bhi | 32 - blo]
__global__ void k_round_max_pack(KP P, uint32_t off) {
  const uint32_t W32 = P.GC >> 5;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < W32; i += gridDim.x * blockDim.x)
    P.xsend[off + i] = P.wlast[i];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    uint32_t blo = 32, bhi = 0;
    for (uint32_t b = 0; b < 32u; ++b)
      if (P.ctl->bl_hist[b]) {
        blo = b < blo ? b : blo;
        bhi = b;
      }
    P.xsend[off + W32] = bhi;
    P.xsend[off + W32 + 1] = 32u - blo;  // 0 when this shard has no alive member
  }
  if (P.tmode)  // the touched columns after the bounds (OR-merged)
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (P.N >> 5); i += gridDim.x * blockDim.x)
      P.xsend[off + W32 + 2u + i] = P.tbits[i];
}

// element-wise max over the shards' blocks (offsets in `offs`) into wlast and blx
__global__ void k_round_max_merge(KP P, const uint32_t* offs, uint32_t* blx) {
  const uint32_t W32 = P.GC >> 5;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < W32 + 2u; i += gridDim.x * blockDim.x) {
    uint32_t v = 0;
    for (uint32_t q = 0; q < P.world; ++q) {
      const uint32_t x = P.xrecv[offs[q] + i];
      v = x > v ? x : v;
    }
    if (i < W32)
      P.wlast[i] = v;
    else
      blx[i - W32] = v;
  }
  if (P.tmode)
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (P.N >> 5); i += gridDim.x * blockDim.x) {
      uint32_t v = 0;
      for (uint32_t q = 0; q < P.world; ++q) v |= P.xrecv[offs[q] + W32 + 2u + i];
      P.tbits[i] = v;
    }
}

// ---------------------------------------------------------------------------------------
// Suspicion timeouts: stream due subject columns of the deadline matrix.
// ---------------------------------------------------------------------------------------
// The due cells (dense: subjects; N x K: columns) in ascending order: one workgroup, an ordered
// compaction in which each thread takes 64 consecutive cells (16-B loads of the column minima, a
// 64-bit mask of its due cells) and one block scan places them, so the sweep's chunks of SW_COLS due
// cells are neighbours in every view row and their cells share lines. (65,536 cells per pass.)
__global__ void __launch_bounds__(1024) k_due(KP P) {
  SWIM_GUARD(P);
  __shared__ uint32_t s_lds[16];
  const uint32_t nc = ncells(P);
  if (threadIdx.x == 0) {  // this period's SYNC counters (k_sync_select on), in place of host memsets
    P.ctl->stage_count = 0u;
    P.ctl->js_n = 0u;
  }
  if (threadIdx.x < SWIM_MAX_WORLD) P.ctl->xs_cnt[threadIdx.x] = 0u;
  if (threadIdx.x < SY_STRIPES) {
    P.ctl->sy_mcnt[threadIdx.x] = 0u;
    P.ctl->sy_acnt[threadIdx.x] = 0u;
  }
  uint32_t base = 0;
  for (uint32_t j0 = 0; j0 < nc; j0 += 65536u) {
    const uint32_t c0 = j0 + 64u * threadIdx.x;
    unsigned long long m = 0ull;
    if (c0 + 64u <= nc) {
      const uint4* cp = reinterpret_cast<const uint4*>(P.colmin + c0);
#pragma unroll
      for (uint32_t q = 0; q < 16u; ++q) {
        const uint4 v = cp[q];
        m |= (unsigned long long)((v.x <= P.period ? 1u : 0u) | (v.y <= P.period ? 2u : 0u) |
                                  (v.z <= P.period ? 4u : 0u) | (v.w <= P.period ? 8u : 0u)) << (4u * q);
      }
    } else {
      for (uint32_t k = 0; c0 + k < nc && k < 64u; ++k)
        if (P.colmin[c0 + k] <= P.period) m |= 1ull << k;
    }
    uint32_t tot;
    uint32_t o = base + block_excl_scan1024((uint32_t)__popcll(m), &tot, s_lds);
    while (m) {
      const uint32_t j = c0 + (uint32_t)__builtin_ctzll(m);
      m &= m - 1ull;
      P.due[o++] = j;
      P.colmin[j] = NONE;  // rebuilt by the sweep from the deadlines it leaves standing
    }
    base += tot;
  }
  if (threadIdx.x == 0) P.ctl->due_count = base;
}

// onSuspicionTimeout (MembershipProtocolImpl.java:637-647) over the due deadline columns. A
// workgroup takes a tile of 256 consecutive observers x SW_COLS consecutive due cells, in two passes:
//   1. column-major, over the subject-major deadlines: thread t reads observer t's deadline of each
//      column (a column's 256 deadlines are one coalesced 1-KiB read), clears the fired and the
//      stopped ones, keeps the fired columns as a 64-bit mask per observer (LDS), and reduces the
//      standing minimum and the removals per column (per wave, then LDS);
//   2. row-major, over the observer-major view: wave w takes rows w, w + 4, ...; lane q clears the
//      row's cell of due column q when it fired. The due cells ascend (k_due), so the lanes of one
//      store hit neighbouring cells of one row: lines are written once for all the cells they hold,
//      not once per cell (the previous sweep: one 128-B line per 4-B cell).
// Removals are counted per observer (one cnt_delta update) and per column (one presence /
// last-removal / column-minimum update per workgroup and column). MembershipEvents (REMOVED with
// the removed record) are allocated per workgroup and tile: a block scan of the rows' fired counts
// and one atomic on the ring's counter (an atomic per wave and row serialised ~10^6 times per launch
// on that one word: 4.7 ms per C3 firing launch instead of ~0.5).
constexpr uint32_t SW_COLS = 64;
__global__ void __launch_bounds__(256) k_susp_sweep(KP P) {
  SWIM_GUARD(P);
  __shared__ uint32_t s_col[SW_COLS], s_rem[SW_COLS], s_min[SW_COLS];
  __shared__ unsigned long long s_fire[256];
  __shared__ uint32_t s_eoff[256], s_scan[4], s_ebase;
  Tally T;
  uint32_t fired = 0;
  const uint32_t n = P.ctl->due_count, tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  const uint32_t nob = (P.nloc + 255u) / 256u, ncb = (n + SW_COLS - 1u) / SW_COLS;
  // the SYNC phase's per-receiver request counts start from zero (in place of two host memsets)
  for (uint32_t i = blockIdx.x * 256u + tid; i < P.N; i += gridDim.x * 256u) {
    P.recv_count[i] = 0u;
    P.recv_fill[i] = 0u;
  }
  for (uint32_t u = blockIdx.x; u < nob * ncb; u += gridDim.x) {
    const uint32_t ob = u % nob, c0 = (u / nob) * SW_COLS;  // neighbouring workgroups: neighbouring observers
    const uint32_t nc = min(SW_COLS, n - c0);
    if (tid < nc) {
      s_col[tid] = P.due[c0 + tid];
      s_rem[tid] = 0u;
      s_min[tid] = NONE;
    }
    __syncthreads();
    const uint32_t li = ob * 256u + tid;
    {  // pass 1 (every lane of the workgroup runs the loop: the per-wave reductions see whole waves)
      const bool valid = li < P.nloc;
      const uint32_t i = P.row0 + (valid ? li : 0u);
      const bool alive = valid && P.alive[i] != 0;
      unsigned long long fm = 0ull;  // fired columns of this observer (ordinary cells: pass 2 clears them)
      for (uint32_t k0 = 0; k0 < nc; k0 += 4u) {
        uint32_t v[4], smin[4] = {NONE, NONE, NONE, NONE};
#pragma unroll
        for (uint32_t q = 0; q < 4u; ++q)  // four columns' deadlines in flight
          v[q] = (valid && k0 + q < nc) ? P.dl[(size_t)s_col[k0 + q] * P.nloc + li] : 0u;
#pragma unroll
        for (uint32_t q = 0; q < 4u; ++q) {
          if (!v[q]) continue;
          const uint32_t k = k0 + q, j = s_col[k];
          uint16_t* dp = P.dl + (size_t)j * P.nloc + li;
          if (!alive) {  // a stopped member's timers never fire: dropped
            *dp = 0u;
            continue;
          }
          const uint32_t dl = dl_dec(v[q], P.period);
          if ((int32_t)(dl - P.period) > 0) {  // still standing: the column's minimum (reduced per wave below)
            smin[q] = dl;
            continue;
          }
          *dp = 0u;
          ++fired;
          const uint32_t subj = subj_of(P, j);
          if (subj == i || (P.rerouted && P.addr[subj] == P.addr[i])) {  // (never in practice)
            apply_record(P, i, subj, SWIM_DEAD, SWIM_R_SUSPICION_TIMEOUT, 0u, P.cnt[i], T);
            continue;
          }
          // updateMembership(DEAD) -> onDeadMemberDetected (MPI:571-587) as in apply_record, with
          // the counts applied once per observer and once per column. A deadline implies a record:
          // every path that clears a cell clears its deadline too (DEAD accepted, crash, join, leave
          // stop), so the cell is present and pass 2 removes it.
          fm |= 1ull << k;
          T.accepted++;
          T.removed++;
        }
        // per column: the wave's removals (one LDS add) and standing minimum (one LDS min)
#pragma unroll
        for (uint32_t q = 0; q < 4u; ++q) {
          const uint32_t k = k0 + q;
          if (k >= nc) continue;  // (uniform)
          const uint32_t nrem = (uint32_t)__popcll(__ballot((fm >> k) & 1ull));
          uint32_t mn = smin[q];
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) mn = min(mn, (uint32_t)__shfl_xor(mn, o, 64));
          if (lane == 0) {
            if (nrem) atomicAdd(&s_rem[k], nrem);
            if (mn != NONE) atomicMin(&s_min[k], mn);
          }
        }
      }
      if (fm) atomicSub(&P.cnt_delta[i], (int32_t)__popcll(fm));
      s_fire[tid] = fm;
      if (P.ecap) {  // the tile's events: row offsets by a block scan, one ring allocation
        uint32_t tot;
        s_eoff[tid] = block_excl_scan1024((uint32_t)__popcll(fm), &tot, s_scan);
        if (tid == 0) s_ebase = tot ? atomicAdd(&P.ctl->event_count, tot) : 0u;
      }
    }
    __syncthreads();
    // pass 2: the fired cells, row by row, lane q on due column q
    const uint32_t jq = lane < nc ? s_col[lane] : 0u;
    const uint32_t sq = lane < nc ? subj_of(P, jq) : 0u;
    const uint32_t bq = (lane < nc && P.dmark) ? P.sid_of[sq] : NONE;  // merge marks (mark_clear)
    for (uint32_t t = wv; t < 256u; t += 4u) {
      const unsigned long long fm = s_fire[t];  // (the same word for every lane: a broadcast)
      if (!fm) continue;  // (uniform)
      const uint32_t lr = ob * 256u + t;
      const bool f = (fm >> lane) & 1ull;
      uint32_t* cellp = P.view + (size_t)lr * P.W + jq;
      uint32_t r0 = 0u;
      if (f && P.ecap) {
        r0 = *cellp;  // the removed record, for the REMOVED event
        if (r0 == SWIM_ABSENT) atomicOr(&P.ctl->overflow, OV_BUG);  // a deadline without a record
      }
      if (f) *cellp = SWIM_ABSENT;
      if (f && bq < P.dsids) P.dmark[(size_t)lr * P.dsids + bq] = 0u;
      if (P.ecap) {
        const uint32_t at = s_ebase + s_eoff[t] + (uint32_t)__popcll(fm & ((1ull << lane) - 1ull));
        if (f) {
          if (at >= P.ecap) {
            atomicOr(&P.ctl->overflow, OV_EVENTS);
          } else {
            swim_event e;
            e.period = P.period;
            e.observer = P.row0 + lr;
            e.subject = sq;
            e.record = r0;
            e.type = (uint8_t)SWIM_EV_REMOVED;
            e.reason = (uint8_t)SWIM_R_SUSPICION_TIMEOUT;
            e.phase = (uint8_t)P.phase;
            e.pad = 0;
            P.events[at] = e;
          }
        }
      }
    }
    __syncthreads();
    if (tid < nc) {
      const uint32_t j = s_col[tid];
      if (s_min[tid] != NONE) atomicMin(&P.colmin[j], s_min[tid]);
      if (s_rem[tid]) {  // the column's removals: presence and last-removal period
        const uint32_t subj = subj_of(P, j);
        atomicSub(&P.pres[subj], s_rem[tid]);
        atomicMax(&P.last_removed[subj], P.period + 1u);
      }
    }
    __syncthreads();
  }
  add_stat(P, ST_SUSP_TIMEOUTS, fired);
  if (blockIdx.x == 0 && tid == 0 && n)  // deadline cells scanned (may exceed 32 bits: no wave sum)
    atomicAdd(&P.stat_shards[ST_SWEEP_CELLS], (unsigned long long)n * P.nloc);
  flush_tally(P, T);
}

// ---------------------------------------------------------------------------------------
// SYNC / SYNC_ACK.
// ---------------------------------------------------------------------------------------
// selectSyncAddress (MembershipProtocolImpl.java:416-427): uniform over the set of addresses
// seeds U otherMembers' addresses, by rejection sampling over address ids (address x = member x's;
// seed addresses are members [0, n_seeds)'s; the own address is never a seed, MPI:166-172).
__device__ __forceinline__ bool sync_addr_valid(const KP& P, uint32_t i, uint32_t own, uint32_t x) {
  if (!P.rerouted) return x != i && (cell_get(P, i, x) != 0u || x < P.n_seeds);
  if (x == own || P.addr[x] != x) return false;  // own address / an id that moved to another address
  if (x < P.n_seeds || cell_get(P, i, x) != 0u) return true;
  for (uint32_t y = P.mv_head[x]; y != NONE; y = P.mv_next[y])  // members restarted on address x
    if (y != i && cell_get(P, i, y) != 0u) return true;
  return false;
}

__device__ uint32_t select_sync_address(const KP& P, uint32_t i) {
  const uint32_t N = P.N;
  const uint32_t own = addr_of(P, i), nseeds = P.n_seeds < N ? P.n_seeds : N;
  // MPI:421-422: nothing to pick when no other member is known and no seed address is not our own
  if (P.cnt[i] == 0u && (nseeds == 0u || (nseeds == 1u && own == 0u))) return NONE;
  uint32_t x = 0;
  for (uint32_t a = 0; a < 64u; ++a) {
    x = (uint32_t)(((uint64_t)draw1(P.seed, K_SYNC_PICK, i, a, 0, P.tick) * N) >> 32);
    if (sync_addr_valid(P, i, own, x)) return x;
  }
  for (uint32_t d = 1; d <= N; ++d) {
    const uint32_t y = (uint32_t)(((uint64_t)x + d) % N);
    if (sync_addr_valid(P, i, own, y)) return y;
  }
  return NONE;
}

__global__ void k_sync_select(KP P) {
  SWIM_GUARD(P);
  const uint32_t i = P.row0 + blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t sent = 0, dlv = 0;
  bool req = false;  // a staged (or remote) request: k_sync_ack's work
  if (i < P.row0 + P.nloc) {
    P.req_to[2 * i] = NONE;
    P.req_to[2 * i + 1] = NONE;
    P.req_stage[2 * i] = NONE;
    P.req_stage[2 * i + 1] = NONE;
    const uint32_t fdt = P.sync_fd[i];
    P.sync_fd[i] = NONE;
    if (P.alive[i]) {
      uint32_t to[2];
      // doSync (:304-320); a member joining this period makes its initial SYNCs instead (k_join_select)
      const bool joins = P.njoin && P.joining[i];
      to[0] = (!joins && P.period % P.S == i % P.S) ? select_sync_address(P, i) : NONE;
      to[1] = fdt;                                                              // MPI:389-397
      for (uint32_t k = 0; k < 2; ++k) {
        if (to[k] == NONE) continue;
        ++sent;
        P.req_to[2 * i + k] = to[k];
        if (!delivered(P, K_SYNC, i, to[k], k, P.tick)) continue;
        ++dlv;
        if (P.rerouted) to[k] = route(P, to[k]);  // the process at the address receives it
        P.req_to[2 * i + k] = to[k];
        if (!is_local(P, to[k])) {  // the table travels to the receiver's shard (k_sync_pack)
          const uint32_t dst = to[k] / P.nloc;
          const uint32_t o = atomicAdd(&P.ctl->xs_cnt[dst], 1u);
          P.xs_pend[(size_t)dst * 2u * P.nloc + o] = 2 * i + k;
          P.req_stage[2 * i + k] = REMOTE;
          req = true;
          continue;
        }
        const uint32_t slot = atomicAdd(&P.ctl->stage_count, 1u);
        if (slot >= P.scap) {
          atomicOr(&P.ctl->overflow, OV_SYNC);
          continue;
        }
        P.req_stage[2 * i + k] = slot;
        P.stage_req[slot] = 2 * i + k;
        req = true;
        recv_one(P, to[k]);
      }
    }
  }
  if (req) sy_push(P.ctl->sy_acnt, P.sy_alist, P.sy_cap, i - P.row0, i);
  add_stat(P, ST_SYNCS_SENT, sent);
  add_stat(P, ST_SYNCS_DELIVERED, dlv);
}

// start0 (MembershipProtocolImpl.java:222-257) of the members joining this period: one SYNC to every
// seed address but the own one, all carrying the joiner's table (one staging slot); the joiner will
// merge only the first SYNC_ACK to come back (take(1), :244-247), canonically the lowest seed address
// whose round trip is delivered (jwin). Thread per member; launched only when some member joins.
// Sharded handles: every shard works out every joiner's jwin (the seeds' shards need it: only jwin's merge
// keeps a SYNC_ACK); the joiner's own shard stages its table for the seeds on that shard and sends it
// to each seed on another shard in the SYNC exchange (jsend, k_sync_pack), whose SYNC_ACK comes back
// in the same record.
__global__ void k_join_select(KP P) {
  SWIM_GUARD(P);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t sent = 0, dlv = 0;
  if (i < P.N && P.joining[i] && P.alive[i]) {
    const bool mine = is_local(P, i);
    P.jwin[i] = NONE;
    P.jslot[i] = NONE;
    const uint32_t nseeds = P.n_seeds < P.N ? P.n_seeds : P.N, own = addr_of(P, i);
    uint32_t slot = NONE;
    for (uint32_t s = 0; s < nseeds; ++s) {
      if (s == own) continue;
      sent += mine ? 1u : 0u;
      if (!delivered(P, K_SYNC, i, s, 2u, P.tick)) continue;
      dlv += mine ? 1u : 0u;
      const uint32_t rcv = route(P, s);
      if (P.jwin[i] == NONE && delivered(P, K_SYNC_ACK, rcv, i, 2u, P.tick + 1u)) P.jwin[i] = rcv;
      if (!mine) continue;
      if (!is_local(P, rcv)) {  // the table travels to the seed's shard
        const uint32_t dst = rcv / P.nloc;
        const uint32_t js = atomicAdd(&P.ctl->js_n, 1u);
        const uint32_t o = atomicAdd(&P.ctl->xs_cnt[dst], 1u);
        if (js >= P.N || o >= 2u * P.nloc) {
          atomicOr(&P.ctl->overflow, OV_SYNC);
          break;
        }
        P.jsend[js] = make_uint2(i, rcv);
        P.xs_pend[(size_t)dst * 2u * P.nloc + o] = JOIN_REQ | js;
        continue;
      }
      if (slot == NONE) {
        slot = atomicAdd(&P.ctl->stage_count, 1u);
        if (slot >= P.scap) {
          atomicOr(&P.ctl->overflow, OV_SYNC);
          break;
        }
        P.stage_req[slot] = 2 * i;
        P.jslot[i] = slot;
      }
      recv_one(P, rcv);
    }
  }
  // a joiner whose initial SYNC_ACK comes back is k_sync_ack's work too (k_sync_ack's own test; once:
  // not when k_sync_select listed it for a request of its own)
  if (i >= P.row0 && i < P.row0 + P.nloc && P.joining[i] && P.jwin[i] != NONE &&
      (P.jslot[i] < P.scap || !is_local(P, P.jwin[i])) && P.req_stage[2 * i] == NONE && P.req_stage[2 * i + 1] == NONE)
    sy_push(P.ctl->sy_acnt, P.sy_alist, P.sy_cap, i - P.row0, i);
  add_stat(P, ST_SYNCS_SENT, sent);
  add_stat(P, ST_SYNCS_DELIVERED, dlv);
}

// bucket entries are 4 * sender + kind (kind 2 = initial SYNC), so a receiver's requests sort in
// (sender, kind) order
__global__ void k_join_scatter(KP P) {
  SWIM_GUARD(P);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < P.N && P.joining[i] && P.alive[i] && is_local(P, i) && P.jslot[i] != NONE && P.jslot[i] < P.scap) {
    const uint32_t nseeds = P.n_seeds < P.N ? P.n_seeds : P.N, own = addr_of(P, i);
    for (uint32_t s = 0; s < nseeds; ++s) {
      if (s == own || !delivered(P, K_SYNC, i, s, 2u, P.tick)) continue;
      const uint32_t rcv = route(P, s);
      if (!is_local(P, rcv)) continue;  // (k_sync_scatter_remote on the seed's shard)
      P.bucket[P.recv_off[rcv] + atomicAdd(&P.recv_fill[rcv], 1u)] = 4u * i + 2u;
    }
  }
}

// prepareSyncDataMsg (MembershipProtocolImpl.java:457-461): payload = sender's table at phase start.
// Dense views in tmode: the touched columns in ascending order (tlist, ntouched) for this period's
// SYNC payloads. One workgroup, an ordered compaction: thread t takes 64 consecutive columns (two
// bitmap words), one block scan places them.
__global__ void __launch_bounds__(1024) k_tlist(KP P) {
  SWIM_GUARD(P);
  __shared__ uint32_t s_lds[16];
  uint32_t base = 0;
  for (uint32_t c0 = 0; c0 < P.N; c0 += 65536u) {
    const uint32_t w = (c0 >> 5) + 2u * threadIdx.x;
    const uint32_t nw = P.N >> 5;  // (N is a multiple of 32 in tmode: swim_create)
    unsigned long long m = 0ull;
    if (w < nw) m = P.tbits[w];
    if (w + 1u < nw) m |= (unsigned long long)P.tbits[w + 1u] << 32;
    uint32_t tot;
    uint32_t o = base + block_excl_scan1024((uint32_t)__popcll(m), &tot, s_lds);
    while (m) {
      P.tlist[o++] = 32u * w + (uint32_t)__builtin_ctzll(m);
      m &= m - 1ull;
    }
    base += tot;
  }
  // beyond a quarter of the columns a gather reads nearly every line of a row anyway: whole rows
  // (16-B streams) this period, ntouched = N
  if (threadIdx.x == 0) P.ctl->ntouched = 4u * base > P.N ? P.N : base;
}


__global__ void __launch_bounds__(256) k_sync_snapshot(KP P) {
  SWIM_GUARD(P);
  uint32_t n = P.ctl->stage_count;
  if (n > P.scap) n = P.scap;
  if (tlisted(P)) {  // the touched columns only: a gather from the sender's row
    const uint32_t T = P.ctl->ntouched;
    for (uint32_t k = blockIdx.x; k < n; k += gridDim.x) {
      const uint32_t* row = P.view + lrow(P, P.stage_req[k] >> 1) * P.W;
      uint32_t* dst = P.stage_sync + (size_t)k * P.W;
      for (uint32_t c = threadIdx.x; c < T; c += blockDim.x) dst[c] = row[P.tlist[c]];
    }
    return;
  }
  const uint32_t W = ncells(P), nv = (P.W & 3u) ? 0u : W / 4u;  // a row = the first ncells cells
  for (uint32_t k = blockIdx.x; k < n; k += gridDim.x) {
    const uint32_t from = P.stage_req[k] >> 1;
    const uint4* src = reinterpret_cast<const uint4*>(P.view + lrow(P, from) * P.W);
    uint4* dst = reinterpret_cast<uint4*>(P.stage_sync + (size_t)k * P.W);
    for (uint32_t c = threadIdx.x; c < nv; c += blockDim.x) dst[c] = src[c];
    for (uint32_t c = nv * 4u + threadIdx.x; c < W; c += blockDim.x)
      P.stage_sync[(size_t)k * P.W + c] = P.view[lrow(P, from) * P.W + c];
  }
}

// exclusive scan of recv_count -> recv_off over the chip: per-tile sums (SCAN_TILE counts per
// workgroup), their scan (k_excl_scan, one workgroup over the tiles), then each tile's own scan
// from its base. (A single 1,024-thread workgroup walking all N counts took 1.8 ms per period at
// N = 2^20.)
constexpr uint32_t SCAN_TILE = 4096;
__global__ void __launch_bounds__(1024) k_scan_tiles(KP P, uint32_t* tsum) {
  SWIM_GUARD(P);
  __shared__ uint32_t s_lds[16];
  const uint32_t b = blockIdx.x * SCAN_TILE + 4u * threadIdx.x;
  uint32_t sum = 0;
  if (b + 3u < P.N) {
    const uint4 v = *reinterpret_cast<const uint4*>(P.recv_count + b);
    sum = v.x + v.y + v.z + v.w;
  } else {
    for (uint32_t k = 0; k < 4u; ++k)
      if (b + k < P.N) sum += P.recv_count[b + k];
  }
  uint32_t tot;
  block_excl_scan1024(sum, &tot, s_lds);
  if (threadIdx.x == 0) tsum[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(1024) k_scan_apply(KP P, const uint32_t* tbase, uint32_t ntiles) {
  SWIM_GUARD(P);
  __shared__ uint32_t s_lds[16];
  const uint32_t b = blockIdx.x * SCAN_TILE + 4u * threadIdx.x;
  uint32_t v[4];
  for (uint32_t k = 0; k < 4u; ++k) v[k] = b + k < P.N ? P.recv_count[b + k] : 0u;
  uint32_t tot;
  uint32_t run = tbase[blockIdx.x] + block_excl_scan1024(v[0] + v[1] + v[2] + v[3], &tot, s_lds);
  for (uint32_t k = 0; k < 4u; ++k)
    if (b + k < P.N) {
      P.recv_off[b + k] = run;
      run += v[k];
    }
  if (blockIdx.x == ntiles - 1u && threadIdx.x == 0) P.recv_off[P.N] = tbase[blockIdx.x] + tot;
}

__global__ void k_sync_scatter(KP P) {
  SWIM_GUARD(P);
  const uint32_t q = 2u * P.row0 + blockIdx.x * blockDim.x + threadIdx.x;
  if (q < 2u * (P.row0 + P.nloc) && P.req_stage[q] != NONE && P.req_stage[q] != REMOTE) {
    const uint32_t to = P.req_to[q];
    const uint32_t pos = P.recv_off[to] + atomicAdd(&P.recv_fill[to], 1u);
    P.bucket[pos] = 4u * (q >> 1) + (q & 1u);
  }
}

__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t* total, uint32_t* lds4) {
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  uint32_t wt;
  const uint32_t x = wave_excl_scan(v, &wt) + v;  // the wave's inclusive scan (DPP)
  if (lane == 63u) lds4[w] = x;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (uint32_t k = 0; k < 4u; ++k) {
    const uint32_t t = lds4[k];
    if (k < w) base += t;
    tot += t;
  }
  __syncthreads();
  *total = tot;
  return base + x - v;
}

// Merge one table into row `obs` (syncMembership, MembershipProtocolImpl.java:463-473),
// cells in parallel, gossip sequence numbers assigned in cell order by a block scan.
// `ack_out` (may be null) receives the row after the merge (onSync's SYNC_ACK payload).
__device__ __forceinline__ void merge_row(const KP& P, uint32_t obs, const uint32_t* src, uint32_t* ack_out,
                                          uint32_t attempt, uint32_t reason, uint32_t snap, uint32_t& seq, Tally& T,
                                          uint32_t& created, uint32_t* lds4) {
  uint32_t* row = P.view + lrow(P, obs) * P.W;
  // Dense rows: cell = subject, 4 cells per thread (16-B loads) when rows are 16-B aligned.
  // N x K rows: one column per thread, walked in subject order (colorder) so gossip sequence
  // numbers come out exactly as in the dense table; untracked subjects hold BASELINE on both
  // sides, and equal records never override (MembershipProtocolImpl.java:489).
  // Cells the incoming record does not override (the common case) never enter updateMembership.
  const uint32_t nc = sync_cells(P);
  const bool listed = tlisted(P);
  const uint32_t per = (!P.nxk && !listed && (P.W & 3u) == 0u) ? 4u : 1u;
  __shared__ uint32_t s_chk[32];  // 1,024-cell chunks with an overridden cell (rows of <= 2^20 cells)
  if (per == 4u) {
    // Most merges change nothing (a converged or converging cluster): first a barrier-free stream
    // over both rows, four 16-B steps per thread in flight, writing the SYNC_ACK payload as if no
    // cell were overridden; only the 1,024-cell chunks with an overriding cell take the ordered pass
    // below (which rewrites their payload).
    __syncthreads();  // every thread is past the previous merge's reads of s_chk
    if (threadIdx.x < 32u) s_chk[threadIdx.x] = 0u;
    __syncthreads();
    bool any = false;
    for (uint32_t c0 = 0; c0 < nc; c0 += 4096u) {
      uint4 s4[4], v4[4];
#pragma unroll
      for (uint32_t u = 0; u < 4u; ++u) {
        const uint32_t c = c0 + 1024u * u + 4u * threadIdx.x;
        s4[u] = c < nc ? *reinterpret_cast<const uint4*>(src + c) : make_uint4(0u, 0u, 0u, 0u);
        v4[u] = c < nc ? *reinterpret_cast<const uint4*>(row + c) : make_uint4(0u, 0u, 0u, 0u);
      }
#pragma unroll
      for (uint32_t u = 0; u < 4u; ++u) {
        const uint32_t c = c0 + 1024u * u + 4u * threadIdx.x;
        const bool ov = (s4[u].x && is_overrides(s4[u].x, v4[u].x)) || (s4[u].y && is_overrides(s4[u].y, v4[u].y)) ||
                        (s4[u].z && is_overrides(s4[u].z, v4[u].z)) || (s4[u].w && is_overrides(s4[u].w, v4[u].w));
        if (ov) {
          const uint32_t ch = c >> 10;
          atomicOr(&s_chk[ch >> 5], 1u << (ch & 31u));
        }
        any |= ov;
        if (ack_out && c < nc) *reinterpret_cast<uint4*>(ack_out + c) = v4[u];
      }
    }
    if (!__syncthreads_or(any)) return;
  }
  for (uint32_t c0 = 0; c0 < nc; c0 += 256u * per) {
    if (per == 4u && !((s_chk[c0 >> 15] >> ((c0 >> 10) & 31u)) & 1u)) continue;  // (uniform)
    const uint32_t c = c0 + per * threadIdx.x;
    uint32_t recs[4], cells[4], nrec = 0;
    if (c < nc) {
      uint32_t sv[4], vv[4], cv[4];
      if (per == 4u) {
        const uint4 s4 = *reinterpret_cast<const uint4*>(src + c);
        const uint4 v4 = *reinterpret_cast<const uint4*>(row + c);
        sv[0] = s4.x, sv[1] = s4.y, sv[2] = s4.z, sv[3] = s4.w;
        vv[0] = v4.x, vv[1] = v4.y, vv[2] = v4.z, vv[3] = v4.w;
        cv[0] = c, cv[1] = c + 1u, cv[2] = c + 2u, cv[3] = c + 3u;
      } else if (listed) {  // the touched columns: payload position c holds column tlist[c]
        cv[0] = P.tlist[c];
        sv[0] = src[c];
        vv[0] = row[cv[0]];
      } else {
        cv[0] = P.nxk ? P.colorder[c] : c;
        sv[0] = src[cv[0]];
        vv[0] = row[cv[0]];
      }
      for (uint32_t k = 0; k < per; ++k) {
        if (sv[k] == 0u || !is_overrides(sv[k], vv[k])) continue;
        const uint32_t subj = subj_of(P, cv[k]);
        const uint32_t rec = apply_record(P, obs, subj, sv[k], reason, attempt, snap, T);
        vv[k] = row[cv[k]];
        if (rec) {
          recs[nrec] = rec;
          cells[nrec] = subj;
          ++nrec;
        }
      }
      if (ack_out) {
        if (per == 4u)
          *reinterpret_cast<uint4*>(ack_out + c) = make_uint4(vv[0], vv[1], vv[2], vv[3]);
        else
          ack_out[listed ? c : cv[0]] = vv[0];
      }
    }
    if (__syncthreads_or(nrec != 0u)) {  // gossip sequence numbers in subject order
      uint32_t total;
      const uint32_t off = block_excl_scan256(nrec, &total, lds4);
      for (uint32_t k = 0; k < nrec; ++k) emit_gossip(P, obs, cells[k], recs[k], seq + off + k);
      created += nrec;
      seq += total;
    }
  }
}

// onSync (MembershipProtocolImpl.java:352-373) at receiver j = blockIdx, requests in
// (sender, kind) order; each SYNC_ACK payload is j's table right after that request's merge.
// SYNC merges at 6 waves per SIMD (80 VGPRs, 28–44 B of scratch) instead of their natural 5: the
// fault-free steady state's merge / ack 23.9 / 17.7 -> 23.4 / 16.9 ms per 60 periods
#define SWIM_SYNC_WAVES 6
// A workgroup per listed member, over a grid of at most SY_GRID workgroups: a period's ~N/S
// receivers (requesters), not a workgroup per member (65,536 launched workgroups took 29 us of the
// fault-free period when ~1,800 had requests; a workgroup per 32 members serialised C3's heal merges).
// The lists are striped (sy_push): the u-th entry is in the last stripe whose count prefix is <= u.
constexpr uint32_t SY_GRID = 2048;
template <typename F>
__device__ __forceinline__ void sy_for_each(const uint32_t* cnt, const uint32_t* list, uint32_t cap, uint32_t* s_pre, F f) {
  if (threadIdx.x < 64u) {  // (wave 0, every lane: SY_STRIPES = 64)
    const uint32_t v = cnt[threadIdx.x];
    uint32_t tot;
    s_pre[threadIdx.x] = wave_excl_scan(v, &tot);
    if (threadIdx.x == 0) s_pre[64] = tot;
  }
  __syncthreads();
  const uint32_t tot = s_pre[64];
  for (uint32_t u = blockIdx.x; u < tot; u += gridDim.x) {
    uint32_t st = 0;
    for (uint32_t step = 32u; step; step >>= 1)
      if (st + step < SY_STRIPES && s_pre[st + step] <= u) st += step;
    f(list[(size_t)st * cap + (u - s_pre[st])]);
    __syncthreads();
  }
}
static_assert(SY_STRIPES == 64, "sy_for_each scans the stripe counts in one wave");
__device__ __forceinline__ void sync_merge_one(const KP& P, uint32_t j, uint32_t* s_list, uint32_t* s_lds4) {
  uint32_t cntj = P.recv_count[j];
  if (cntj == 0u) return;
  if (cntj > (uint32_t)BUCKET_MAX) {
    if (threadIdx.x == 0) atomicOr(&P.ctl->overflow, OV_BUCKET);
    cntj = BUCKET_MAX;
  }
  const uint32_t off = P.recv_off[j];
  for (uint32_t k = threadIdx.x; k < cntj; k += blockDim.x) s_list[k] = P.bucket[off + k];
  __syncthreads();
  if (threadIdx.x == 0) {  // insertion sort: bucket entry 4 * sender + kind
    for (uint32_t a = 1; a < cntj; ++a) {
      const uint32_t v = s_list[a];
      uint32_t b = a;
      while (b > 0 && s_list[b - 1] > v) {
        s_list[b] = s_list[b - 1];
        --b;
      }
      s_list[b] = v;
    }
  }
  __syncthreads();
  Tally T;
  uint32_t created = 0;
  uint32_t seq = P.gseq[j];
  const uint32_t snap = P.cnt[j];
  for (uint32_t k = 0; k < cntj; ++k) {
    const uint32_t b = s_list[k], from = b >> 2, kind = b & 3u;
    const uint32_t q = 2u * from + (kind & 1u);  // request index of a periodic / FD-triggered SYNC
    const uint32_t* src;
    uint32_t* ack;
    if (kind == 2u) {  // a joiner's initial SYNC; only the seed it will take the SYNC_ACK of keeps one
      if (is_local(P, from)) {
        const uint32_t slot = P.jslot[from];
        src = P.stage_sync + (size_t)slot * P.W;
        ack = P.jwin[from] == j ? P.stage_ack + (size_t)slot * P.W : nullptr;
      } else {  // from another shard: its record [JOIN_REQ | from, j, table] among this period's received ones
        __shared__ uint32_t s_jg;
        const size_t rw = sync_rec_words(P);
        if (threadIdx.x == 0) s_jg = NONE;
        __syncthreads();
        for (uint32_t g = threadIdx.x; g < P.ctl->xr_n; g += blockDim.x)
          if (P.xrecv[(size_t)g * rw] == (JOIN_REQ | from) && P.xrecv[(size_t)g * rw + 1] == j) s_jg = g;
        __syncthreads();
        const uint32_t g = s_jg;
        if (g == NONE) {  // (invariant: k_sync_scatter_remote listed it from that record)
          if (threadIdx.x == 0) atomicOr(&P.ctl->overflow, OV_BUG);
          continue;
        }
        src = P.xrecv + (size_t)g * rw + 2;
        ack = P.jwin[from] == j ? P.xsend + (size_t)g * rw + 2 : nullptr;
        if (threadIdx.x == 0) {  // the record goes back to the joiner's shard in the SYNC_ACK exchange
          P.xsend[(size_t)g * rw] = P.jwin[from] == j ? (JOIN_REQ | from) : NONE;
          P.xsend[(size_t)g * rw + 1] = j;
        }
      }
      merge_row(P, j, src, ack, 0x80000000u | from, SWIM_R_SYNC, snap, seq, T, created, s_lds4);
      continue;
    }
    if (is_local(P, from)) {
      const uint32_t slot = P.req_stage[q];
      src = P.stage_sync + (size_t)slot * P.W;
      ack = P.stage_ack + (size_t)slot * P.W;
    } else {  // request from another shard: payload in the received record, ack into the same
      const size_t g = (size_t)P.rs_ref[q] * sync_rec_words(P);  // position of the send buffer
      src = P.xrecv + g + 2;
      ack = P.xsend + g + 2;
      if (threadIdx.x == 0) {
        P.xsend[g] = q;
        P.xsend[g + 1] = j;
      }
    }
    merge_row(P, j, src, ack, q, SWIM_R_SYNC, snap, seq, T, created, s_lds4);
  }
  if (threadIdx.x == 0) P.gseq[j] = seq;
  add_stat(P, ST_MERGE_CELLS, threadIdx.x == 0 ? cntj * sync_cells(P) : 0u);
  add_stat(P, ST_GOSSIPS_CREATED, created);
  flush_tally(P, T);
}

__global__ void __launch_bounds__(256, SWIM_SYNC_WAVES) k_sync_merge(KP P) {
  SWIM_GUARD(P);
  __shared__ uint32_t s_list[BUCKET_MAX];
  __shared__ uint32_t s_lds4[4];
  __shared__ uint32_t s_pre[SY_STRIPES + 1];
  // (sy_for_each's barrier after each receiver: s_list is refilled for the next one)
  sy_for_each(P.ctl->sy_mcnt, P.sy_mlist, P.sy_cap, s_pre, [&](uint32_t j) { sync_merge_one(P, j, s_list, s_lds4); });
}

// onSyncAck (MembershipProtocolImpl.java:343-349) at requester i = blockIdx.
__device__ __forceinline__ void sync_ack_one(const KP& P, uint32_t i, uint32_t* s_lds4) {
  uint32_t kd[3], to[3], n = 0;  // kind 0 / 1: request 2i + kind; kind 2: the initial SYNC's first ack
  for (uint32_t k = 0; k < 2; ++k) {
    const uint32_t qq = 2 * i + k;
    if (P.req_stage[qq] == NONE) continue;
    const uint32_t t = P.req_to[qq];
    if (!delivered(P, K_SYNC_ACK, t, i, k, P.tick)) continue;
    kd[n] = k;
    to[n] = t;
    ++n;
  }
  if (P.njoin && P.joining[i] && P.jwin[i] != NONE && (P.jslot[i] < P.scap || !is_local(P, P.jwin[i]))) {  // as k_join_select
    kd[n] = 2u;
    to[n] = P.jwin[i];
    ++n;
  }
  if (n == 0) return;
  for (uint32_t a = 1; a < n; ++a)  // (responder, kind) order
    for (uint32_t b = a; b > 0 && (to[b] < to[b - 1] || (to[b] == to[b - 1] && kd[b] < kd[b - 1])); --b) {
      uint32_t x = kd[b];
      kd[b] = kd[b - 1];
      kd[b - 1] = x;
      x = to[b];
      to[b] = to[b - 1];
      to[b - 1] = x;
    }
  Tally T;
  uint32_t created = 0;
  uint32_t seq = P.gseq[i];
  const uint32_t snap = P.cnt[i];
  for (uint32_t k = 0; k < n; ++k) {
    const uint32_t* src;
    uint32_t attempt, reason = SWIM_R_SYNC;
    if (kd[k] == 2u) {  // syncMembership(onStart = true): reason INITIAL_SYNC (MPI:463-473)
      src = is_local(P, to[k]) ? P.stage_ack + (size_t)P.jslot[i] * P.W
                               : P.xrecv + (size_t)P.jack_ref[i] * sync_rec_words(P) + 2;  // (the seed's shard)
      attempt = 0x80000000u | to[k];
      reason = SWIM_R_INITIAL_SYNC;
    } else {
      const uint32_t qq = 2 * i + kd[k], slot = P.req_stage[qq];
      attempt = (to[k] << 1) | kd[k];
      src = slot == REMOTE ? P.xrecv + (size_t)P.ack_ref[qq] * sync_rec_words(P) + 2 : P.stage_ack + (size_t)slot * P.W;
    }
    merge_row(P, i, src, nullptr, attempt, reason, snap, seq, T, created, s_lds4);
  }
  if (threadIdx.x == 0) P.gseq[i] = seq;
  add_stat(P, ST_ACKS_DELIVERED, threadIdx.x == 0 ? n : 0u);
  add_stat(P, ST_ACK_CELLS, threadIdx.x == 0 ? n * sync_cells(P) : 0u);
  add_stat(P, ST_GOSSIPS_CREATED, created);
  flush_tally(P, T);
}

// A workgroup per listed requester (k_sync_select, k_join_select), SY_GRID at most
__global__ void __launch_bounds__(256, SWIM_SYNC_WAVES) k_sync_ack(KP P) {
  SWIM_GUARD(P);
  __shared__ uint32_t s_lds4[4];
  __shared__ uint32_t s_pre[SY_STRIPES + 1];
  sy_for_each(P.ctl->sy_acnt, P.sy_alist, P.sy_cap, s_pre, [&](uint32_t i) { sync_ack_one(P, i, s_lds4); });
}

// ---------------------------------------------------------------------------------------
// Observability.
// ---------------------------------------------------------------------------------------
// Order-independent digests of every (observer, subject) record and deadline, the same sums
// for dense and N x K tables (an untracked subject contributes BASELINE in every row).
// one observer's deadlines (column-strided u16 cells), decoded to the oracle's deadline + 1 (0 = none)
// at period t, into a dense row: one 2-B element per row of a strided copy is the DMA engines' slow path
__global__ void k_read_dl(KP P, uint32_t lr, uint32_t t, uint32_t* out, uint32_t ncol) {
  for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < ncol; c += gridDim.x * blockDim.x) {
    const uint32_t e = P.dl[(size_t)c * P.nloc + lr];
    out[c] = e ? dl_dec(e, t) + 1u : 0u;
  }
}

__global__ void k_digest(KP P, unsigned long long* out) {
  const uint64_t K = 0x9E3779B97F4A7C15ull;
  const uint32_t N = P.N, nloc = P.nloc, row0 = P.row0, nc = ncells(P);
  unsigned long long a = 0, b = 0;
  const size_t total = (size_t)nloc * N;
  for (size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x; x < total; x += (size_t)gridDim.x * blockDim.x) {
    const uint32_t li = (uint32_t)(x / N), j = (uint32_t)(x % N);  // x = local observer * N + subject
    const uint32_t v = cell_get(P, row0 + li, j);
    if (v) a += fmix64(((uint64_t)row0 * N + x) * K + v);
  }
  const size_t dtot = (size_t)nc * nloc;
  for (size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x; x < dtot; x += (size_t)gridDim.x * blockDim.x) {
    const uint32_t e = P.dl[x];  // x = cell * nloc + local observer
    if (e) {
      const uint32_t d = dl_dec(e, P.period) + 1u;  // the oracle's deadline + 1
      const uint64_t subj = subj_of(P, (uint32_t)(x / nloc)), obs = row0 + x % nloc;
      b += fmix64((obs * N + subj) * K + d);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
  }
  if ((threadIdx.x & 63u) == 0) {
    atomicAdd(&out[0], a);
    atomicAdd(&out[1], b);
  }
}

__global__ void k_kat_overrides(const uint32_t* r1, const uint32_t* r0, uint8_t* out, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = is_overrides(r1[i], r0[i]) ? 1 : 0;
}

__global__ void k_kat_philox4(uint64_t seed, uint32_t kind, const uint32_t* abct, uint32_t* out, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const u32x4 v = draw4(seed, kind, abct[4 * i], abct[4 * i + 1], abct[4 * i + 2], abct[4 * i + 3]);
    out[4 * i] = v.x;
    out[4 * i + 1] = v.y;
    out[4 * i + 2] = v.z;
    out[4 * i + 3] = v.w;
  }
}

__global__ void k_kat_philox(uint64_t seed, uint32_t kind, const uint32_t* abct, uint32_t* out, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = draw1(seed, kind, abct[4 * i], abct[4 * i + 1], abct[4 * i + 2], abct[4 * i + 3]);
}

// The scans every kernel builds its compactions on (DPP wave scan, 1,024-thread block scan), on
// known inputs: one 1,024-thread workgroup per 1,024 elements, every lane active
__global__ void __launch_bounds__(1024) k_kat_scan(const uint32_t* in, uint32_t* wexcl, uint32_t* wtot,
                                                   uint32_t* bexcl, uint32_t* btot) {
  __shared__ uint32_t s_lds[16];
  const uint64_t i = (uint64_t)blockIdx.x * 1024u + threadIdx.x;
  const uint32_t v = in[i];
  uint32_t wt = 0, bt = 0;
  wexcl[i] = wave_excl_scan(v, &wt);
  if ((threadIdx.x & 63u) == 0u) wtot[i >> 6] = wt;
  bexcl[i] = block_excl_scan1024(v, &bt, s_lds);
  if (threadIdx.x == 0u) btot[blockIdx.x] = bt;
}

}  // namespace swim

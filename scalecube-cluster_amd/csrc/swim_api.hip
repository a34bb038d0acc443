// swim_api.hip — host side of libswimhip.so: the C ABI declared in include/swimhip.h.
//
// Owns all device state of one simulated cluster and launches one protocol period as a fixed
// sequence of kernels on the handle's stream (no host round trips inside a period). This is
// the replacement for ClusterImpl's per-member wiring of FailureDetectorImpl,
// GossipProtocolImpl and MembershipProtocolImpl (core/ClusterImpl.java:170-227) for N members.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "swim_kernels.hip"

using namespace swim;

namespace {

constexpr int NCLASS = 12;  // timing classes, see swim_kernel_time
constexpr uint32_t RB_CAP = 2048;  // slot entry bitmaps (k_slot_bm)
// exchanges whose every count follows from the status rows of the exchange before them (tr_period)
enum XKnown : uint32_t { XK_NONE = 0, XK_NEED, XK_ACK };
constexpr uint32_t SLOT_IDS_GRID = 64;  // k_dict_free's least workgroups while it copies short slots' entry ids
constexpr uint32_t RB_GRID = 256;  // k_slot_bm's workgroups (a grid stride over the commit's new slots)
#ifndef SWIM_RS_FUSE_ALL
#define SWIM_RS_FUSE_ALL 0  // (tests: every radix sort in one launch of CS_FUSE workgroups at most)
#endif
constexpr uint32_t DICT_GRID = 128;  // workgroups of the record-dictionary kernels (grid-stride)

uint32_t pow2ceil(uint64_t v) {
  uint64_t p = 1;
  while (p < v) p <<= 1;
  return (uint32_t)std::min<uint64_t>(p, 1ull << 31);
}

}  // namespace

struct swim_handle {
  swim_config cfg{};
  uint32_t N = 0, G = 1, S = 1, TPP = 5, GC = 0, scap = 0, ecap = 0;
  uint64_t period = 0;
  uint64_t part_t0 = 0, part_t1 = 0;
  hipStream_t stream = nullptr;
  KP base{};
  // period in flight (sharded handles stop at exchanges)
  KP cur{};
  int pc = 0;
  uint32_t q = 0;
  // sharding
  uint32_t world = 1, rank = 0;
  bool sharded = false;  // periods stop at exchanges: world > 1, or world 1 with a transport (a test of it)
  uint32_t n_leaving = 0;  // swim_leave calls so far (the stop check runs only once one happened)
  uint32_t n0 = 0;          // members started at create (swim_config.n_initial)
  std::vector<uint8_t> started;  // ids ever started (spare slots: until swim_join / swim_restart)
  void* xsend = nullptr;
  void* xrecv = nullptr;
  uint64_t xsend_words = 0, xrecv_words = 0;
  uint32_t* d_xcounts = nullptr;
  uint32_t* d_blx = nullptr;
  // gossip commits: sort keys/values (ping-pong) and the radix sort's counters (k_commit, k_rs_*)
  uint32_t *cs_ghist = nullptr, *cs_ctr = nullptr, *cs_stat = nullptr;
  uint32_t cs_maxt = 1;
  // k_gossip_apply launch: persistent workgroups (one or two per CU) and their dynamic LDS bytes
  uint32_t apply_blocks = 1, apply_blocks_b = 1, apply_waves_b = 1;
  bool dict_on = false;  // batching enabled: commits keep the record dictionary
  size_t apply_lds = 0, apply_lds_b = 0;  // k_gossip_apply / k_gossip_apply_b (batch slots)
  // shards of at most this many rows pull with a workgroup's 4 waves per receiver: one wave per
  // member would leave the chip's SIMDs at most 4 waves each (16 per CU; C2's 4,096 members on 256
  // CUs gain, 65,536 lose; the same split of select and of the batched apply measured slower:
  // DESIGN.md §6.5)
  uint32_t split_rows = 4096;
  uint32_t CC = 0;  // record ring of the gossip batches
  uint32_t dthr_cap = 0;  // entries of the allocated delay threshold table (swim_set_delay)
  uint32_t* crash_ids = nullptr;  // [N] the members one swim_crash call stops (allocated on first use)
  uint32_t* deliver_buf = nullptr;  // swim_deliver_records: subjects, then records (grown on demand)
  uint32_t* d_rowbuf = nullptr;     // swim_read_deadlines: one decoded row (allocated on first use)
  uint32_t deliver_cap = 0;
  unsigned long long* ck[2] = {nullptr, nullptr};
  unsigned long long* cv[2] = {nullptr, nullptr};
  // sharded gossip rounds: pairs sent / received, need-bitmap width, scan scratch
  uint32_t n_out_pairs = 0, n_in_pairs = 0, nneed = 0;
  uint32_t sync_rl = 0;  // cells of a SYNC row exchanged this period (sharded, read at the SYNC phase)
  uint32_t out_pairs[SWIM_MAX_WORLD] = {0};
  unsigned long long* d_digest = nullptr;
  uint32_t* d_scan = nullptr;  // k_scan_tiles sums and their exclusive scan
  // quiet periods: the gossip rounds of a period in which no member holds a gossip are
  // skipped (one k_quiet_rounds instead of ~15 launches per round). The test runs after the FD commit,
  // every period while the last one was quiet and every QUIET_EVERY-th period otherwise (a host stop)
  bool quiet_skip = true;   // SWIMHIP_QUIET=0 at swim_create: always run the rounds (tests: A/B)
  // gossips the host calls between periods may have staged (leave, spread, metadata updates, delivered
  // records): with the FD phase's own (one per member) they bound the FD commit's batch
  uint64_t host_staged = 0;
  bool last_quiet = false;
  bool period_quiet = false;  // this period's rounds were skipped
  uint64_t quiet_periods = 0;
  uint32_t* d_quiet = nullptr;
  uint32_t* h_quiet = nullptr;  // pinned
  std::vector<void*> allocs;
  // library-driven exchanges (swim_shard_set_transport / swim_shard_comm_init)
  swim_transport tr{};
  bool has_tr = false;
  ncclComm_t comm = nullptr;
  uint64_t* d_status = nullptr;  // [(1 + world) * (XS_CNT + world)]: this rank's status row, then all ranks'
  uint32_t xpend = 0;  // XsKind whose k_xstatus row awaits xpost
  uint32_t xknown = 0;  // XK_*: the exchange period_resume returned has counts the last status rows give
  // Pinned host words of the exchanges (sharded handles): small copies from pageable memory go through
  // a staging buffer and wait for it, so every copy of a period's exchanges is pinned
  struct XPin {
    uint64_t head[2];                                      // the status row's host half {code, op}
    uint32_t chead[4];                                     // a commit block's header
    uint32_t offs[SWIM_MAX_WORLD];                         // commit blocks' tail offsets
    uint32_t cnt[SWIM_MAX_WORLD];                          // N x K track counts
    uint32_t bhead[2];                                     // a received commit block's header
    uint64_t xrow[XS_CNT + SWIM_MAX_WORLD];                // host-driven exchanges: this rank's row
    uint64_t rows[SWIM_MAX_WORLD * (XS_CNT + SWIM_MAX_WORLD)];  // the gathered status rows
  };
  XPin* xp = nullptr;
  std::vector<uint8_t> hsend, hrecv;  // host staging of a host_staged transport
  std::string err;
  // timing
  bool timing = false;
  uint32_t tmask = ~0u;  // kernel classes bracketed by HIP events while timing
  std::vector<hipEvent_t> pool;
  struct Pending {
    int cls;
    hipEvent_t a, b;
  };
  std::vector<Pending> pending;
  double acc_ms[NCLASS] = {0};
  uint64_t acc_n[NCLASS] = {0};
};

namespace {

int fail(swim_handle* h, int code, const std::string& what) {
  if (h) h->err = what;
  return code;
}

#define HIPC(h, expr)                                                                              \
  do {                                                                                             \
    hipError_t e_ = (expr);                                                                        \
    if (e_ != hipSuccess) return fail((h), SWIM_EHIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

#define HIPC_RC(h, rcp, expr)                                                                      \
  do {                                                                                             \
    hipError_t e_ = (expr);                                                                        \
    if (e_ != hipSuccess) {                                                                        \
      *(rcp) = fail((h), SWIM_EHIP, std::string(#expr ": ") + hipGetErrorString(e_));              \
      return false;                                                                                \
    }                                                                                              \
  } while (0)

template <typename T>
int dalloc(swim_handle* h, T** p, size_t count) {
  void* q = nullptr;
  if (count == 0) count = 1;
  hipError_t e = hipMalloc(&q, count * sizeof(T));
  if (e != hipSuccess)
    return fail(h, SWIM_ENOMEM, "hipMalloc(" + std::to_string(count * sizeof(T)) + " B): " + hipGetErrorString(e));
  h->allocs.push_back(q);
  *p = (T*)q;
  return SWIM_OK;
}

void free_all(swim_handle* h) {
  if (h->comm) (void)ncclCommDestroy(h->comm);
  h->comm = nullptr;
  for (void* p : h->allocs) (void)hipFree(p);
  h->allocs.clear();
  if (h->h_quiet) (void)hipHostFree(h->h_quiet);
  h->h_quiet = nullptr;
  if (h->xp) (void)hipHostFree(h->xp);
  h->xp = nullptr;
  for (auto ev : h->pool) (void)hipEventDestroy(ev);
  for (auto& pe : h->pending) {
    (void)hipEventDestroy(pe.a);
    (void)hipEventDestroy(pe.b);
  }
  h->pool.clear();
  h->pending.clear();
  if (h->stream) (void)hipStreamDestroy(h->stream);
  h->stream = nullptr;
}

hipEvent_t take_event(swim_handle* h) {
  if (!h->pool.empty()) {
    hipEvent_t e = h->pool.back();
    h->pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

void resolve_timing(swim_handle* h) {
  for (auto& pe : h->pending) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, pe.a, pe.b) == hipSuccess) {
      h->acc_ms[pe.cls] += ms;
      h->acc_n[pe.cls] += 1;
    }
    h->pool.push_back(pe.a);
    h->pool.push_back(pe.b);
  }
  h->pending.clear();
}

// launch helper: optional per-launch HIP-event bracketing on the handle's stream
// SWIMHIP_DEBUG_SYNC=1: synchronize after every timed launch and name the first kernel that
// fails (a device fault otherwise surfaces at the next copy, far from its cause)
bool debug_sync() {
  static const bool on = [] {
    const char* e = std::getenv("SWIMHIP_DEBUG_SYNC");
    return e && *e == '1';
  }();
  return on;
}

template <typename F>
void timed(swim_handle* h, int cls, const char* name, F&& launch) {
  if (!h->timing || !((h->tmask >> cls) & 1u)) {
    launch();
  } else {
    hipEvent_t a = take_event(h), b = take_event(h);
    (void)hipEventRecord(a, h->stream);
    launch();
    (void)hipEventRecord(b, h->stream);
    h->pending.push_back({cls, a, b});
  }
  if (debug_sync()) {
    const hipError_t e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) {  // stop at once: nothing more may run on a faulted device
      std::fprintf(stderr, "swimhip debug: %s (period %llu, phase pc %d) failed: %s\n", name,
                   (unsigned long long)h->period, h->pc, hipGetErrorString(e));
      std::fflush(stderr);
      std::_Exit(3);
    }
  }
}

uint32_t blocks_for(uint64_t n, uint32_t bs) { return (uint32_t)std::max<uint64_t>(1, (n + bs - 1) / bs); }

void memset_ctl_u32(swim_handle* h, size_t offset) {
  (void)hipMemsetAsync(reinterpret_cast<char*>(h->base.ctl) + offset, 0, 4, h->stream);
}

// ---- one protocol period as a resumable sequence ---------------------
// Unsharded handles run a period straight through. Sharded handles (world > 1) stop at each
// cross-shard exchange, describe it in a swim_xchg, and resume after the host's collective.
enum Pc : int { PC_FD = 0, PC_FD_TRACK, PC_FD_C, PC_R_MAX, PC_R_SEL, PC_R_NEED, PC_R_WIN, PC_R_PULL, PC_R_C, PC_SUSP, PC_SYNC_REQ, PC_SYNC_ACK, PC_END };

void set_phase(swim_handle* h, KP& P, uint32_t phase) {
  const uint32_t t = (uint32_t)h->period, G = h->G, TPP = h->TPP;
  P = h->base;
  P.period = t;
  P.part_active = (h->period >= h->part_t0 && h->period < h->part_t1) ? 1u : 0u;
  P.phase = phase;
  P.tick = t * TPP + phase;
  if (phase == 0) {
    P.round = t * G;
    P.create_round = t * G;
  } else if (phase <= G) {
    P.round = t * G + phase - 1;
    P.create_round = t * G + phase;
    P.act = P.act_ring + (size_t)(P.round & 255u) * P.astride;  // this round's active list
  } else {
    P.round = (t + 1) * G;
    P.create_round = (t + 1) * G;
  }
}

// N x K: allocate the requested columns (one thread per subject), then re-sort the column order
void track_commit(swim_handle* h, const KP& P) {
  hipLaunchKernelGGL(k_track_alloc, dim3(1), dim3(1024), 0, h->stream, P);
  hipLaunchKernelGGL(k_colorder, dim3(1), dim3(256), 0, h->stream, P);
}

void xchg_clear(swim_xchg* x, uint32_t op, uint32_t world) {
  std::memset(x, 0, sizeof *x);
  x->op = op;
  x->world = world;
}

int check_overflow(swim_handle* h);

// words after a commit exchange block's gossips: per-word liveness, bit-length bounds, and (dense
// tmode) the touched-column bitmap
uint64_t commit_tail(const swim_handle* h) { return h->GC / 32 + 2ull + (h->base.tmode ? h->N / 32 : 0u); }

// Order the phase's gossips by (subject, record) and commit them: one k_commit launch. stg != nullptr: the local stage, counted on the device (no host round trip); otherwise
// the n gathered gossips already in h->ck[0] / h->cv[0].
int commit_sorted(swim_handle* h, const KP& P0, const uint4* stg, uint32_t n, uint32_t bound = NONE,
                  bool fused = false) {
  hipStream_t s = h->stream;
  KP P = P0;
  if (P.batch_commit && !h->base.batched) {  // from now on the ring may hold batch slots
    h->base.batched = 1u;
    h->cur.batched = 1u;
    P.batched = 1u;
    // the live one-gossip slots committed before get their counts too (slot_gossips reads them)
    hipLaunchKernelGGL(k_commit_wsum, dim3(64), dim3(256), 0, s, P, 1u);
  }
  CSort C{h->ck[0], h->cv[0], h->ck[1], h->cv[1], h->cs_ghist, h->cs_ctr, h->cs_stat, h->cs_maxt, 0u, 0u};
  // key = subject << 32 | record (user gossips: subject N + origin) or origin << 32 | subject
  C.npass = (32u + bitlen(2u * h->N - 1u) + 7u) / 8u;
  // launch the radix kernels only when the batch may need them: the sharded batch size is known
  // here; a local stage is bounded by the phase (`bound`: a gossip round stages at most one
  // refutation per member, MPI:549-569; k_commit fails loudly if a bound is ever exceeded)
  const bool big = stg != nullptr ? bound > CS_SMALL : n > CS_SMALL;
  // radix grids of the tiles the bound allows (a gossip round: nloc / CS_TILE), not of the stage's
  // capacity: launches that find a small batch return at once, and are cheaper the smaller they are
  const uint32_t tiles = stg ? (bound == NONE ? h->cs_maxt : std::min(h->cs_maxt, blocks_for(bound, CS_TILE)))
                             : std::max<uint32_t>(1, (n + CS_TILE - 1) / CS_TILE);
  C.radix = big ? tiles : 0u;
  timed(h, 7, "k_commit", [&] {
    hipLaunchKernelGGL(k_commit, dim3(1), dim3(CS_THREADS), 0, s, P, stg, n, C);
    if (big && (tiles <= CS_FUSE || fused || SWIM_RS_FUSE_ALL)) {
      hipLaunchKernelGGL(k_rs_fused, dim3(std::min(tiles, CS_FUSE)), dim3(CS_THREADS), 0, s, P, stg, n, C);
    } else if (big) {
      hipLaunchKernelGGL(k_rs_hist, dim3(tiles), dim3(CS_THREADS), 0, s, P, stg, n, C);
      for (uint32_t p = 0; p < C.npass; ++p) {
        const bool even = (p & 1u) == 0u;
        hipLaunchKernelGGL(k_rs_pass, dim3(tiles), dim3(CS_THREADS), 0, s, P, stg, n, C, p, even ? C.k0 : C.k1,
                           even ? C.v0 : C.v1, even ? C.k1 : C.k0, even ? C.v1 : C.v0);
      }
      const bool in0 = (C.npass & 1u) == 0u;
      const unsigned long long* ks = in0 ? C.k0 : C.k1;
      hipLaunchKernelGGL(k_rs_slots, dim3(tiles), dim3(CS_THREADS), 0, s, P, stg, n, C, ks);
      hipLaunchKernelGGL(k_excl_scan, dim3(1), dim3(CS_THREADS), 0, s, C.stat, C.stat + C.maxt, C.maxt);
      hipLaunchKernelGGL(k_rs_commit, dim3(tiles), dim3(CS_THREADS), 0, s, P, stg, n, C, ks, in0 ? C.v0 : C.v1);
      hipLaunchKernelGGL(k_rs_fin, dim3(1), dim3(1), 0, s, P, stg, n, C);
    }
    // batch slots: the gossips per bitmap word of the words this commit wrote (counter weights)
    // (with the dictionary on, in k_dict_claim's launch)
    if (P.batched && !h->dict_on) hipLaunchKernelGGL(k_commit_wsum, dim3(64), dim3(256), 0, s, P, 0u);
    // the record dictionary of the batched apply: every commit while batching is
    // enabled, so records committed before the first batch have their entries too. (One launch with
    // grid barriers between the steps measured slower: 38 us against ~4 per launch, §6.5.) The short
    // slots' entry ids (16-bit ids) are copied in k_dict_free's launch, after the entries.
    if (h->dict_on) {
      hipLaunchKernelGGL(k_dict_claim, dim3(DICT_GRID), dim3(256), 0, s, P, P.batched);
      hipLaunchKernelGGL(k_dict_entries, dim3(DICT_GRID), dim3(256), 0, s, P);
      hipLaunchKernelGGL(k_dict_free, dim3(std::max<uint32_t>(P.cid16 ? SLOT_IDS_GRID : 1u, P.dsids / 256)), dim3(256), 0,
                         s, P, P.cid16);
      // the entry bitmaps of this commit's long batch ranges (dsids bytes of LDS per workgroup)
      if (P.batched && P.rb_cap) hipLaunchKernelGGL(k_slot_bm, dim3(RB_GRID), dim3(256), P.dsids, s, P);
    }
  });
  return SWIM_OK;
}

// The end of a pack before an exchange. A host that performs the exchange itself (swim_shard_step) reads
// the send buffer once swim_shard_step returns, so the stream is synchronized here; the library's own
// transports are ordered on the stream already (RCCL enqueues on it; a host-staged transport copies the
// buffer out and synchronizes before its callback), so they skip this host stop (round 6: 7 of a
// period's ~2 x (4 + 4G) host stops at G = 5 are these).
hipError_t xorder(swim_handle* h) { return h->has_tr ? hipSuccess : hipStreamSynchronize(h->stream); }

// An exchange's device-side failure, on the rank whose state raised it (the others report "rank q failed")
int xown_fail(swim_handle* h, uint32_t kind) {
  switch (kind) {
    case XS_COMMIT:
    case XS_DONE: {
      const int rc = check_overflow(h);
      return rc ? rc : fail(h, SWIM_EOVERFLOW, "simulator buffer overflow");
    }
    case XS_SEL: return fail(h, SWIM_EOVERFLOW, "active list too long for sharded need bitmaps");
    case XS_WIN: return fail(h, SWIM_EOVERFLOW, "gossip exchange buffer too small");
    case XS_SYNC: return fail(h, SWIM_EOVERFLOW, "SYNC exchange over sync_capacity");
    default: return fail(h, SWIM_EINVAL, "shard exchange: unknown status kind");
  }
}

// The host half of an exchange whose counts k_xstatus wrote into `row` (this rank's status row, after the
// status all-gather, or read back by xready): pack the send buffer and set this rank's send counts.
int xpost(swim_handle* h, swim_xchg* x, const uint64_t* row) {
  const uint32_t kind = h->xpend, W = h->world;
  h->xpend = XS_NONE;
  hipStream_t s = h->stream;
  KP& P = h->cur;
  P.xsend = reinterpret_cast<uint32_t*>(h->xsend);
  switch (kind) {
    case XS_COMMIT: {
      // Once any member left (n_leaving: the same on every rank, swim_leave is collective), each block
      // starts with a header {gossips, stopped members, 0, 0} and carries the members this shard
      // stopped (k_leave_stop) after its gossips: liveness is replicated. Block layout:
      //   [header (leaves only) | gossips 4n | stopped (leaves only) | wlast W32 | bhi | 32 - blo]
      const uint32_t n = (uint32_t)row[XS_A0], ns = (uint32_t)row[XS_A1];
      const uint32_t hdr = h->n_leaving ? 4u : 0u;
      uint32_t* xs = P.xsend;
      if (hdr) {
        h->xp->chead[0] = n;
        h->xp->chead[1] = ns;
        h->xp->chead[2] = h->xp->chead[3] = 0u;
        HIPC(h, hipMemcpyAsync(xs, h->xp->chead, 16, hipMemcpyHostToDevice, s));
      }
      if (n) HIPC(h, hipMemcpyAsync(xs + hdr, P.stg, (size_t)n * 16, hipMemcpyDeviceToDevice, s));
      if (ns) HIPC(h, hipMemcpyAsync(xs + hdr + 4u * n, P.stop_list, (size_t)ns * 4, hipMemcpyDeviceToDevice, s));
      HIPC(h, hipMemsetAsync(&P.ctl->stg_count, 0, 8, s));  // stg_count and n_stop
      hipLaunchKernelGGL(k_round_max_pack, dim3(64), dim3(256), 0, s, P, hdr + 4u * n + ns);
      x->send_words = row[XS_CNT];
      break;
    }
    case XS_TRACK:  // (k_track_pack ran before k_xstatus)
      x->send_words = row[XS_CNT];
      return SWIM_OK;
    case XS_SEL: {  // (1) registrations with receivers on other shards
      h->nneed = ((uint32_t)row[XS_A0] + 31u) / 32u;
      uint32_t n_rec = 0;
      for (uint32_t q = 0; q < W; ++q) {
        x->send_counts[q] = row[XS_CNT + q];
        h->out_pairs[q] = (uint32_t)(row[XS_CNT + q] / 2);
        n_rec += h->out_pairs[q];
      }
      h->n_out_pairs = n_rec;
      if (n_rec) hipLaunchKernelGGL(k_gossip_pack_pairs, dim3(blocks_for(n_rec, 256)), dim3(256), 0, s, P, n_rec);
      break;
    }
    case XS_WIN:  // (3) the needed window words
      for (uint32_t q = 0; q < W; ++q) x->send_counts[q] = row[XS_CNT + q];
      P.nneed = h->nneed;
      hipLaunchKernelGGL(k_gossip_pack_sparse, dim3(std::min<uint32_t>(h->n_out_pairs, 8192)), dim3(256), 0, s, P,
                         h->n_out_pairs, h->nneed);
      break;
    case XS_SYNC: {  // tables of requesters whose receiver lives on another shard
      h->sync_rl = (uint32_t)row[XS_A0];  // (the same on every shard: tbits are merged)
      const uint32_t n_rec = (uint32_t)row[XS_A1];
      for (uint32_t q = 0; q < W; ++q) x->send_counts[q] = row[XS_CNT + q];
      if (n_rec) hipLaunchKernelGGL(k_sync_pack, dim3(std::min<uint32_t>(n_rec, 4096)), dim3(256), 0, s, P, n_rec);
      break;
    }
    case XS_DONE:
      resolve_timing(h);
      return SWIM_OK;
    default:
      return fail(h, SWIM_EINVAL, "shard exchange: unknown status kind");
  }
  HIPC(h, xorder(h));
  return SWIM_OK;
}

// An exchange whose counts are on the device: k_xstatus writes them, and what this
// shard's state says is wrong, into this rank's status row. With a transport the row rides the status
// all-gather, one host stop for both, and tr_period runs xpost after it; a host that performs the
// exchanges itself (swim_shard_step) reads the row back here and goes on at once. x->op is set.
int xready(swim_handle* h, const KP& P, swim_xchg* x, XsArgs a) {
  if (!h->d_status || !h->xp || !h->xsend) return fail(h, SWIM_EINVAL, "sharded handle: swim_shard_attach or a transport first");
  a.world = h->world;
  hipLaunchKernelGGL(k_xstatus, dim3(1), dim3(64), 0, h->stream, (const Ctl*)P.ctl, (const uint32_t*)P.woff,
                     h->d_status, a);
  h->xpend = a.kind;
  if (h->has_tr) return SWIM_OK;
  uint64_t* row = h->xp->xrow;
  HIPC(h, hipMemcpyAsync(row, h->d_status, 8ull * (XS_CNT + h->world), hipMemcpyDeviceToHost, h->stream));
  HIPC(h, hipStreamSynchronize(h->stream));
  if (row[XS_ERR]) {
    h->xpend = XS_NONE;
    return xown_fail(h, a.kind);
  }
  return xpost(h, x, row);
}

// Commit the phase's staged gossips. Unsharded: in place, sized on the device (overflow is
// reported at the next swim_sync; k_gossip_prep lists nothing once it is set, so a run never
// feeds a wrapped ring to the gossip kernels). Sharded: the host all-gathers every shard's stage
// first (returns true: exchange pending); all shards then sort the same batch.
bool commit_begin(swim_handle* h, const KP& P, swim_xchg* x, int* rc, uint32_t bound = NONE, bool fused = false) {
  if (!h->sharded) {
    *rc = commit_sorted(h, P, P.stg, 0u, bound, fused);
    return false;
  }
  // {overflow, stg_count, n_stop} go into the status row (k_xstatus): a sharded run stops at the first
  // phase whose buffers overflowed, every rank at the same exchange; the block is packed after (xpost)
  XsArgs a{};
  a.kind = XS_COMMIT;
  a.cap = P.stg_cap;
  a.hdr = h->n_leaving ? 4u : 0u;
  a.nloc = h->n_leaving ? P.nloc : 0u;
  a.tail = commit_tail(h);
  xchg_clear(x, SWIM_X_ALLGATHER, h->world);
  *rc = xready(h, P, x, a);
  return *rc == SWIM_OK;
}

int commit_end(swim_handle* h, const KP& P, const swim_xchg* x) {
  hipStream_t s = h->stream;
  const uint32_t* xr = reinterpret_cast<const uint32_t*>(h->xrecv);
  uint32_t total = 0, *offs = h->xp->offs;
  const uint64_t tail = commit_tail(h);  // wlast + bounds (+ touched columns) after each shard's gossips
  for (uint32_t q = 0; q < h->world; ++q) {
    const uint32_t* blk = xr + q * x->recv_stride;
    uint32_t c = 0, ns = 0, hdr = 0;
    if (h->n_leaving) {  // the block's header: gossips and stopped members
      uint32_t* head = h->xp->bhead;
      HIPC(h, hipMemcpyAsync(head, blk, 8, hipMemcpyDeviceToHost, s));
      HIPC(h, hipStreamSynchronize(s));
      c = head[0];
      ns = head[1];
      hdr = 4u;
      if (hdr + 4ull * c + ns + tail != x->recv_counts[q])
        return fail(h, SWIM_EINVAL, "commit exchange: block header does not match its size");
      if (ns && q != h->rank)
        hipLaunchKernelGGL(k_stop_remote, dim3(blocks_for(ns, 256)), dim3(256), 0, s, P, blk + hdr + 4u * c, ns);
    } else {
      c = (uint32_t)((x->recv_counts[q] - tail) / 4);
    }
    offs[q] = (uint32_t)(q * x->recv_stride + hdr + 4ull * c + ns);
    if (c)
      hipLaunchKernelGGL(k_stage_keys, dim3(blocks_for(c, 256)), dim3(256), 0, s, P,
                         reinterpret_cast<const uint4*>(blk + hdr), c, total, h->ck[0], h->cv[0]);
    total += c;
  }
  // liveness maxima first: the commit itself then raises the new words on every shard alike
  HIPC(h, hipMemcpyAsync(h->d_xcounts, offs, 4ull * h->world, hipMemcpyHostToDevice, s));
  KP Q = P;
  Q.xrecv = xr;
  hipLaunchKernelGGL(k_round_max_merge, dim3(64), dim3(256), 0, s, Q, h->d_xcounts, h->d_blx);
  return commit_sorted(h, P, nullptr, total);
}

// Quiet periods: after the FD commit, may any member hold a gossip in this period's
// rounds (k_quiet_check)? If none may, the rounds' bookkeeping is written in one launch and the
// period goes on at the suspicion phase: ~15 launches per round fewer, and on sharded handles 4
// exchanges per round fewer. The test reads replicated state on sharded handles (the ring, wlast and
// the commit counts are the same on every shard after the commit exchange), so every rank takes the
// same branch; the exchange status rows carry the resume point (tr_status), so ranks that did not
// would fail together instead of exchanging mismatched buffers. Handles with delayed-message rings,
// leaves or joins in flight always run their rounds.
constexpr uint64_t QUIET_EVERY = 8;  // periods between tests while the last test found gossips held
int quiet_rounds(swim_handle* h, bool* quiet) {
  *quiet = false;
  h->period_quiet = false;
  if (!h->quiet_skip || h->base.dq || h->n_leaving || h->base.njoin) return SWIM_OK;
  if (!h->last_quiet && h->period % QUIET_EVERY != 0) return SWIM_OK;
  hipStream_t s = h->stream;
  KP Q;
  set_phase(h, Q, 1);  // the period's first gossip round
  hipLaunchKernelGGL(k_quiet_check, dim3(1), dim3(1024), 0, s, Q, Q.round, h->d_quiet);
  HIPC(h, hipMemcpyAsync(h->h_quiet, h->d_quiet, 4, hipMemcpyDeviceToHost, s));
  HIPC(h, hipStreamSynchronize(s));
  h->last_quiet = *h->h_quiet == 0u;
  if (!h->last_quiet) return SWIM_OK;
  timed(h, 7, "k_quiet_rounds", [&] {
    hipLaunchKernelGGL(k_quiet_rounds, dim3(blocks_for(h->base.nloc, 256)), dim3(256), 0, s, Q, Q.round, h->G);
    if (h->dict_on) hipLaunchKernelGGL(k_dict_free, dim3(std::max<uint32_t>(1, Q.dsids / 256)), dim3(256), 0, s, Q, 0u);
  });
  h->quiet_periods++;
  h->period_quiet = true;
  *quiet = true;
  return SWIM_OK;
}

// Runs the current period from h->pc. Returns SWIM_OK with x->op = SWIM_X_DONE at the end of
// the period, or SWIM_OK with another op when an exchange must happen first (world > 1).
int period_resume(swim_handle* h, swim_xchg* x) {
  const uint32_t N = h->N, G = h->G, W = h->world, nloc = h->base.nloc;
  const bool SH = h->sharded;  // exchanges happen (world > 1, or a world-1 handle with a transport)
  uint32_t& RL = h->sync_rl;  // cells of this period's SYNC rows (dense N or touched, N x K the K columns)
  const uint32_t gL = blocks_for(nloc, 256);
  hipStream_t s = h->stream;
  KP& P = h->cur;
  int rc = SWIM_OK;
  for (;;) {
    switch (h->pc) {
      case PC_FD:  // phase 0: failure detector
        set_phase(h, P, 0);
        h->pc = PC_FD_TRACK;
        if (P.nxk) {  // N x K: columns for the subjects this FD phase changes first
          timed(h, 0, "k_fd_track", [&] { hipLaunchKernelGGL(k_fd_track, dim3(gL), dim3(256), 0, s, P); });
          if (SH) {  // every shard's requests to every shard: all allocate the same columns
            P.xsend = reinterpret_cast<uint32_t*>(h->xsend);
            hipLaunchKernelGGL(k_track_pack, dim3(1), dim3(256), 0, s, P);
            xchg_clear(x, SWIM_X_ALLGATHER, W);
            XsArgs a{};
            a.kind = XS_TRACK;
            a.cap = P.tcap;
            return xready(h, P, x, a);
          }
          track_commit(h, P);
        }
        break;
      case PC_FD_TRACK:
        if (P.nxk && SH) {
          uint32_t* cnt = h->xp->cnt;
          for (uint32_t q = 0; q < W; ++q) cnt[q] = (uint32_t)x->recv_counts[q];
          HIPC(h, hipMemcpyAsync(h->d_xcounts, cnt, 4ull * W, hipMemcpyHostToDevice, s));
          P.xrecv = reinterpret_cast<const uint32_t*>(h->xrecv);
          hipLaunchKernelGGL(k_track_unpack, dim3(1), dim3(256), 0, s, P, h->d_xcounts, (uint32_t)x->recv_stride);
          track_commit(h, P);
        }
        timed(h, 0, "k_fd", [&] { hipLaunchKernelGGL(k_fd, dim3(gL), dim3(256), 0, s, P); });
        // a DEST_GONE ack (restarted address) removes the probed member in this phase: its count
        // change is visible from the first gossip round on, as at the end of every other phase
        timed(h, 7, "k_finalize", [&] { hipLaunchKernelGGL(k_finalize, dim3(gL), dim3(256), 0, s, P); });
        h->pc = PC_FD_C;
        {  // the phase's batch is bounded: at most two FD gossips per member (a SUSPECT, then a DEAD of a
           // DEST_GONE ack, MPI:376-404) plus what the host calls since the last period staged. A bound
           // within CS_FUSE tiles sorts a storm's batch in one k_rs_fused launch (or in k_commit's LDS
           // sort) instead of the eleven-launch radix chain sized for the stage's capacity
          const uint64_t fd_bound = std::min<uint64_t>(2ull * nloc + h->host_staged, NONE - 1u);
          h->host_staged = 0;
          if (commit_begin(h, P, x, &rc, (uint32_t)fd_bound)) return SWIM_OK;
        }
        if (rc) return rc;
        break;
      case PC_FD_C: {
        if (SH && (rc = commit_end(h, P, x))) return rc;
        h->q = 0;
        bool quiet = false;
        if ((rc = quiet_rounds(h, &quiet))) return rc;
        h->pc = quiet ? PC_SUSP : PC_R_MAX;
        break;
      }
      case PC_R_MAX:  // phases 1..G: gossip rounds
        set_phase(h, P, 1 + h->q);
        h->pc = PC_R_SEL;
        break;
      case PC_R_SEL:
        if (SH) {  // liveness + bounds over every shard arrived with the last commit
          P.blx = h->d_blx;
          HIPC(h, hipMemsetAsync(P.ctl->xg_cnt, 0, sizeof(uint32_t) * SWIM_MAX_WORLD, s));
        }
        timed(h, 7, "k_gossip_prep", [&] { hipLaunchKernelGGL(k_gossip_prep, dim3(1), dim3(1024), 0, s, P); });
        timed(h, 8, "k_gossip_select", [&] {
          hipLaunchKernelGGL(P.hd4 ? k_gossip_select_h4 : k_gossip_select, dim3(blocks_for(nloc, 4)), dim3(256), 0, s, P);
        });
        timed(h, 10, "k_gossip_pairfill", [&] { hipLaunchKernelGGL(k_gossip_pairfill, dim3(1024), dim3(256), 0, s, P); });
        timed(h, 10, "k_gossip_pairprune", [&] { hipLaunchKernelGGL(k_gossip_pairprune, dim3(2048), dim3(256), 0, s, P); });
        if (P.dq)  // rings exist once a delay was set; messages in flight arrive even after it is reset
          timed(h, 10, "k_gossip_pairdelay", [&] { hipLaunchKernelGGL(k_gossip_pairdelay, dim3(1024), dim3(256), 0, s, P); });
        h->pc = PC_R_NEED;
        if (SH) {  // (1) registrations with receivers on other shards (packed by xpost)
          xchg_clear(x, SWIM_X_ALLTOALLV, W);
          XsArgs a{};
          a.kind = XS_SEL;
          return xready(h, P, x, a);
        }
        h->pc = PC_R_PULL;
        break;
      case PC_R_NEED: {  // (2) receiver side: what each received pair's receiver still lacks
        if (x->recv_stride == 0) {  // no shard registered a remote receiver: nothing to ask or ship
          h->n_in_pairs = 0;
          h->pc = PC_R_PULL;
          break;
        }
        uint64_t words = 0;
        for (uint32_t q = 0; q < W; ++q) words += x->recv_counts[q];
        const uint32_t n_in = (uint32_t)(words / 2);
        uint64_t back[SWIM_MAX_WORLD];
        for (uint32_t q = 0; q < W; ++q) back[q] = x->recv_counts[q] / 2 * h->nneed;
        h->n_in_pairs = n_in;
        P.nneed = h->nneed;
        P.xsend = reinterpret_cast<uint32_t*>(h->xsend);
        P.xrecv = reinterpret_cast<const uint32_t*>(h->xrecv);
        if (n_in) {
          hipLaunchKernelGGL(k_gossip_need, dim3(std::min<uint32_t>(n_in, 8192)), dim3(256), 0, s, P, n_in, h->nneed);
          hipLaunchKernelGGL(k_excl_scan, dim3(1), dim3(CS_THREADS), 0, s, P.rtot, P.roff, n_in);
        }
        xchg_clear(x, SWIM_X_ALLTOALLV, W);
        for (uint32_t q = 0; q < W; ++q) x->send_counts[q] = back[q];
        HIPC(h, xorder(h));
        h->pc = PC_R_WIN;
        h->xknown = XK_NEED;
        return SWIM_OK;
      }
      case PC_R_WIN: {  // (3) sender side: ship the needed window words
        const uint32_t n_out = h->n_out_pairs;
        P.xsend = reinterpret_cast<uint32_t*>(h->xsend);
        P.xrecv = reinterpret_cast<const uint32_t*>(h->xrecv);
        P.nneed = h->nneed;
        xchg_clear(x, SWIM_X_ALLTOALLV, W);
        h->pc = PC_R_PULL;
        if (n_out) {  // per-peer volumes from the scanned word counts (k_xstatus), packed by xpost
          hipLaunchKernelGGL(k_gossip_wcount, dim3(blocks_for(n_out, 256)), dim3(256), 0, s, P, n_out, h->nneed);
          hipLaunchKernelGGL(k_excl_scan, dim3(1), dim3(CS_THREADS), 0, s, P.wcnt, P.woff, n_out + 1);
          XsArgs a{};
          a.kind = XS_WIN;
          a.cap = (uint32_t)std::min<uint64_t>(h->xsend_words, NONE);
          for (uint32_t q = 0; q < W; ++q) a.bnd[q + 1] = a.bnd[q] + h->out_pairs[q];
          return xready(h, P, x, a);
        }
        return SWIM_OK;
      }
      case PC_R_PULL:
        if (SH) {
          P.xrecv = reinterpret_cast<const uint32_t*>(h->xrecv);
          P.nneed = h->nneed;
          if (h->n_in_pairs)
            hipLaunchKernelGGL(k_gossip_unpack, dim3(blocks_for(h->n_in_pairs, 256)), dim3(256), 0, s, P,
                               h->n_in_pairs);
        }
        timed(h, 9, "k_gossip_inhist", [&] { hipLaunchKernelGGL(k_gossip_inhist, dim3(blocks_for(nloc, 4)), dim3(256), 0, s, P); });
        timed(h, 1, "k_gossip_pull", [&] {
          // small shards: a workgroup per receiver, its 4 waves splitting the active list
          const bool split = nloc <= std::min(PULL_SPLIT_N, h->split_rows);
          if (P.dq)
            hipLaunchKernelGGL(k_gossip_pull_dq, dim3(blocks_for(nloc, 4)), dim3(256), 0, s, P);
          else if (P.loss_mode == 1u)  // the loss draws' instance (§3.16's split, for registers)
            hipLaunchKernelGGL(split ? k_gossip_pull_loss_s4 : k_gossip_pull_loss, dim3(split ? nloc : blocks_for(nloc, 4)),
                               dim3(256), 0, s, P);
          else
            hipLaunchKernelGGL(split ? k_gossip_pull_s4 : k_gossip_pull, dim3(split ? nloc : blocks_for(nloc, 4)),
                               dim3(256), 0, s, P);
        });
        timed(h, 11, "k_gossip_record", [&] { hipLaunchKernelGGL(k_gossip_record, dim3(REC_GRID), dim3(256), 0, s, P); });
        timed(h, 2, "k_gossip_apply", [&] {
          // with the record dictionary (gossip batching on, the default) the batched apply runs whether
          // or not the ring holds batch slots: one-gossip slots (probabilistic loss, delays) are subject
          // runs it takes as run tops (C4's lossy storm: apply 373 -> 104 ms per 20 periods, §6.4)
          if (P.batched || h->dict_on)
            hipLaunchKernelGGL(P.cid16 ? (P.hd4 ? k_gossip_apply_b16_h4 : k_gossip_apply_b16)
                                       : (P.hd4 ? k_gossip_apply_b_h4 : k_gossip_apply_b),
                               dim3(h->apply_blocks_b), dim3(64 * h->apply_waves_b), h->apply_lds_b, s, P);
          else
            hipLaunchKernelGGL(P.hd4 ? k_gossip_apply_h4 : k_gossip_apply, dim3(h->apply_blocks), dim3(APPLY_THREADS),
                               h->apply_lds, s, P);
        });
        timed(h, 7, "k_finalize", [&] { hipLaunchKernelGGL(k_finalize, dim3(gL), dim3(256), 0, s, P); });
        if (h->n_leaving) hipLaunchKernelGGL(k_leave_stop, dim3(gL), dim3(256), 0, s, P);
        h->pc = PC_R_C;
        if (commit_begin(h, P, x, &rc, nloc)) return SWIM_OK;
        if (rc) return rc;
        break;
      case PC_R_C:
        if (SH && (rc = commit_end(h, P, x))) return rc;
        h->q++;
        h->pc = h->q < G ? PC_R_MAX : PC_SUSP;
        break;
      case PC_SUSP:  // phase G+1: suspicion timeouts
        set_phase(h, P, G + 1);
        timed(h, 7, "k_due", [&] { hipLaunchKernelGGL(k_due, dim3(1), dim3(1024), 0, s, P); });
        timed(h, 3, "k_susp_sweep", [&] { hipLaunchKernelGGL(k_susp_sweep, dim3(2048), dim3(256), 0, s, P); });
        timed(h, 7, "k_finalize", [&] { hipLaunchKernelGGL(k_finalize, dim3(gL), dim3(256), 0, s, P); });
        // phase G+2: SYNC requests
        set_phase(h, P, G + 2);
        // (stage_count and xs_cnt were reset by k_due, recv_count / recv_fill by k_susp_sweep)
        if (P.tmode)  // the touched columns this period's SYNC payloads carry
          timed(h, 7, "k_tlist", [&] { hipLaunchKernelGGL(k_tlist, dim3(1), dim3(1024), 0, s, P); });
        timed(h, 7, "k_sync_select", [&] { hipLaunchKernelGGL(k_sync_select, dim3(gL), dim3(256), 0, s, P); });
        if (P.njoin) hipLaunchKernelGGL(k_join_select, dim3(blocks_for(N, 256)), dim3(256), 0, s, P);
        timed(h, 6, "k_sync_snapshot", [&] { hipLaunchKernelGGL(k_sync_snapshot, dim3(1024), dim3(256), 0, s, P); });
        h->pc = PC_SYNC_REQ;
        if (SH) {  // tables of requesters whose receiver lives on another shard (row cells RL: k_xstatus)
          xchg_clear(x, SWIM_X_ALLTOALLV, W);
          XsArgs a{};
          a.kind = XS_SYNC;
          a.cap = h->scap;
          a.tmode = P.tmode;
          a.N = N;
          a.rl_dense = P.W;
          return xready(h, P, x, a);
        }
        break;
      case PC_SYNC_REQ: {
        uint32_t n_rec = 0;
        if (SH) {
          uint64_t words = 0;
          for (uint32_t q = 0; q < W; ++q) words += x->recv_counts[q];
          n_rec = (uint32_t)(words / (RL + 2u));
          if (n_rec > h->scap) return fail(h, SWIM_EOVERFLOW, "SYNC exchange over sync_capacity");
          P.xrecv = reinterpret_cast<const uint32_t*>(h->xrecv);
          P.xsend = reinterpret_cast<uint32_t*>(h->xsend);
          if (n_rec) hipLaunchKernelGGL(k_sync_unpack, dim3(blocks_for(n_rec, 256)), dim3(256), 0, s, P, n_rec);
        }
        timed(h, 7, "k_scan", [&] {
          const uint32_t nt = blocks_for(N, SCAN_TILE);
          hipLaunchKernelGGL(k_scan_tiles, dim3(nt), dim3(1024), 0, s, P, h->d_scan);
          hipLaunchKernelGGL(k_excl_scan, dim3(1), dim3(CS_THREADS), 0, s, h->d_scan, h->d_scan + nt, nt);
          hipLaunchKernelGGL(k_scan_apply, dim3(nt), dim3(1024), 0, s, P, h->d_scan + nt, nt);
        });
        timed(h, 7, "k_sync_scatter", [&] {
          hipLaunchKernelGGL(k_sync_scatter, dim3(blocks_for(2ull * nloc, 256)), dim3(256), 0, s, P);
        });
        if (n_rec) hipLaunchKernelGGL(k_sync_scatter_remote, dim3(blocks_for(n_rec, 256)), dim3(256), 0, s, P, n_rec);
        if (P.njoin) hipLaunchKernelGGL(k_join_scatter, dim3(blocks_for(N, 256)), dim3(256), 0, s, P);
        timed(h, 4, "k_sync_merge", [&] { hipLaunchKernelGGL(k_sync_merge, dim3(std::min(nloc, SY_GRID)), dim3(256), 0, s, P); });
        timed(h, 7, "k_finalize", [&] { hipLaunchKernelGGL(k_finalize, dim3(gL), dim3(256), 0, s, P); });
        h->pc = PC_SYNC_ACK;
        if (SH) {  // SYNC_ACK tables back to the requesters' shards, in the order received
          uint64_t back[SWIM_MAX_WORLD];
          for (uint32_t q = 0; q < W; ++q) back[q] = x->recv_counts[q];
          xchg_clear(x, SWIM_X_ALLTOALLV, W);
          for (uint32_t q = 0; q < W; ++q) x->send_counts[q] = back[q];
          HIPC(h, xorder(h));
          h->xknown = XK_ACK;
          return SWIM_OK;
        }
        break;
      }
      case PC_SYNC_ACK:  // phase G+3: SYNC_ACK
        set_phase(h, P, G + 3);
        if (SH) {
          uint64_t words = 0;
          for (uint32_t q = 0; q < W; ++q) words += x->recv_counts[q];
          const uint32_t n_rec = (uint32_t)(words / (RL + 2u));
          P.xrecv = reinterpret_cast<const uint32_t*>(h->xrecv);
          if (n_rec) hipLaunchKernelGGL(k_sync_ack_unpack, dim3(blocks_for(n_rec, 256)), dim3(256), 0, s, P, n_rec);
        }
        timed(h, 5, "k_sync_ack", [&] { hipLaunchKernelGGL(k_sync_ack, dim3(std::min(nloc, SY_GRID)), dim3(256), 0, s, P); });
        timed(h, 7, "k_finalize", [&] { hipLaunchKernelGGL(k_finalize, dim3(gL), dim3(256), 0, s, P); });
        h->pc = PC_END;  // the SYNC and SYNC_ACK gossips (both created at round (t+1)G)
        // (no host-side bound: SYNC merges re-spread what they accept. After a quiet period's rounds the
        // batch is small or empty, so it is sorted by the single-launch chain, k_rs_fused, which walks
        // any number of tiles on its CS_FUSE workgroups, instead of the eleven launches sized for the
        // stage's capacity: steady65k ten launches fewer per period)
        if (commit_begin(h, P, x, &rc, NONE, h->period_quiet)) return SWIM_OK;
        if (rc) return rc;
        break;
      case PC_END: {
        if (SH && (rc = commit_end(h, P, x))) return rc;
        if (P.hd4) {  // escape entries of swept / rewritten slots become tombstones
          memset_ctl_u32(h, offsetof(Ctl, hx_live));
          timed(h, 7, "k_hx_sweep", [&] { hipLaunchKernelGGL(k_hx_sweep, dim3(1024), dim3(256), 0, s, P); });
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return fail(h, SWIM_EHIP, std::string("kernel launch: ") + hipGetErrorString(e));
        if (h->base.njoin) {  // the joins of this period are complete
          HIPC(h, hipMemsetAsync(h->base.joining, 0, N, s));
          h->base.njoin = 0;
        }
        h->period++;
        h->pc = PC_FD;
        xchg_clear(x, SWIM_X_DONE, W);
        return SWIM_OK;
      }
    }
  }
}

int step_one(swim_handle* h) {
  swim_xchg x;
  int rc = period_resume(h, &x);
  if (rc) return rc;
  return x.op == SWIM_X_DONE ? SWIM_OK : fail(h, SWIM_EINVAL, "sharded handle: use swim_shard_step");
}

int check_overflow(swim_handle* h) {
  uint32_t ov = 0, why = 0;
  HIPC(h, hipMemcpyAsync(&ov, &h->base.ctl->overflow, 4, hipMemcpyDeviceToHost, h->stream));
  HIPC(h, hipMemcpyAsync(&why, &h->base.ctl->ov_detail, 4, hipMemcpyDeviceToHost, h->stream));
  HIPC(h, hipStreamSynchronize(h->stream));
  if (ov) {
    char buf[512];
    std::snprintf(buf, sizeof buf,
                  "simulator buffer overflow mask 0x%x (1 events, 2 gossip slots, 4 sync staging, 8 apply spill list, "
                  "16 sync bucket, 32 invariant, 64 infectedFrom bookkeeping, 128 N x K columns, 256 infection-round "
                  "escape table); infectedFrom "
                  "detail 0x%x (1 misprediction, 2 records per pair, 4 pruned pairs, 8 delivery records, 16 in-history)",
                  ov, why);
    return fail(h, SWIM_EOVERFLOW, buf);
  }
  return SWIM_OK;
}

// ---- library-driven exchanges ---------------------------------------------
// The library-owned RCCL communicator as a transport: collectives on the handle's stream
int rccl_allgather(void* ctx, const void* send, void* recv, uint64_t bytes, void* stream) {
  swim_handle* h = static_cast<swim_handle*>(ctx);
  return ncclAllGather(send, recv, bytes, ncclUint8, h->comm, static_cast<hipStream_t>(stream)) == ncclSuccess ? 0 : -1;
}
int rccl_alltoallv(void* ctx, const void* send, const uint64_t* sb, void* recv, const uint64_t* rb, void* stream) {
  swim_handle* h = static_cast<swim_handle*>(ctx);
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint64_t so = 0, ro = 0;
  if (ncclGroupStart() != ncclSuccess) return -1;
  bool ok = true;
  for (uint32_t q = 0; q < h->world && ok; ++q) {
    if (sb[q] && ncclSend(static_cast<const uint8_t*>(send) + so, sb[q], ncclUint8, (int)q, h->comm, s) != ncclSuccess)
      ok = false;
    if (ok && rb[q] && ncclRecv(static_cast<uint8_t*>(recv) + ro, rb[q], ncclUint8, (int)q, h->comm, s) != ncclSuccess)
      ok = false;
    so += sb[q];
    ro += rb[q];
  }
  const bool ended = ncclGroupEnd() == ncclSuccess;  // (the group is closed on every path)
  return ok && ended ? 0 : -1;
}

// One all-gather of n bytes per rank through the transport (send / recv: device buffers)
// A collective that failed on this rank leaves its peers inside theirs: the library-owned communicator
// is aborted (ncclCommAbort), so this rank's later calls fail at once instead of posting into a broken
// group, and the peers' RCCL calls return an error or time out (RCCL has no cross-rank notification; a
// host transport's own timeout, e.g. gloo's, ends the peers' wait there).
int tr_broken(swim_handle* h, const char* what) {
  if (h->comm) {
    (void)ncclCommAbort(h->comm);
    h->comm = nullptr;
    h->has_tr = false;
  }
  return fail(h, SWIM_ERCCL, what);
}

int tr_allgather(swim_handle* h, const void* send, void* recv, uint64_t n) {
  if (!h->tr.host_staged) {
    if (h->tr.allgather(h->tr.ctx, send, recv, n, h->stream))
      return tr_broken(h, "shard exchange: all-gather failed");
    return SWIM_OK;
  }
  const uint64_t W = h->world;
  if (h->hsend.size() < n) h->hsend.resize(n);
  HIPC(h, hipMemcpyAsync(h->hsend.data(), send, n, hipMemcpyDeviceToHost, h->stream));
  HIPC(h, hipStreamSynchronize(h->stream));
  if (h->hrecv.size() < W * n) h->hrecv.resize(W * n);  // (after the last copy out of it has completed)
  if (h->tr.allgather(h->tr.ctx, h->hsend.data(), h->hrecv.data(), n, nullptr))
    return fail(h, SWIM_ERCCL, "shard exchange: all-gather failed");
  HIPC(h, hipMemcpyAsync(recv, h->hrecv.data(), W * n, hipMemcpyHostToDevice, h->stream));
  return SWIM_OK;
}

int tr_alltoallv(swim_handle* h, const uint64_t* sb, const uint64_t* rb) {
  if (!h->tr.host_staged) {
    if (h->tr.alltoallv(h->tr.ctx, h->xsend, sb, h->xrecv, rb, h->stream))
      return tr_broken(h, "shard exchange: all-to-all-v failed");
    return SWIM_OK;
  }
  uint64_t st = 0, rt = 0;
  for (uint32_t q = 0; q < h->world; ++q) {
    st += sb[q];
    rt += rb[q];
  }
  if (h->hsend.size() < st) h->hsend.resize(st);
  if (st) HIPC(h, hipMemcpyAsync(h->hsend.data(), h->xsend, st, hipMemcpyDeviceToHost, h->stream));
  HIPC(h, hipStreamSynchronize(h->stream));
  // (grown only now: the last exchange's copy to the device out of it has completed)
  if (h->hrecv.size() < rt) h->hrecv.resize(rt);
  if (h->tr.alltoallv(h->tr.ctx, h->hsend.data(), sb, h->hrecv.data(), rb, nullptr))
    return fail(h, SWIM_ERCCL, "shard exchange: all-to-all-v failed");
  if (rt) HIPC(h, hipMemcpyAsync(h->xrecv, h->hrecv.data(), rt, hipMemcpyHostToDevice, h->stream));
  return SWIM_OK;
}

// The status all-gather every exchange starts with: row = {error code, op | swim_leave calls << 32,
// send words / counts}. Every rank learns every rank's counts (an all-to-all-v needs them before the
// data moves) and every error: a failure one rank detects fails all of them at the same exchange,
// never a hang. The leave count rides along because it sets the layout of every commit block (a
// {gossips, stopped} header once any member left): ranks that disagree fail instead of misreading.
int tr_status(swim_handle* h, int code, const swim_xchg& x, std::vector<uint64_t>* rows) {
  const uint32_t W = h->world, R = XS_CNT + W;
  // (the resume point too: ranks that took different branches of a period fail here, "out of step")
  const uint64_t op = code ? ~0ull : ((uint64_t)h->n_leaving << 32 | (uint64_t)(uint32_t)h->pc << 8 | x.op);
  uint64_t* row = h->xp->xrow;  // (free here: xready's read-back serves host-driven exchanges only)
  if (!code && h->xpend) {  // k_xstatus wrote the rest of the row
    h->xp->head[0] = 0;
    h->xp->head[1] = op;
    HIPC(h, hipMemcpyAsync(h->d_status, h->xp->head, 16, hipMemcpyHostToDevice, h->stream));
  } else {
    h->xpend = XS_NONE;
    for (uint32_t i = 0; i < R; ++i) row[i] = 0ull;
    row[0] = (uint64_t)(int64_t)code;
    row[1] = op;
    if (!code && x.op == SWIM_X_ALLGATHER) row[XS_CNT] = x.send_words;
    if (!code && x.op == SWIM_X_ALLTOALLV)
      for (uint32_t q = 0; q < W; ++q) row[XS_CNT + q] = x.send_counts[q];
    HIPC(h, hipMemcpyAsync(h->d_status, row, 8ull * R, hipMemcpyHostToDevice, h->stream));
  }
  int rc = tr_allgather(h, h->d_status, h->d_status + R, 8ull * R);
  if (rc) return rc;
  HIPC(h, hipMemcpyAsync(h->xp->rows, h->d_status + R, 8ull * W * R, hipMemcpyDeviceToHost, h->stream));
  HIPC(h, hipStreamSynchronize(h->stream));
  rows->assign(h->xp->rows, h->xp->rows + (size_t)W * R);
  return SWIM_OK;
}

// The rows of an exchange whose counts the last status rows give (tr_period): XK_NEED after the
// registrations (rank a sends rank b one need bitmap of nneed_a words per pair b registered with a:
// rows[b][XS_CNT + a] / 2 pairs, nneed_a from a's active-list length, rows[a][XS_A0]); XK_ACK after the
// SYNC requests (rank a sends rank b back what it received from b: the transposed counts).
void known_rows(swim_handle* h, uint32_t known, std::vector<uint64_t>* rows) {
  const uint32_t W = h->world, R = XS_CNT + W;
  std::vector<uint64_t>& v = *rows;
  std::vector<uint64_t> cnt((size_t)W * W);
  for (uint32_t a = 0; a < W; ++a)
    for (uint32_t b = 0; b < W; ++b)
      cnt[(size_t)a * W + b] = known == XK_NEED ? v[(size_t)b * R + XS_CNT + a] / 2 * ((v[(size_t)a * R + XS_A0] + 31u) / 32u)
                                                : v[(size_t)b * R + XS_CNT + a];
  for (uint32_t a = 0; a < W; ++a)
    for (uint32_t b = 0; b < W; ++b) v[(size_t)a * R + XS_CNT + b] = cnt[(size_t)a * W + b];
}

// One period of a sharded handle with a transport: period_resume up to each exchange, the status
// all-gather, the collective, resume.
int tr_period(swim_handle* h) {
  const uint32_t W = h->world, R = XS_CNT + W;
  std::vector<uint64_t> rows;
  swim_xchg x;  // carries each exchange's receive counts into the resumed period
  xchg_clear(&x, SWIM_X_DONE, W);
  for (;;) {
    h->xpend = XS_NONE;
    h->xknown = XK_NONE;
    int rc = period_resume(h, &x);
    if (!rc && h->xknown != XK_NONE) {
      // The need bitmaps answer the registrations, and the SYNC_ACK tables the SYNC requests: every
      // rank's counts of these two exchanges follow from the status rows of the exchange before them
      // (nothing between them can fail on one rank alone: every rank's SYNC batch is checked against
      // its rank's capacity at the SYNC status), so they take no status all-gather and no host stop.
      known_rows(h, h->xknown, &rows);
      h->xknown = XK_NONE;
    } else {
      if (!rc && x.op == SWIM_X_DONE) {  // the period's end: every rank's overflow flag joins the status
        XsArgs a{};
        a.kind = XS_DONE;
        rc = xready(h, h->cur, &x, a);
      }
      const std::string mine = rc ? h->err : std::string();
      const uint32_t kind = h->xpend;
      const int src = tr_status(h, rc, x, &rows);
      if (src) return src;
      if (!rc && kind && rows[(size_t)h->rank * R + XS_ERR]) {
        h->xpend = XS_NONE;
        return xown_fail(h, kind);
      }
      for (uint32_t q = 0; q < W; ++q) {
        const uint64_t e = rows[(size_t)q * R] ? rows[(size_t)q * R] : rows[(size_t)q * R + XS_ERR];
        if (e) {
          h->xpend = XS_NONE;
          if (rc) return fail(h, rc, mine);
          return fail(h, (int)(int64_t)e, "shard exchange: rank " + std::to_string(q) + " failed");
        }
      }
      for (uint32_t q = 1; q < W; ++q) {
        if ((rows[(size_t)q * R + 1] >> 32) != (rows[1] >> 32))
          return fail(h, SWIM_EINVAL, "shard exchange: ranks disagree on swim_leave calls (rank " + std::to_string(q) + ")");
        if (rows[(size_t)q * R + 1] != rows[1]) return fail(h, SWIM_EINVAL, "shard exchange: ranks out of step");
      }
      if (kind == XS_SYNC)  // every rank's received SYNC batch within its sync_capacity (before the SYNC_ACK)
        for (uint32_t r = 0; r < W; ++r) {
          uint64_t in = 0;
          for (uint32_t q = 0; q < W; ++q) in += rows[(size_t)q * R + XS_CNT + r];
          if (in / (rows[(size_t)r * R + XS_A0] + 2u) > (rows[(size_t)r * R + XS_A1] >> 32))
            return fail(h, SWIM_EOVERFLOW, "SYNC exchange over sync_capacity on rank " + std::to_string(r));
        }
      if (h->xpend && (rc = xpost(h, &x, &rows[(size_t)h->rank * R]))) return rc;
    }
    if (x.op == SWIM_X_DONE) return SWIM_OK;
    if (x.op == SWIM_X_ALLGATHER) {
      uint64_t m = 0;
      for (uint32_t q = 0; q < W; ++q) m = std::max(m, rows[(size_t)q * R + XS_CNT]);
      if (m * W > h->xrecv_words) return fail(h, SWIM_EOVERFLOW, "shard exchange: all-gather over the receive buffer");
      if (m && (rc = tr_allgather(h, h->xsend, h->xrecv, 4ull * m))) return rc;
      for (uint32_t q = 0; q < W; ++q) x.recv_counts[q] = rows[(size_t)q * R + XS_CNT];
      x.recv_stride = m;
    } else if (x.op == SWIM_X_ALLTOALLV) {
      uint64_t sb[SWIM_MAX_WORLD], rb[SWIM_MAX_WORLD], vol = 0;
      for (uint32_t r = 0; r < W; ++r) {  // every rank checks every rank's volumes: all fail together
        uint64_t out = 0, in = 0;
        for (uint32_t q = 0; q < W; ++q) {
          out += rows[(size_t)r * R + XS_CNT + q];
          in += rows[(size_t)q * R + XS_CNT + r];
        }
        if (out > h->xsend_words || in > h->xrecv_words)
          return fail(h, SWIM_EOVERFLOW, "shard exchange over the buffer capacity on rank " + std::to_string(r));
        vol += out;
      }
      for (uint32_t q = 0; q < W; ++q) {
        sb[q] = 4ull * rows[(size_t)h->rank * R + XS_CNT + q];
        rb[q] = 4ull * rows[(size_t)q * R + XS_CNT + h->rank];
        x.recv_counts[q] = rb[q] / 4;
      }
      if (vol && (rc = tr_alltoallv(h, sb, rb))) return rc;
      x.recv_stride = vol;  // the global volume: 0 lets the library skip ahead
    } else {
      return fail(h, SWIM_EINVAL, "shard exchange: unknown op");
    }
  }
}

// the status rows (device) and the exchanges' pinned host words of a sharded handle
int status_buffers(swim_handle* h) {
  const uint32_t W = h->world, R = XS_CNT + W;
  int rc = SWIM_OK;
  if (!h->d_status && (rc = dalloc(h, &h->d_status, (size_t)(1 + W) * R))) return rc;
  if (!h->xp && hipHostMalloc(reinterpret_cast<void**>(&h->xp), sizeof(swim_handle::XPin), hipHostMallocDefault) != hipSuccess) {
    h->xp = nullptr;
    return fail(h, SWIM_ENOMEM, "hipHostMalloc(exchange words)");
  }
  return SWIM_OK;
}

// exchange buffers and the status rows of a handle that drives its own exchanges
int tr_buffers(swim_handle* h) {
  int rc = status_buffers(h);
  if (rc) return rc;
  if (!h->xsend) {
    uint64_t sw = 0, rw = 0;
    if ((rc = swim_shard_buffer_words(h, &sw, &rw))) return rc;
    uint32_t *a = nullptr, *b = nullptr;
    if ((rc = dalloc(h, &a, sw)) || (rc = dalloc(h, &b, rw))) return rc;
    h->xsend = a;
    h->xrecv = b;
    h->xsend_words = sw;
    h->xrecv_words = rw;
  }
  return SWIM_OK;
}

}  // namespace

extern "C" {

int swim_create(const swim_config* cfg, swim_handle** out) {
  if (!cfg || !out) return SWIM_EINVAL;
  *out = nullptr;
  const swim_config& c = *cfg;
  if (c.n_members < 2 || c.n_members > (1u << 20) || c.mode > 1 || c.n_initial > c.n_members ||
      (c.n_initial && c.n_initial < c.n_members && c.mode != 0) ||
      (c.mode == 1 && (c.tracked_subjects < 1 || c.tracked_subjects > c.n_members)) ||
      c.ping_interval_ms <= 0 ||
      c.gossip_interval_ms <= 0 || c.gossip_fanout < 1 || c.gossip_fanout > MAXF || c.ping_req_members < 0 ||
      c.ping_req_members > MAXK || c.sync_interval_ms <= 0 || c.gossip_repeat_mult < 0 || c.suspicion_mult < 0)
    return SWIM_EINVAL;
  const uint32_t world = c.shard_world ? c.shard_world : 1u;
  if (world > SWIM_MAX_WORLD || c.shard_rank >= world || c.n_members % world) return SWIM_EINVAL;
  // gossip ring: a multiple of 1,024 slots (64-slot chunks, 32-slot bitmap words in aligned quads);
  // a power of two masks ids, any other size takes them mod GC
  if (c.gossip_capacity && (c.gossip_capacity % 1024u || c.gossip_capacity > (1u << 28))) return SWIM_EINVAL;
  if (c.dict_subjects && ((c.dict_subjects & (c.dict_subjects - 1u)) || c.dict_subjects < 4u || c.dict_subjects > (1u << 20)))
    return SWIM_EINVAL;
  // one receiver's entry bitmap (dict_subjects bytes) plus its spill list must fit a workgroup's 160 KiB
  // of LDS: at most 131,072 blocks
  if (c.dict_subjects && 4ull * aw_words(c.dict_subjects) > 160ull * 1024u) {
    std::fprintf(stderr, "swim_create: dict_subjects %u needs %llu B of LDS per receiver (> 160 KiB; at most 131072)\n",
                 c.dict_subjects, 4ull * aw_words(c.dict_subjects));
    return SWIM_EINVAL;
  }
  // suspicion deadlines are u16 cells decoded within +-2^14 periods of the current one (swim_device.h,
  // dl_dec): the timeout, suspicionMult * bit_length(N) periods (ClusterMath.java:123-125), must stay
  // well inside that window (a 64-period margin for the phases a deadline is read in)
  if ((uint64_t)c.suspicion_mult * bitlen(c.n_members) + 64u >= (1u << 14)) {
    std::fprintf(stderr, "swim_create: suspicionMult %d x bit_length(%u) periods does not fit the u16 deadline "
                         "window (< %u periods)\n", c.suspicion_mult, c.n_members, (1u << 14) - 64u);
    return SWIM_EINVAL;
  }
  if ((c.infection_round_bits != 0u && c.infection_round_bits != 4u && c.infection_round_bits != 8u) ||
      c.gossip_batching > 1u ||
      (c.record_capacity && ((c.record_capacity & (c.record_capacity - 1)) || c.record_capacity < 1024u)))
    return SWIM_EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return SWIM_EHIP;
  if (c.device < 0 || c.device >= ndev) return SWIM_EINVAL;
  if (hipSetDevice(c.device) != hipSuccess) return SWIM_EHIP;

  swim_handle* h = new (std::nothrow) swim_handle();
  if (!h) return SWIM_ENOMEM;
  h->cfg = c;
  const uint32_t N = c.n_members;
  h->N = N;
  h->G = (uint32_t)std::max(1, c.ping_interval_ms / c.gossip_interval_ms);
  h->S = (uint32_t)std::max(1, c.sync_interval_ms / c.ping_interval_ms);
  h->TPP = h->G + 4;
  // default gossip ring: ~4 GiB of holdings (N x GC x 4 B), between 8 Ki and 256 Ki slots
  h->GC = c.gossip_capacity ? c.gossip_capacity
                            : std::max<uint32_t>(8192u, std::min<uint32_t>(262144u, pow2ceil((1ull << 30) / N + 1) / 2));
  // SYNC staging rows: at most one periodic doSync per member every S periods (staggered) plus
  // one FD-triggered SYNC per member per period (MPI:385-397), so N + ceil(N/S) never
  // overflows; the default takes that bound unless the two payload slabs (8 B per cell) would
  // exceed ~30 % of the device's free memory.
  if (c.sync_capacity) {
    h->scap = c.sync_capacity;
  } else {
    size_t free_b = 0, total_b = 0;
    (void)hipMemGetInfo(&free_b, &total_b);
    const uint64_t bound = (uint64_t)N + (N + h->S - 1) / h->S;
    const uint64_t fit = (uint64_t)(free_b * 0.30) / (8ull * (c.mode == 1 ? c.tracked_subjects : N));
    h->scap = (uint32_t)std::max<uint64_t>(64, std::min(bound, fit));
  }
  h->ecap = c.event_capacity;
  h->n0 = c.n_initial ? c.n_initial : N;
  h->started.assign(N, 0);
  std::fill(h->started.begin(), h->started.begin() + h->n0, 1);
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    return SWIM_EHIP;
  }

  KP& P = h->base;
  P.N = N;
  P.GC = h->GC;
  P.gpow2 = (h->GC & (h->GC - 1)) == 0 ? 1u : 0u;
  P.gmask = h->GC - 1;
  P.G = h->G;
  P.S = h->S;
  P.f = (uint32_t)c.gossip_fanout;
  P.kreq = (uint32_t)c.ping_req_members;
  P.rm = (uint32_t)c.gossip_repeat_mult;
  P.mult = (uint32_t)c.suspicion_mult;
  P.n_seeds = c.n_seeds;
  P.time_left_pos = (c.ping_interval_ms - c.ping_timeout_ms) > 0 ? 1u : 0u;
  // a holder with infection round inf still counts the gossip as held at the start of round
  // inf + sweep + 1 (sweepGossips runs after that round's sends, GossipProtocolImpl.java:150-153),
  // and sweep <= 2 * (rm * bitlen(N) + 1); expiry = inf + sweepmax bounds every holder.
  P.sweepmax = 2u * (P.rm * bitlen(N) + 1u) + 1u;
  // infectedFrom horizon: a delivery of round t can suppress sends up to round
  // t + 1 + gossipPeriodsToSpread
  P.hzn = P.rm * bitlen(N) + 1u;
  {  // apply's LDS table: >= 2 slots per possible distinct subject (N), at most the build's cap;
     // a smaller table lets two 1,024-thread workgroups share a CU
    uint32_t lg = 6;
    while (lg < HCAP_LOG && (1ull << lg) < 2ull * N) ++lg;
    P.apply_hlog = lg;
    const uint64_t pres_words = N <= 32u * PRES_WORDS ? (N + 31u) / 32u : 0u;
    h->apply_lds = 4ull * (2ull * (1ull << lg) + SPILL_CAP + (SWIM_APPLY_PAIR ? 2u : 1u) * pres_words);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c.device);
    h->split_rows = 16u * (uint32_t)std::max(1, cus);
    const uint32_t per_cu = h->apply_lds <= 72u * 1024u ? 2u : 1u;  // 160 KiB LDS, 2,048 threads per CU
    h->apply_blocks = (uint32_t)std::max(1, cus) * per_cu;
    // the batch-slot variant: one receiver per wave, up to AW_WAVES waves per workgroup, each with
    // its own entry bitmap (dict_subjects bytes); as many workgroups per CU as the 160 KiB of LDS
    // (and 2,048 threads) allow
    P.dsids = c.dict_subjects ? c.dict_subjects : DICT_SIDS;
    const uint64_t wave_lds = 4ull * aw_words(P.dsids);
    h->apply_waves_b = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(AW_WAVES, (160ull * 1024u) / wave_lds));
    h->apply_lds_b = wave_lds * h->apply_waves_b;
    const uint32_t per_cu_b = std::max<uint32_t>(
        1, std::min<uint32_t>(2048 / (64 * h->apply_waves_b), (uint32_t)((160u * 1024u) / h->apply_lds_b)));
    h->apply_blocks_b = (uint32_t)std::max(1, cus) * per_cu_b;
    // the dynamic LDS each apply instance launches with (checked: a refused size fails here, not at
    // the first step)
    hipError_t lds_rc = hipSuccess;
    auto lds_attr = [&lds_rc](const void* k, uint64_t bytes) {
      const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
      if (e != hipSuccess && lds_rc == hipSuccess) lds_rc = e;
    };
    for (const void* k : {reinterpret_cast<const void*>(&k_gossip_apply), reinterpret_cast<const void*>(&k_gossip_apply_h4)})
      lds_attr(k, h->apply_lds);
    for (const void* k : {reinterpret_cast<const void*>(&k_gossip_apply_b), reinterpret_cast<const void*>(&k_gossip_apply_b_h4),
                          reinterpret_cast<const void*>(&k_gossip_apply_b16),
                          reinterpret_cast<const void*>(&k_gossip_apply_b16_h4)})
      lds_attr(k, h->apply_lds_b);
    lds_attr(reinterpret_cast<const void*>(&k_slot_bm), P.dsids);
    if (lds_rc != hipSuccess) {
      std::fprintf(stderr, "swim_create: dynamic LDS of the apply kernels refused (%s; apply %llu B, batched %llu B)\n",
                   hipGetErrorString(lds_rc), (unsigned long long)h->apply_lds, (unsigned long long)h->apply_lds_b);
      free_all(h);
      delete h;
      return SWIM_EHIP;
    }
  }
  if (P.sweepmax + P.hzn + 1u >= 256u) {  // infection rounds are kept mod 2^8 (swim_device.h, hd)
    std::fprintf(stderr, "swim_create: gossipRepeatMult %u too large for N=%u (sweep %u + horizon %u rounds > 254)\n",
                 P.rm, N, P.sweepmax, P.hzn);
    free_all(h);
    delete h;
    return SWIM_EINVAL;
  }
  P.ecap = h->ecap;
  P.scap = h->scap;
  P.seed = c.seed;
  h->world = world;
  h->rank = c.shard_rank;
  h->sharded = world > 1;
  P.world = world;
  P.rank = c.shard_rank;
  P.nloc = N / world;
  P.row0 = c.shard_rank * P.nloc;
  P.nxk = c.mode == 1 ? 1u : 0u;
  P.W = P.nxk ? c.tracked_subjects : N;  // cells per view row
  P.blx = nullptr;
  // gossip records: batch slots keep their gossips in a ring of their own; a phase stages at most
  // as many gossips as can be live (the commit raises OV_GOSSIP beyond the ring)
  h->CC = c.record_capacity ? c.record_capacity
                            : std::min<uint32_t>(1u << 24, std::max<uint32_t>(1u << 21, pow2ceil(4ull * h->GC)));
  P.cmask = h->CC - 1u;
  P.batch_commit = c.gossip_batching == 0 ? 1u : 0u;  // no loss set yet
  P.batched = 0u;  // set by the first batch commit (swim_api: commit_sorted)
  P.stg_cap = h->CC;
  P.loss_mode = 0;
  P.loss_thr = 0;
  // message delays: off until swim_set_delay
  P.delay_on = 0;
  P.dthr = nullptr;
  P.dthr_n = 0;
  P.dq = nullptr;
  P.dq_head = nullptr;
  P.dq_rhead = nullptr;
  P.dqcap = 0;
  P.dq_live = 0;
  P.gint = (uint32_t)c.gossip_interval_ms;
  P.pto = (uint32_t)std::max(0, c.ping_timeout_ms);
  P.pint = (uint32_t)std::max(0, c.ping_interval_ms);
  P.mto = (uint32_t)std::max(0, c.metadata_timeout_ms);
  P.link = nullptr;
  P.inlink = nullptr;
  P.rerouted = 0;
  P.njoin = 0;

  const size_t NN = (size_t)P.nloc * P.W;  // this shard's rows
  const size_t NL = P.nloc;
  int rc = SWIM_OK;
  uint8_t* group = nullptr;
#define ALLOC(ptr, count)                       \
  if (rc == SWIM_OK) rc = dalloc(h, &(ptr), (count));
  ALLOC(P.view, NN);
  ALLOC(P.dl, NN);
  {  // spill table: room for every (row, cell) at load 1/2 (what the dense inbox held) up to 2^25 slots
     // (16 B each: <= 512 MiB); a round that spills more keys than that raises OV_SPILL
    const uint32_t spc = pow2ceil(std::min<uint64_t>(1ull << 25, std::max<uint64_t>(1ull << 16, 2ull * NN)));
    ALLOC(P.sp_key, spc);
    ALLOC(P.sp_val, spc);
    ALLOC(P.sp_used, spc);
    P.spmask = spc - 1u;
    uint32_t* nl = nullptr;
    ALLOC(nl, N);
    P.none_last = nl;
  }
  ALLOC(P.hb, NL * (h->GC / 32));
  ALLOC(P.wb, NL * (h->GC / 32));
  // infection rounds: 8 bits per (member, slot), or 4-bit offsets + the escape table
  P.hd4 = c.infection_round_bits == 4u || (c.infection_round_bits == 0u && NL * (uint64_t)h->GC > (96ull << 30));
  ALLOC(P.hd, P.hd4 ? NL * h->GC / 2 : NL * h->GC);
  P.gc8 = nullptr;
  P.hx = nullptr;
  P.hxmask = 0;
  if (P.hd4) {
    uint8_t* g8 = nullptr;
    ALLOC(g8, h->GC);
    P.gc8 = g8;
    // 256 entries per local row, 2^20 .. 2^27 (8 B each: <= 1 GiB)
    const uint32_t hxcap = pow2ceil(std::min<uint64_t>(1ull << 27, std::max<uint64_t>(1ull << 20, NL * 256ull)));
    ALLOC(P.hx, hxcap);
    P.hxmask = hxcap - 1u;
  }
  ALLOC(P.mm, NL * (h->GC / 32));
  ALLOC(P.colmin, P.W);
  // touched columns (dense views without spare slots: every other column is BASELINE in every row)
  P.tmode = (!P.nxk && h->n0 == N && N % 32u == 0u) ? 1u : 0u;
  if (P.tmode) {
    ALLOC(P.tbits, N / 32);
    ALLOC(P.tlist, N);
  }
  if (P.nxk) {
    ALLOC(P.colmap, N);
    ALLOC(P.colsubj, P.W);
    ALLOC(P.colorder, P.W);
    ALLOC(P.track_req, N);
    P.tcap = std::min<uint32_t>(N, TRACK_SORT);
    ALLOC(P.track_list, P.tcap);
  }
  ALLOC(P.cnt, N);
  ALLOC(P.cnt_delta, N);
  ALLOC(P.alive, N);
  ALLOC(P.leaving, N);
  ALLOC(P.stopf, N);
  ALLOC(P.stop_list, NL);
  ALLOC(P.leave_slot, N);
  ALLOC(P.addr, N);
  ALLOC(P.occ, N);
  ALLOC(P.mv_head, N);
  ALLOC(P.mv_next, N);
  ALLOC(P.joining, N);
  ALLOC(P.jslot, N);
  ALLOC(P.jwin, N);
  ALLOC(P.jsend, N);
  ALLOC(P.jack_ref, N);
  ALLOC(group, N);
  ALLOC(P.fd_epoch, N);
  ALLOC(P.fd_cursor, N);
  ALLOC(P.g_epoch, N);
  ALLOC(P.g_cursor, N);
  ALLOC(P.gseq, N);
  ALLOC(P.fseq, N);
  ALLOC(P.sync_fd, N);
  ALLOC(P.peers, (size_t)N * c.gossip_fanout);
  ALLOC(P.npeers, N);
  ALLOC(P.g_sr, h->GC);
  ALLOC(P.g_hash, h->GC);
  ALLOC(P.g_cref, h->GC);
  ALLOC(P.c_sr, h->CC);
  ALLOC(P.c_hash, h->CC);
  h->dict_on = c.gossip_batching == 0;
  if (h->dict_on) {
    // 16-bit entry ids while every id (dict_subjects x 8 ways) and the two sentinels fit (else 32-bit)
    P.cid16 = (P.dsids * DICT_WAYS <= 65536u) ? 1u : 0u;
    if (P.cid16) {
      ALLOC(P.c_id16, h->CC);
      ALLOC(P.g_sid, h->GC);
    } else {
      ALLOC(P.c_id, h->CC);
    }
    ALLOC(P.sid_of, N);
    ALLOC(P.d_subj, P.dsids);
    ALLOC(P.d_rec, (size_t)P.dsids * DICT_WAYS);
    ALLOC(P.d_last, (size_t)P.dsids * DICT_WAYS);
    ALLOC(P.d_free, P.dsids);
    ALLOC(P.d_gen, P.dsids);
    ALLOC(P.dmark, NL * P.dsids);
    // slot entry bitmaps of long record ranges (k_slot_bm), a ring of RB_CAP of dsids bytes each
    P.rb_cap = RB_CAP;
    if (P.rb_cap) {
      ALLOC(P.rb_bits, (size_t)P.rb_cap * (P.dsids / 4u));
      ALLOC(P.rb_tag, P.rb_cap);
      ALLOC(P.g_rb, h->GC);
    }
  }
  ALLOC(P.wsum, h->GC / 32);
  ALLOC(P.scnt, h->GC);
  ALLOC(P.g_create, h->GC);
  ALLOC(P.nb, NL * (h->GC / 32));
  P.nsumw = std::min<uint32_t>(NSUM, std::max<uint32_t>(1u, h->GC / 1024u));
  ALLOC(P.nsum, NL * P.nsumw);
  ALLOC(P.lack, NL * P.nsumw);
  ALLOC(P.lack_round, N);
  ALLOC(P.stg, P.stg_cap);
  ALLOC(P.xg_pend, 2ull * world * NL * c.gossip_fanout);
  ALLOC(P.xs_pend, 2ull * world * NL);
  ALLOC(P.rs_ref, 2ull * N);
  ALLOC(P.ack_ref, 2ull * N);
  ALLOC(h->d_xcounts, SWIM_MAX_WORLD + 1);
  ALLOC(P.runw, h->GC / 32);
  if (world > 1) {
    const size_t pin = (size_t)(N - P.nloc) * c.gossip_fanout, pout = NL * c.gossip_fanout, nw = h->GC / 1024;
    ALLOC(P.rpairs, 2 * pin);
    ALLOC(P.rneed, pin * nw);
    ALLOC(P.rpref, pin * nw);
    ALLOC(P.rtot, pin);
    ALLOC(P.roff, pin);
    ALLOC(P.wcnt, pout + 1);
    ALLOC(P.woff, pout + 1);
    if (rc == SWIM_OK) (void)hipMemsetAsync(P.wcnt, 0, (pout + 1) * 4, h->stream);
  }
  for (int k = 0; k < 2; ++k) {
    ALLOC(h->ck[k], (size_t)P.stg_cap * world);
    ALLOC(h->cv[k], (size_t)P.stg_cap * world);
  }
  h->cs_maxt = (uint32_t)((P.stg_cap * (uint64_t)world + CS_TILE - 1) / CS_TILE);
  ALLOC(h->cs_ghist, CS_MAXPASS * 256);
  ALLOC(h->cs_ctr, CS_MAXPASS + 1);
  ALLOC(h->cs_stat, (size_t)CS_MAXPASS * h->cs_maxt * 256);
  ALLOC(h->d_blx, 2);
  ALLOC(P.wlast, h->GC / 32);
  ALLOC(P.in_cnt, N);
  ALLOC(P.in_list, (size_t)N * INCAP);
  ALLOC(P.in_ov, 2ull * N * c.gossip_fanout);
  ALLOC(P.alist, 2ull * N);
  P.astride = h->GC / 32 + 8;  // + a quad of slack: k_gossip_select reads the list 16 B at a time
  ALLOC(P.act_ring, 256ull * P.astride);
  P.act = P.act_ring;
  ALLOC(P.actpos, h->GC / 32);
  ALLOC(P.held, N);
  ALLOC(P.due, N);
  ALLOC(P.events, std::max<uint32_t>(1, h->ecap));
  ALLOC(P.pres, N);
  ALLOC(P.last_removed, N);
  ALLOC(P.meta_cur, N);
  P.meta_view = nullptr;  // allocated by the first swim_update_metadata
  ALLOC(P.req_to, 2ull * N);
  ALLOC(P.req_stage, 2ull * N);
  ALLOC(P.stage_req, h->scap);
  ALLOC(P.stage_sync, (size_t)h->scap * P.W);
  ALLOC(P.stage_ack, (size_t)h->scap * P.W);
  ALLOC(P.recv_count, N);
  ALLOC(P.recv_off, N + 1ull);
  ALLOC(P.recv_fill, N);
  ALLOC(P.bucket, 2ull * h->scap);  // local requests + requests received from other shards
  P.sy_cap = (uint32_t)((NL + SY_STRIPES - 1) / SY_STRIPES);  // SYNC work lists (sy_push)
  ALLOC(P.sy_mlist, (size_t)SY_STRIPES * P.sy_cap);
  ALLOC(P.sy_alist, (size_t)SY_STRIPES * P.sy_cap);
  {  // infectedFrom bookkeeping: in-history rings, delivery records, pruned pairs
    const uint64_t f = (uint64_t)c.gossip_fanout, W32 = h->GC / 32;
    // deliveries recorded per round: those whose receiver may select the sender within the
    // horizon (may_select's reach at a full view), x2 for margin
    const uint64_t reach = std::min<uint64_t>(N, (uint64_t)(P.hzn + 1) * f * 2 + 64 + 64);
    const uint64_t rec_round = std::max<uint64_t>(64, 2 * (uint64_t)P.nloc * f * reach / N);
    P.rcap = pow2ceil(std::max<uint64_t>(4096, rec_round * (P.hzn + 1)));
    P.bcap = pow2ceil(std::min<uint64_t>(1ull << 30, std::max<uint64_t>(1 << 16, P.rcap * std::max<uint64_t>(1, W32 / 2))));
    P.spcap = (uint32_t)std::max<uint64_t>(4096, std::min<uint64_t>((uint64_t)P.nloc * f, 65536));
    P.pwcap = (uint32_t)std::min<uint64_t>(1ull << 26, std::max<uint64_t>(1 << 16, (uint64_t)P.spcap * (W32 + 4)));
  }
  ALLOC(P.ih, NL * IHCAP);
  ALLOC(P.ih_head, N);
  ALLOC(P.ih_snd, NL * IHCAP);
  ALLOC(P.ih_rhead, NL * 256);
  ALLOC(P.dbg_send, 2ull * N);
  ALLOC(P.dbg_log, 256 * 8);
  ALLOC(P.rec_hdr, P.rcap);
  ALLOC(P.rec_len, P.rcap);
  ALLOC(P.rec_body, P.bcap);
  ALLOC(P.sp_list, P.spcap);
  ALLOC(P.sp_recs, (size_t)P.spcap * MAXREC);
  ALLOC(P.sp_dq, P.spcap);
  ALLOC(P.pw, P.pwcap);
  ALLOC(P.rp_list, P.spcap);
  ALLOC(P.ctl, 1);
  ALLOC(P.stat_shards, (size_t)STAT_SHARDS * STAT_STRIDE);
  ALLOC(h->d_digest, 2);
  ALLOC(h->d_scan, 2ull * ((N + SCAN_TILE - 1) / SCAN_TILE));
  ALLOC(h->d_quiet, 1);
#undef ALLOC
  if (rc == SWIM_OK && hipHostMalloc(reinterpret_cast<void**>(&h->h_quiet), 4, hipHostMallocDefault) != hipSuccess)
    rc = fail(h, SWIM_ENOMEM, "hipHostMalloc(4 B)");
  if (const char* e = std::getenv("SWIMHIP_QUIET")) h->quiet_skip = *e != '0';
  P.group = group;
  if (rc != SWIM_OK) {
    std::fprintf(stderr, "swim_create: %s\n", h->err.c_str());
    free_all(h);
    delete h;
    return rc;
  }
  hipStream_t s = h->stream;
  const uint32_t fill_blocks = 4096;
  // converged start: every view holds every member ALIVE incarnation 0 (MPI:139 + initial SYNC);
  // spare slots (ids >= n_initial) are in no view
  const uint32_t n0 = h->n0;
  if (n0 == N)
    hipLaunchKernelGGL(k_fill_u32, dim3(fill_blocks), dim3(256), 0, s, P.view, NN, SWIM_PACK(0, SWIM_ALIVE));
  else
    hipLaunchKernelGGL(k_init_rows, dim3(fill_blocks), dim3(256), 0, s, P.view, NN, P.W, n0);
  hipLaunchKernelGGL(k_iota_u32, dim3(blocks_for(N, 256)), dim3(256), 0, s, P.addr, N, N);
  hipLaunchKernelGGL(k_iota_u32, dim3(blocks_for(N, 256)), dim3(256), 0, s, P.occ, N, n0);
  hipLaunchKernelGGL(k_fill_u32, dim3(blocks_for(N, 256)), dim3(256), 0, s, P.mv_head, (size_t)N, NONE);
  hipLaunchKernelGGL(k_fill_u32, dim3(blocks_for(N, 256)), dim3(256), 0, s, P.mv_next, (size_t)N, NONE);
  (void)hipMemsetAsync(P.joining, 0, N, s);
  (void)hipMemsetAsync(P.dl, 0, NN * 2, s);
  (void)hipMemsetAsync(P.sp_key, 0, ((size_t)P.spmask + 1) * 8, s);
  (void)hipMemsetAsync(P.sp_val, 0, ((size_t)P.spmask + 1) * 4, s);
  (void)hipMemsetAsync(const_cast<uint32_t*>(P.none_last), 0, (size_t)N * 4, s);
  (void)hipMemsetAsync(P.hb, 0, NL * (h->GC / 32) * 4, s);
  (void)hipMemsetAsync(P.wb, 0, NL * (h->GC / 32) * 4, s);
  if (P.hd4) {
    (void)hipMemsetAsync(P.hd, 0, NL * (h->GC / 2), s);
    (void)hipMemsetAsync(const_cast<uint8_t*>(P.gc8), 0, h->GC, s);
    (void)hipMemsetAsync(P.hx, 0, ((size_t)P.hxmask + 1) * 8, s);
  }
  hipLaunchKernelGGL(k_fill_u32, dim3(blocks_for(P.W, 256)), dim3(256), 0, s, P.colmin, (size_t)P.W, NONE);
  if (P.tmode) (void)hipMemsetAsync(P.tbits, 0, (size_t)N / 8, s);
  if (P.nxk) {
    hipLaunchKernelGGL(k_fill_u32, dim3(blocks_for(N, 256)), dim3(256), 0, s, P.colmap, (size_t)N, NONE);
    (void)hipMemsetAsync(P.track_req, 0, (size_t)N * 4, s);
  }
  hipLaunchKernelGGL(k_fill_u32, dim3(blocks_for(N, 256)), dim3(256), 0, s, P.cnt, (size_t)N, n0 - 1);
  // presence is per shard: observers of this shard holding the subject (all but the subject itself).
  // The started members of this shard's rows are [row0, min(n0, row0 + nloc)); a subject of them is
  // held by all but itself, any other started subject by all of them, a spare slot by none
  const uint32_t ls = n0 > P.row0 ? std::min(n0, P.row0 + P.nloc) - P.row0 : 0u;  // started local rows
  (void)hipMemsetAsync(P.pres, 0, (size_t)N * 4, s);
  hipLaunchKernelGGL(k_fill_u32, dim3(blocks_for(n0, 256)), dim3(256), 0, s, P.pres, (size_t)n0, ls);
  if (ls) hipLaunchKernelGGL(k_fill_u32, dim3(blocks_for(ls, 256)), dim3(256), 0, s, P.pres + P.row0, (size_t)ls, ls - 1);
  hipLaunchKernelGGL(k_fill_u32, dim3(blocks_for(N, 256)), dim3(256), 0, s, P.sync_fd, (size_t)N, NONE);
  (void)hipMemsetAsync(P.cnt_delta, 0, (size_t)N * 4, s);
  (void)hipMemsetAsync(P.alive, 1, n0, s);
  if (n0 < N) (void)hipMemsetAsync(P.alive + n0, 0, N - n0, s);
  (void)hipMemsetAsync(P.leaving, 0, N, s);
  (void)hipMemsetAsync(P.stopf, 0, N, s);
  hipLaunchKernelGGL(k_fill_u32, dim3(blocks_for(N, 256)), dim3(256), 0, s, P.leave_slot, (size_t)N, NONE);
  (void)hipMemsetAsync(group, 0, N, s);
  (void)hipMemsetAsync(P.fd_epoch, 0, (size_t)N * 4, s);
  (void)hipMemsetAsync(P.fd_cursor, 0, (size_t)N * 4, s);
  (void)hipMemsetAsync(P.g_epoch, 0, (size_t)N * 4, s);
  (void)hipMemsetAsync(P.g_cursor, 0, (size_t)N * 4, s);
  (void)hipMemsetAsync(P.gseq, 0, (size_t)N * 4, s);
  (void)hipMemsetAsync(P.fseq, 0, (size_t)N * 4, s);
  (void)hipMemsetAsync(P.in_cnt, 0, (size_t)N * 4, s);
  (void)hipMemsetAsync(P.nb, 0, NL * (h->GC / 32) * 4, s);
  (void)hipMemsetAsync(P.g_create, 0, (size_t)h->GC * 4, s);
  (void)hipMemsetAsync(P.last_removed, 0, (size_t)N * 4, s);
  (void)hipMemsetAsync(P.meta_cur, 0, (size_t)N * 4, s);
  (void)hipMemsetAsync(P.ctl, 0, sizeof(Ctl), s);
  if (h->dict_on) {
    (void)hipMemsetAsync(P.sid_of, 0xFF, (size_t)N * 4, s);
    (void)hipMemsetAsync(P.d_subj, 0xFF, (size_t)P.dsids * 4, s);
    (void)hipMemsetAsync(P.d_rec, 0, (size_t)P.dsids * DICT_WAYS * 4, s);
    (void)hipMemsetAsync(P.d_last, 0, (size_t)P.dsids * DICT_WAYS * 4, s);
    hipLaunchKernelGGL(k_fill_u32, dim3(blocks_for(P.dsids, 256)), dim3(256), 0, s, P.d_gen, (size_t)P.dsids, 1u);
    (void)hipMemsetAsync(P.dmark, 0, NL * P.dsids * 4, s);
    if (P.rb_cap) {
      (void)hipMemsetAsync(P.rb_tag, 0xFF, (size_t)P.rb_cap * 4, s);
      (void)hipMemsetAsync(P.g_rb, 0xFF, (size_t)h->GC * 4, s);
    }
  }
  (void)hipMemsetAsync(P.wlast, 0, (size_t)(h->GC / 32) * 4, s);
  (void)hipMemsetAsync(P.runw, 0, (size_t)(h->GC / 32) * 4, s);
  (void)hipMemsetAsync(P.g_cref, 0, (size_t)h->GC * 8, s);
  (void)hipMemsetAsync(P.wsum, 0, (size_t)(h->GC / 32) * 4, s);
  (void)hipMemsetAsync(P.scnt, 0, (size_t)h->GC * 2, s);
  (void)hipMemsetAsync(P.held, 0, (size_t)N * 4, s);
  (void)hipMemsetAsync(P.ih_head, 0, (size_t)N * 4, s);
  (void)hipMemsetAsync(P.ih_rhead, 0, NL * 256 * 4, s);
  hipLaunchKernelGGL(k_fill_u32, dim3(blocks_for(N, 256)), dim3(256), 0, s, P.lack_round, (size_t)N, NONE);
  (void)hipMemsetAsync(P.dbg_send, 0, (size_t)N * 16, s);
  (void)hipMemsetAsync(P.dbg_log, 0, 256 * 8 * 4, s);
  {
    const char* w = std::getenv("SWIMHIP_DEBUG_WATCH");
    P.dbg_watch = w ? (uint32_t)std::strtoul(w, nullptr, 10) : NONE;
  }
  hipLaunchKernelGGL(k_fill_u32, dim3(64), dim3(256), 0, s, reinterpret_cast<uint32_t*>(P.actpos), (size_t)h->GC / 16,
                     NONE);
  {  // every started member of this shard starts with others = n0 - 1; n0 members alive
    const uint32_t all = ls, alive = ls;  // of this shard
    (void)hipMemcpyAsync(&P.ctl->bl_hist[bitlen(n0)], &all, 4, hipMemcpyHostToDevice, s);
    (void)hipMemcpyAsync(&P.ctl->alive_count, &alive, 4, hipMemcpyHostToDevice, s);
    (void)hipStreamSynchronize(s);
  }
  (void)hipMemsetAsync(P.stat_shards, 0, (size_t)STAT_SHARDS * STAT_STRIDE * 8, s);
  hipError_t e = hipStreamSynchronize(s);
  if (e == hipSuccess) e = hipGetLastError();
  if (e != hipSuccess) {
    std::fprintf(stderr, "swim_create: init failed: %s\n", hipGetErrorString(e));
    free_all(h);
    delete h;
    return SWIM_EHIP;
  }
  *out = h;
  return SWIM_OK;
}

int swim_destroy(swim_handle* h) {
  if (!h) return SWIM_EINVAL;
  if (h->stream) (void)hipStreamSynchronize(h->stream);
#ifdef SWIM_SEL_PROF
  {  // k_gossip_select phase profile (wall clock at 100 MHz, summed over waves)
    unsigned long long ph[12] = {};
    if (hipMemcpy(ph, h->base.dbg_log, sizeof ph, hipMemcpyDeviceToHost) == hipSuccess)
      std::fprintf(stderr, "select phases (wave-ms): holdings %.1f peers %.1f infectedFrom %.1f register %.1f\n",
                   ph[8] / 1e5, ph[9] / 1e5, ph[10] / 1e5, ph[11] / 1e5);
  }
#endif
#ifdef SWIM_APPLY_PROF
  {  // k_gossip_apply phase profile (wall clock at 100 MHz, summed over workgroups)
    unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpy(ph, h->base.dbg_log, sizeof ph, hipMemcpyDeviceToHost) == hipSuccess) {
      std::fprintf(stderr, "apply phases (workgroup-ms): init %.1f compact %.1f items %.1f subjects %.1f\n",
                   ph[0] / 1e5, ph[1] / 1e5, ph[2] / 1e5, ph[3] / 1e5);
      std::fprintf(stderr, "apply_b phases (wave-ms): bitmap init %.1f words+records %.1f merge %.1f spill %.1f\n",
                   ph[4] / 1e5, ph[5] / 1e5, ph[6] / 1e5, ph[7] / 1e5);
    }
    unsigned long long fw[20] = {};
    if (hipMemcpy(fw, h->base.dbg_log, sizeof fw, hipMemcpyDeviceToHost) == hipSuccess)
      std::fprintf(stderr, "apply_b receipt words received whole %llu of %llu; their records %llu of %llu\n", fw[14],
                   fw[15], fw[12], fw[13]);
    std::fprintf(stderr, "apply_b records in ranges of >= 64 records: %llu\n", fw[16]);
    std::fprintf(stderr, "apply_b words+records split (wave-ms): words %.1f long ranges %.1f short ranges %.1f\n",
                 fw[17] / 1e5, fw[18] / 1e5, fw[19] / 1e5);
  }
#endif
  free_all(h);
  delete h;
  return SWIM_OK;
}

int swim_set_loss(swim_handle* h, uint32_t loss_bp) {
  if (!h || loss_bp > 10000) return SWIM_EINVAL;
  KP& P = h->base;
  if (loss_bp > 0 && loss_bp < 10000 && P.batched) {
    // NetworkEmulator draws per message, i.e. per gossip: a live slot of several gossips would
    // have to split. Refuse loudly instead.
    uint32_t* d = reinterpret_cast<uint32_t*>(h->d_digest);  // scratch word
    HIPC(h, hipMemsetAsync(d, 0, 4, h->stream));
    hipLaunchKernelGGL(k_multi_live, dim3(256), dim3(256), 0, h->stream, P, d);
    uint32_t multi = 0;
    HIPC(h, hipMemcpyAsync(&multi, d, 4, hipMemcpyDeviceToHost, h->stream));
    HIPC(h, hipStreamSynchronize(h->stream));
    if (multi)
      return fail(h, SWIM_EINVAL,
                  "swim_set_loss: a probabilistic loss draws per gossip, but live ring slots hold batches of several "
                  "gossips (DESIGN.md 3.12): set the loss before they are created, or create with gossip_batching = 1");
  }
  if (loss_bp == 0) {
    P.loss_mode = 0;
  } else if (loss_bp >= 10000) {
    P.loss_mode = 2;
  } else {
    P.loss_mode = 1;
    P.loss_thr = (uint32_t)(((uint64_t)loss_bp << 32) / 10000u);
  }
  P.batch_commit = (h->cfg.gossip_batching == 0 && P.loss_mode != 1u && !P.delay_on) ? 1u : 0u;
  return SWIM_OK;
}

// NetworkEmulator.setDefaultOutboundSettings(loss, meanDelay) of every member, the delay part
// (NetworkEmulator.java:81-84,189-201,358-368). Each message draws an exponential
// delay of mean `mean_ms`: GossipRequests are handled delay / gossipInterval rounds later (a
// per-receiver ring of messages in flight), ping / ping-req / metadata round trips must come back
// within their timeouts. Delays draw per message, i.e. per gossip: like a probabilistic loss they
// need one gossip per ring slot. Unsharded handles; rings sized for test-scale clusters.
int swim_set_delay(swim_handle* h, uint32_t mean_ms) {
  if (!h || mean_ms > 60000) return SWIM_EINVAL;
  KP& P = h->base;
  if (h->pc != PC_FD) return fail(h, SWIM_EINVAL, "swim_set_delay: a period is in flight");
  if (mean_ms == 0) {  // new messages travel at once; those in flight still arrive (k_gossip_pull)
    P.delay_on = 0;
    P.batch_commit = (h->cfg.gossip_batching == 0 && P.loss_mode != 1u) ? 1u : 0u;
    return SWIM_OK;
  }
  if (P.batched) {  // the same refusal as a probabilistic loss
    uint32_t* d = reinterpret_cast<uint32_t*>(h->d_digest);
    HIPC(h, hipMemsetAsync(d, 0, 4, h->stream));
    hipLaunchKernelGGL(k_multi_live, dim3(256), dim3(256), 0, h->stream, P, d);
    uint32_t multi = 0;
    HIPC(h, hipMemcpyAsync(&multi, d, 4, hipMemcpyDeviceToHost, h->stream));
    HIPC(h, hipStreamSynchronize(h->stream));
    if (multi)
      return fail(h, SWIM_EINVAL,
                  "swim_set_delay: delays draw per gossip, but live ring slots hold batches of several gossips "
                  "(DESIGN.md 3.12): set the delay before they are created, or create with gossip_batching = 1");
  }
  // dthr[k] = ceil(2^32 (1 - exp(-k / mean))) for every k a 32-bit draw can reach (the oracle
  // computes the same table with the same expression). Built and checked on the host first: a
  // refused call leaves the handle exactly as it was (the live table, dq_live and the rings).
  std::vector<uint32_t> thr;
  for (uint32_t k = 0;; ++k) {
    const double t = std::ceil(std::ldexp(-std::expm1(-(double)k / (double)mean_ms), 32));
    if (t > 4294967295.0) break;
    thr.push_back((uint32_t)t);
  }
  // an entry matters until its message arrived and left the infectedFrom horizon: the per-round
  // head history (256 rounds) must reach that far back
  const uint32_t live = ((uint32_t)thr.size() - 1u) / P.gint + P.hzn + 1u;
  if (live >= 256u) return fail(h, SWIM_EINVAL, "swim_set_delay: delays this long (in gossip rounds) exceed the ring history");
  if (!P.dq && P.nloc > 65536u)
    return fail(h, SWIM_EINVAL, "swim_set_delay: the delayed-message rings are sized for clusters up to 65,536 members");
  if (!P.dq) {  // per receiver: messages in flight plus the arrived ones still inside the horizon
    // A receiver pushes up to (in-degree x window) entries per round and each stays up to dq_live
    // rounds: a 1 s mean on LAN (200 ms rounds, dq_live ~ 136 rounds) under 2 % loss at 256 members
    // pushes ~5e4 entries per receiver and round at its peak (every message of every window draws a
    // delay, held gossips included), and the exponential tail keeps some entries live for ~110
    // rounds. The ring takes the most entries per receiver (up to 2^23) that 1/16 of the free device
    // memory allows (SWIMHIP_DQCAP: a power of two instead); one that still wraps over a live entry
    // raises OV_IFROM (IF_DELAYQ).
    size_t free_b = 0, total_b = 0;
    (void)hipMemGetInfo(&free_b, &total_b);
    uint32_t cap = 1u << 23;
    while (cap > 4096u && (uint64_t)P.nloc * cap * 16u > free_b / 16u) cap >>= 1;
    if (const char* e = std::getenv("SWIMHIP_DQCAP")) {
      const unsigned long v = std::strtoul(e, nullptr, 10);
      if (v >= 64u && v <= (1ul << 26) && (v & (v - 1ul)) == 0ul) cap = (uint32_t)v;
    }
    uint4* dq = nullptr;
    uint32_t *head = nullptr, *rhead = nullptr;
    int rc = dalloc(h, &dq, (size_t)P.nloc * cap);
    if (!rc) rc = dalloc(h, &head, h->N);
    if (!rc) rc = dalloc(h, &rhead, (size_t)P.nloc * 256u);
    if (rc) return rc;
    HIPC(h, hipMemsetAsync(head, 0, (size_t)h->N * 4, h->stream));
    HIPC(h, hipMemsetAsync(rhead, 0, (size_t)P.nloc * 256u * 4, h->stream));
    P.dq = dq;
    P.dq_head = head;
    P.dq_rhead = rhead;
    P.dqcap = cap;
  }
  if (thr.size() > h->dthr_cap) {  // (a smaller earlier table stays allocated until swim_destroy)
    uint32_t* dt = nullptr;
    int rc = dalloc(h, &dt, thr.size());
    if (rc) return rc;
    P.dthr = dt;
    h->dthr_cap = (uint32_t)thr.size();
  }
  HIPC(h, hipMemcpyAsync(const_cast<uint32_t*>(P.dthr), thr.data(), thr.size() * 4, hipMemcpyHostToDevice, h->stream));
  P.dthr_n = (uint32_t)thr.size();
  P.dq_live = std::max(P.dq_live, live);  // entries pushed under an earlier, longer mean stay covered
  HIPC(h, hipStreamSynchronize(h->stream));
  P.delay_on = 1;
  P.batch_commit = 0;  // one gossip per slot while delays are on
  return SWIM_OK;
}

int swim_set_partition(swim_handle* h, const uint8_t* group, uint32_t n, uint64_t t0, uint64_t t1) {
  if (!h || !group || n != h->N) return SWIM_EINVAL;
  HIPC(h, hipMemcpyAsync(const_cast<uint8_t*>(h->base.group), group, n, hipMemcpyHostToDevice, h->stream));
  HIPC(h, hipStreamSynchronize(h->stream));
  h->part_t0 = t0;
  h->part_t1 = t1;
  return SWIM_OK;
}

namespace {
// flip one bit of a lazily allocated N x N bitmap on the device
int set_bitmap_bit(swim_handle* h, const uint8_t** field, uint64_t bit, int on) {
  const size_t bytes = ((size_t)h->N * h->N + 7) / 8;
  if (!*field) {
    uint8_t* l = nullptr;
    int rc = dalloc(h, &l, bytes);
    if (rc) return rc;
    HIPC(h, hipMemsetAsync(l, 0, bytes, h->stream));
    *field = l;
  }
  uint8_t byte = 0;
  uint8_t* dp = const_cast<uint8_t*>(*field) + (bit >> 3);
  HIPC(h, hipMemcpyAsync(&byte, dp, 1, hipMemcpyDeviceToHost, h->stream));
  HIPC(h, hipStreamSynchronize(h->stream));
  if (on)
    byte |= (uint8_t)(1u << (bit & 7));
  else
    byte &= (uint8_t) ~(1u << (bit & 7));
  HIPC(h, hipMemcpyAsync(dp, &byte, 1, hipMemcpyHostToDevice, h->stream));
  HIPC(h, hipStreamSynchronize(h->stream));
  return SWIM_OK;
}
}  // namespace

int swim_block_link(swim_handle* h, uint32_t src, uint32_t dst, int blocked) {
  if (!h || src >= h->N || dst >= h->N) return SWIM_EINVAL;
  return set_bitmap_bit(h, &h->base.link, (uint64_t)src * h->N + dst, blocked);
}

int swim_block_inbound(swim_handle* h, uint32_t dst, uint32_t src, int blocked) {
  if (!h || src >= h->N || dst >= h->N) return SWIM_EINVAL;
  return set_bitmap_bit(h, &h->base.inlink, (uint64_t)dst * h->N + src, blocked);
}

int swim_leave(swim_handle* h, const uint32_t* ids, uint32_t n) {
  if (!h || (n && !ids)) return SWIM_EINVAL;
  if (h->pc != PC_FD) return fail(h, SWIM_EINVAL, "swim_leave: a period is in flight");
  for (uint32_t k = 0; k < n; ++k)
    if (ids[k] >= h->N) return SWIM_EINVAL;
  for (uint32_t k = 0; k < n; ++k) {
    if (h->base.nxk) {  // the member's own record leaves the baseline: give it a column
      hipLaunchKernelGGL(k_track_one, dim3(1), dim3(64), 0, h->stream, h->base, ids[k]);
      track_commit(h, h->base);
    }
    hipLaunchKernelGGL(k_leave, dim3(1), dim3(64), 0, h->stream, h->base, ids[k]);
    h->host_staged += 1;
  }
  h->n_leaving += n;
  HIPC(h, hipStreamSynchronize(h->stream));
  HIPC(h, hipGetLastError());
  return SWIM_OK;
}

namespace {
// a spare slot x starts at address a (ClusterImpl.start): table = itself ALIVE inc 0, fresh cursors,
// initial SYNC to the seeds in this period's SYNC phase (k_join_select)
int start_member(swim_handle* h, uint32_t x, uint32_t a) {
  hipLaunchKernelGGL(k_join_one, dim3(1), dim3(256), 0, h->stream, h->base, x, a);
  h->started[x] = 1;
  h->base.njoin++;
  return SWIM_OK;
}

int join_checks(swim_handle* h, uint32_t n) {
  // (N x K views hold BASELINE for every untracked subject in every row: a joiner's table, which knows
  // only itself, is not one. Sharded handles: every rank makes the same call)
  if (h->base.nxk) return fail(h, SWIM_EINVAL, "join / restart: dense handles only");
  if (h->pc != PC_FD) return fail(h, SWIM_EINVAL, "join / restart: a period is in flight");
  const uint64_t seeds = std::min<uint64_t>(h->cfg.n_seeds, h->N);
  if ((uint64_t)(h->base.njoin + n) * std::max<uint64_t>(1, seeds) > h->scap)
    return fail(h, SWIM_EINVAL, "join / restart: too many initial SYNCs in one period for sync_capacity");
  return SWIM_OK;
}
}  // namespace

int swim_join(swim_handle* h, const uint32_t* ids, uint32_t n) {
  if (!h || (n && !ids)) return SWIM_EINVAL;
  int rc = join_checks(h, n);
  if (rc) return rc;
  std::vector<uint32_t> occ(h->N);
  HIPC(h, hipMemcpyAsync(occ.data(), h->base.occ, (size_t)h->N * 4, hipMemcpyDeviceToHost, h->stream));
  HIPC(h, hipStreamSynchronize(h->stream));
  for (uint32_t k = 0; k < n; ++k) {
    if (ids[k] >= h->N || h->started[ids[k]] || occ[ids[k]] != NONE)
      return fail(h, SWIM_EINVAL, "swim_join: not a free spare slot");
    for (uint32_t q = 0; q < k; ++q)
      if (ids[q] == ids[k]) return fail(h, SWIM_EINVAL, "swim_join: duplicate id");
  }
  for (uint32_t k = 0; k < n; ++k) start_member(h, ids[k], ids[k]);
  HIPC(h, hipStreamSynchronize(h->stream));
  HIPC(h, hipGetLastError());
  return SWIM_OK;
}

int swim_restart(swim_handle* h, const uint32_t* old_ids, const uint32_t* new_ids, uint32_t n) {
  if (!h || (n && (!old_ids || !new_ids))) return SWIM_EINVAL;
  int rc = join_checks(h, n);
  if (rc) return rc;
  const uint32_t N = h->N;
  std::vector<uint32_t> occ(N), addr(N);
  std::vector<uint8_t> alive(N);
  HIPC(h, hipMemcpyAsync(occ.data(), h->base.occ, (size_t)N * 4, hipMemcpyDeviceToHost, h->stream));
  HIPC(h, hipMemcpyAsync(addr.data(), h->base.addr, (size_t)N * 4, hipMemcpyDeviceToHost, h->stream));
  HIPC(h, hipMemcpyAsync(alive.data(), h->base.alive, N, hipMemcpyDeviceToHost, h->stream));
  HIPC(h, hipStreamSynchronize(h->stream));
  for (uint32_t k = 0; k < n; ++k) {
    const uint32_t o = old_ids[k], x = new_ids[k];
    if (o >= N || x >= N || !h->started[o] || alive[o] || h->started[x] || occ[addr[o]] != NONE)
      return fail(h, SWIM_EINVAL, "swim_restart: old id must be stopped with its address free, new id a spare slot");
    for (uint32_t q = 0; q < k; ++q)
      if (new_ids[q] == x || addr[old_ids[q]] == addr[o]) return fail(h, SWIM_EINVAL, "swim_restart: duplicate");
  }
  h->base.rerouted = 1;
  for (uint32_t k = 0; k < n; ++k) start_member(h, new_ids[k], addr[old_ids[k]]);
  HIPC(h, hipStreamSynchronize(h->stream));
  HIPC(h, hipGetLastError());
  return SWIM_OK;
}

int swim_crash(swim_handle* h, const uint32_t* ids, uint32_t n) {
  if (!h || (n && !ids)) return SWIM_EINVAL;
  std::vector<uint8_t> alive(h->N);
  HIPC(h, hipMemcpyAsync(alive.data(), h->base.alive, h->N, hipMemcpyDeviceToHost, h->stream));
  HIPC(h, hipStreamSynchronize(h->stream));
  for (uint32_t k = 0; k < n; ++k)
    if (ids[k] >= h->N) return SWIM_EINVAL;
  std::vector<uint32_t> down;  // the distinct members this call stops
  for (uint32_t k = 0; k < n; ++k) {
    const uint32_t c = ids[k];
    if (!alive[c]) continue;
    alive[c] = 0;
    down.push_back(c);
  }
  if (!down.empty()) {  // one launch for the whole set (k_crash_many)
    if (!h->crash_ids) {
      int rc = dalloc(h, &h->crash_ids, h->N);
      if (rc) return rc;
    }
    HIPC(h, hipMemcpyAsync(h->crash_ids, down.data(), down.size() * 4, hipMemcpyHostToDevice, h->stream));
    const uint32_t chunks = blocks_for(h->base.W, CRASH_PIECE);
    hipLaunchKernelGGL(k_crash_many, dim3((uint32_t)down.size() * chunks), dim3(256), 0, h->stream, h->base,
                       h->crash_ids, (uint32_t)down.size(), chunks);
  }
  HIPC(h, hipMemcpyAsync(h->base.alive, alive.data(), h->N, hipMemcpyHostToDevice, h->stream));
  HIPC(h, hipStreamSynchronize(h->stream));
  HIPC(h, hipGetLastError());
  return SWIM_OK;
}

int swim_update_metadata(swim_handle* h, const uint32_t* ids, uint32_t n) {
  if (!h || (n && !ids)) return SWIM_EINVAL;
  if (h->pc != PC_FD) return fail(h, SWIM_EINVAL, "swim_update_metadata: a period is in flight");
  for (uint32_t k = 0; k < n; ++k)
    if (ids[k] >= h->N) return SWIM_EINVAL;
  if (!h->base.meta_view) {  // first metadata change: every stored version is the initial one
    uint32_t* mv = nullptr;
    const size_t cells = (size_t)h->base.nloc * h->base.W;
    int rc = dalloc(h, &mv, cells);
    if (rc) return rc;
    HIPC(h, hipMemsetAsync(mv, 0, cells * 4, h->stream));
    h->base.meta_view = mv;
  }
  for (uint32_t k = 0; k < n; ++k) {
    if (h->base.nxk) {  // the member's own record leaves the baseline: give it a column
      hipLaunchKernelGGL(k_track_one, dim3(1), dim3(64), 0, h->stream, h->base, ids[k]);
      track_commit(h, h->base);
    }
    hipLaunchKernelGGL(k_update_meta, dim3(1), dim3(64), 0, h->stream, h->base, ids[k]);
    h->host_staged += 1;
  }
  HIPC(h, hipStreamSynchronize(h->stream));
  HIPC(h, hipGetLastError());
  return SWIM_OK;
}

int swim_spread(swim_handle* h, uint32_t origin, uint32_t tag) {
  if (!h || origin >= h->N) return SWIM_EINVAL;
  if (h->pc != PC_FD) return fail(h, SWIM_EINVAL, "swim_spread: a period is in flight");
  hipLaunchKernelGGL(k_spread, dim3(1), dim3(64), 0, h->stream, h->base, origin, tag);
  h->host_staged += 1;
  HIPC(h, hipStreamSynchronize(h->stream));
  HIPC(h, hipGetLastError());
  return SWIM_OK;
}

int swim_deliver_records(swim_handle* h, uint32_t observer, const uint32_t* subjects, const uint32_t* records,
                         uint32_t n, uint32_t reason) {
  if (!h || observer >= h->N || (n && (!subjects || !records))) return SWIM_EINVAL;
  const uint32_t base_reason = reason & ~SWIM_DELIVER_FORWARD;
  if (base_reason != SWIM_R_SYNC && base_reason != SWIM_R_MEMBERSHIP_GOSSIP && base_reason != SWIM_R_INITIAL_SYNC)
    return fail(h, SWIM_EINVAL, "swim_deliver_records: reason must be SYNC, INITIAL_SYNC or MEMBERSHIP_GOSSIP");
  if ((reason & SWIM_DELIVER_FORWARD) && base_reason != SWIM_R_MEMBERSHIP_GOSSIP)
    return fail(h, SWIM_EINVAL, "swim_deliver_records: SWIM_DELIVER_FORWARD goes with MEMBERSHIP_GOSSIP");
  for (uint32_t k = 0; k < n; ++k)
    if (subjects[k] >= h->N || records[k] == SWIM_ABSENT)
      return fail(h, SWIM_EINVAL, "swim_deliver_records: subject out of range or an absent record");
  if (h->pc != PC_FD) return fail(h, SWIM_EINVAL, "swim_deliver_records: a period is in flight");
  if (n == 0) return SWIM_OK;
  if (2ull * n > h->deliver_cap) {
    uint32_t* d = nullptr;
    int rc = dalloc(h, &d, 2ull * n);
    if (rc) return rc;
    h->deliver_buf = d;
    h->deliver_cap = 2u * n;
  }
  hipStream_t s = h->stream;
  HIPC(h, hipMemcpyAsync(h->deliver_buf, subjects, (size_t)n * 4, hipMemcpyHostToDevice, s));
  HIPC(h, hipMemcpyAsync(h->deliver_buf + n, records, (size_t)n * 4, hipMemcpyHostToDevice, s));
  KP P;
  set_phase(h, P, 0);  // the coming period: its deadlines, FD tick and first gossip round
  if (P.nxk) {  // every shard requests (and so allocates) the same columns
    hipLaunchKernelGGL(k_deliver_track, dim3(1), dim3(256), 0, s, P, h->deliver_buf, h->deliver_buf + n, n,
                       (reason & SWIM_DELIVER_FORWARD) ? 1u : 0u);
    track_commit(h, P);
  }
  hipLaunchKernelGGL(k_deliver, dim3(1), dim3(64), 0, s, P, observer, h->deliver_buf, h->deliver_buf + n, n, reason);
  h->host_staged += 2ull * n;  // (a forwarded copy and a spread per record at most)
  hipLaunchKernelGGL(k_finalize, dim3(blocks_for(P.nloc, 256)), dim3(256), 0, s, P);
  HIPC(h, hipStreamSynchronize(s));
  HIPC(h, hipGetLastError());
  return SWIM_OK;
}

int swim_trace(swim_handle* h, uint32_t mask) {
  if (!h || (mask & ~SWIM_TRACE_FD)) return SWIM_EINVAL;
  h->base.trace = mask;
  return SWIM_OK;
}

int swim_step_async(swim_handle* h, uint32_t periods) {
  if (!h) return SWIM_EINVAL;
  if (h->sharded && !h->has_tr)
    return fail(h, SWIM_EINVAL, "sharded handle: attach a transport (swim_shard_comm_init) or use swim_shard_step");
  for (uint32_t p = 0; p < periods; ++p) {
    int rc = h->sharded ? tr_period(h) : step_one(h);
    if (rc) return rc;
  }
  return SWIM_OK;
}

int swim_sync(swim_handle* h) {
  if (!h) return SWIM_EINVAL;
  HIPC(h, hipStreamSynchronize(h->stream));
  resolve_timing(h);
  return check_overflow(h);
}

int swim_step(swim_handle* h, uint32_t periods) {
  int rc = swim_step_async(h, periods);
  if (rc) return rc;
  return swim_sync(h);
}

int swim_drain_events(swim_handle* h, swim_event* buf, uint64_t cap, uint64_t* n_out) {
  if (!h || !n_out) return SWIM_EINVAL;
  uint32_t cnt = 0;
  HIPC(h, hipMemcpyAsync(&cnt, &h->base.ctl->event_count, 4, hipMemcpyDeviceToHost, h->stream));
  HIPC(h, hipStreamSynchronize(h->stream));
  if (!buf && cap == 0) {  // count and discard: a consumer that only counts (bench.py's converge window)
    HIPC(h, hipMemsetAsync(&h->base.ctl->event_count, 0, 4, h->stream));
    HIPC(h, hipStreamSynchronize(h->stream));
    *n_out = std::min(cnt, h->ecap);
    if (cnt > h->ecap) return fail(h, SWIM_EOVERFLOW, "event buffer overflow");
    return SWIM_OK;
  }
  const uint32_t have = std::min(cnt, h->ecap);
  std::vector<swim_event> ev(have);
  if (have) HIPC(h, hipMemcpyAsync(ev.data(), h->base.events, (size_t)have * sizeof(swim_event), hipMemcpyDeviceToHost, h->stream));
  HIPC(h, hipMemsetAsync(&h->base.ctl->event_count, 0, 4, h->stream));
  HIPC(h, hipStreamSynchronize(h->stream));
  std::sort(ev.begin(), ev.end(), [](const swim_event& a, const swim_event& b) {
    if (a.period != b.period) return a.period < b.period;
    if (a.observer != b.observer) return a.observer < b.observer;
    if (a.phase != b.phase) return a.phase < b.phase;
    if (a.subject != b.subject) return a.subject < b.subject;
    if (a.type != b.type) return a.type < b.type;
    if (a.reason != b.reason) return a.reason < b.reason;
    return a.record < b.record;
  });
  const uint64_t n = std::min<uint64_t>(cap, ev.size());
  if (n && buf) std::memcpy(buf, ev.data(), n * sizeof(swim_event));
  *n_out = n;
  if (cnt > h->ecap || ev.size() > cap) return fail(h, SWIM_EOVERFLOW, "event buffer overflow");
  return SWIM_OK;
}

namespace {
// N x K: the allocated columns' subjects (host copy)
int tracked_columns(swim_handle* h, std::vector<uint32_t>* subj) {
  uint32_t nc = 0;
  HIPC(h, hipMemcpyAsync(&nc, &h->base.ctl->ncols, 4, hipMemcpyDeviceToHost, h->stream));
  HIPC(h, hipStreamSynchronize(h->stream));
  nc = std::min(nc, h->base.W);
  subj->resize(nc);
  if (nc) HIPC(h, hipMemcpyAsync(subj->data(), h->base.colsubj, (size_t)nc * 4, hipMemcpyDeviceToHost, h->stream));
  HIPC(h, hipStreamSynchronize(h->stream));
  return SWIM_OK;
}
}  // namespace

int swim_read_view(swim_handle* h, uint32_t observer, uint32_t* row, uint32_t n) {
  if (!h || !row || observer - h->base.row0 >= h->base.nloc || n != h->N) return SWIM_EINVAL;
  const size_t lr = observer - h->base.row0;
  if (!h->base.nxk) {
    HIPC(h, hipMemcpyAsync(row, h->base.view + lr * h->N, (size_t)n * 4, hipMemcpyDeviceToHost, h->stream));
    HIPC(h, hipStreamSynchronize(h->stream));
    return SWIM_OK;
  }
  std::vector<uint32_t> subj, cells;
  int rc = tracked_columns(h, &subj);
  if (rc) return rc;
  cells.resize(subj.size());
  if (!subj.empty())
    HIPC(h, hipMemcpyAsync(cells.data(), h->base.view + lr * h->base.W, subj.size() * 4, hipMemcpyDeviceToHost,
                           h->stream));
  HIPC(h, hipStreamSynchronize(h->stream));
  std::fill(row, row + n, BASELINE);  // untracked subjects: the converged record
  for (size_t c = 0; c < subj.size(); ++c) row[subj[c]] = cells[c];
  return SWIM_OK;
}

int swim_read_deadlines(swim_handle* h, uint32_t observer, uint32_t* row, uint32_t n) {
  if (!h || !row || observer - h->base.row0 >= h->base.nloc || n != h->N) return SWIM_EINVAL;
  // cell-major u16 storage: strided 2D copy of one observer column, decoded at the coming period
  // (the absolute deadline + 1, as the oracle keeps it)
  const uint32_t t = (uint32_t)h->period;
  std::vector<uint32_t> subj;
  if (h->base.nxk) {
    int rc = tracked_columns(h, &subj);
    if (rc) return rc;
  }
  const size_t ncol = h->base.nxk ? subj.size() : h->N;
  if (!h->d_rowbuf) {
    int rc = dalloc(h, &h->d_rowbuf, h->N);
    if (rc) return rc;
  }
  std::vector<uint32_t> cells(ncol);
  if (ncol) {
    hipLaunchKernelGGL(k_read_dl, dim3(blocks_for(ncol, 256)), dim3(256), 0, h->stream, h->base,
                       observer - h->base.row0, t, h->d_rowbuf, (uint32_t)ncol);
    HIPC(h, hipMemcpyAsync(cells.data(), h->d_rowbuf, ncol * 4, hipMemcpyDeviceToHost, h->stream));
  }
  HIPC(h, hipStreamSynchronize(h->stream));
  std::fill(row, row + n, 0u);
  for (size_t c = 0; c < ncol; ++c) row[h->base.nxk ? subj[c] : c] = cells[c];
  return SWIM_OK;
}

int swim_digest(swim_handle* h, uint64_t* vd, uint64_t* dd) {
  if (!h) return SWIM_EINVAL;
  HIPC(h, hipMemsetAsync(h->d_digest, 0, 16, h->stream));
  KP Q = h->base;
  Q.period = (uint32_t)h->period;  // deadlines decode at the coming period (dl_dec)
  hipLaunchKernelGGL(k_digest, dim3(4096), dim3(256), 0, h->stream, Q, h->d_digest);
  unsigned long long out[2];
  HIPC(h, hipMemcpyAsync(out, h->d_digest, 16, hipMemcpyDeviceToHost, h->stream));
  HIPC(h, hipStreamSynchronize(h->stream));
  if (vd) *vd = out[0];
  if (dd) *dd = out[1];
  return SWIM_OK;
}

namespace {
// presence per subject; N x K keeps it only for tracked subjects: an untracked one is held by
// every alive observer but itself
int presence_host(swim_handle* h, std::vector<uint32_t>* pres, std::vector<uint8_t>* alive) {
  const uint32_t N = h->N;
  pres->resize(N);
  alive->resize(N);
  HIPC(h, hipMemcpyAsync(pres->data(), h->base.pres, (size_t)N * 4, hipMemcpyDeviceToHost, h->stream));
  HIPC(h, hipMemcpyAsync(alive->data(), h->base.alive, N, hipMemcpyDeviceToHost, h->stream));
  if (h->base.nxk) {
    std::vector<uint32_t> colmap(N);
    uint32_t alive_count = 0;
    HIPC(h, hipMemcpyAsync(colmap.data(), h->base.colmap, (size_t)N * 4, hipMemcpyDeviceToHost, h->stream));
    HIPC(h, hipMemcpyAsync(&alive_count, &h->base.ctl->alive_count, 4, hipMemcpyDeviceToHost, h->stream));
    HIPC(h, hipStreamSynchronize(h->stream));
    for (uint32_t j = 0; j < N; ++j)  // alive_count: alive observers of this shard
      if (colmap[j] == NONE) (*pres)[j] = alive_count - (((*alive)[j] && j - h->base.row0 < h->base.nloc) ? 1u : 0u);
  }
  HIPC(h, hipStreamSynchronize(h->stream));
  return SWIM_OK;
}
}  // namespace

int swim_read_presence(swim_handle* h, uint32_t* present, uint32_t* last_removed, uint32_t n) {
  if (!h || n != h->N) return SWIM_EINVAL;
  if (present) {
    std::vector<uint32_t> pres;
    std::vector<uint8_t> alive;
    int rc = presence_host(h, &pres, &alive);
    if (rc) return rc;
    std::memcpy(present, pres.data(), (size_t)n * 4);
  }
  if (last_removed)
    HIPC(h, hipMemcpyAsync(last_removed, h->base.last_removed, (size_t)n * 4, hipMemcpyDeviceToHost, h->stream));
  HIPC(h, hipStreamSynchronize(h->stream));
  return SWIM_OK;
}

int swim_stats_get(swim_handle* h, swim_stats* out) {
  if (!h || !out) return SWIM_EINVAL;
  Ctl ctl;
  HIPC(h, hipMemcpyAsync(&ctl, h->base.ctl, sizeof ctl, hipMemcpyDeviceToHost, h->stream));
  std::vector<uint32_t> pres;
  std::vector<uint8_t> alive;
  int prc = presence_host(h, &pres, &alive);
  if (prc) return prc;
  std::vector<unsigned long long> shards((size_t)STAT_SHARDS * STAT_STRIDE);
  HIPC(h, hipMemcpyAsync(shards.data(), h->base.stat_shards, shards.size() * 8, hipMemcpyDeviceToHost, h->stream));
  HIPC(h, hipStreamSynchronize(h->stream));
  unsigned long long stats[ST_COUNT] = {0};
  for (uint32_t sh = 0; sh < STAT_SHARDS; ++sh)
    for (int i = 0; i < ST_COUNT; ++i) stats[i] += shards[(size_t)sh * STAT_STRIDE + i];
  std::memset(out, 0, sizeof *out);
  out->period = h->period;
  out->fd_probes = stats[ST_FD_PROBES];
  out->fd_direct_ok = stats[ST_FD_DIRECT_OK];
  out->fd_ping_req = stats[ST_FD_PING_REQ];
  out->fd_suspect_events = stats[ST_FD_SUSPECT_EV];
  out->fd_alive_events = stats[ST_FD_ALIVE_EV];
  out->gossips_created = stats[ST_GOSSIPS_CREATED];
  out->gossip_first_receipts = stats[ST_GOSSIP_RECEIPTS];
  out->gossip_sends = stats[ST_GOSSIP_SENDS] - stats[ST_GOSSIP_SUPP];
  out->syncs_sent = stats[ST_SYNCS_SENT];
  out->syncs_delivered = stats[ST_SYNCS_DELIVERED];
  out->sync_acks_delivered = stats[ST_ACKS_DELIVERED];
  out->records_accepted = stats[ST_ACCEPTED];
  out->events_added = stats[ST_ADDED];
  out->events_removed = stats[ST_REMOVED];
  out->suspicion_timeouts = stats[ST_SUSP_TIMEOUTS];
  out->refutations = stats[ST_REFUTATIONS];
  out->overflow = ctl.overflow;
  out->gossip_scanned = stats[ST_G_SCANNED];
  out->gossip_probes = stats[ST_G_PROBES];
  out->sweep_cells = stats[ST_SWEEP_CELLS];
  out->merge_cells = stats[ST_MERGE_CELLS];
  out->ack_cells = stats[ST_ACK_CELLS];
  out->live_gossip_slots = ctl.gcount - ctl.glo;
  out->gossip_hd_words = stats[ST_G_HDREAD];
  out->gossip_window_words = stats[ST_G_WINW];
  out->gossip_pull_words = stats[ST_G_PULLW];
  out->infected_pruned_pairs = stats[ST_IF_PAIRS];
  out->infected_records = stats[ST_IF_RECORDS];
  out->infected_suppressed = stats[ST_GOSSIP_SUPP];
  out->apply_words = stats[ST_APPLY_WORDS];
  out->apply_runs = stats[ST_APPLY_RUNS];
  out->apply_subjects = stats[ST_APPLY_SUBJ];
  out->fd_dead_events = stats[ST_FD_DEAD_EV];
  out->apply_spills = stats[ST_APPLY_SPILL];
  out->apply_records = stats[ST_APPLY_RECS];
  out->events_updated = stats[ST_UPDATED];
  out->apply_pairs = stats[ST_APPLY_PAIRS];
  out->commit_radix = stats[ST_COMMIT_RADIX];
  out->apply_skipped = stats[ST_APPLY_SKIP];
  out->apply_bitmaps = stats[ST_APPLY_RBM];
  out->quiet_periods = h->quiet_periods;
  out->apply_bitmap_records = stats[ST_APPLY_RBREC];
  out->escape_entries = ctl.hx_live;
  out->escape_capacity = h->base.hd4 ? (uint64_t)h->base.hxmask + 1u : 0u;
  {  // gossips in the live slots: the record ring from the oldest live slot's first record
    uint32_t c_lo = ctl.ccount;
    if (ctl.gcount != ctl.glo && ctl.gcount - ctl.glo <= h->GC) {
      uint2 cr;
      HIPC(h, hipMemcpy(&cr, h->base.g_cref + (ctl.glo % h->GC), 8, hipMemcpyDeviceToHost));
      c_lo = cr.x;
    }
    out->live_gossip_records = ctl.ccount - c_lo;
  }
  uint64_t nc = 0;
  for (uint32_t j = 0; j < h->N; ++j)
    if (!alive[j]) nc += pres[j];
  out->not_converged = nc;
  return SWIM_OK;
}

const char* swim_last_error(swim_handle* h) { return h ? h->err.c_str() : "null handle"; }

int swim_kat_is_overrides(const uint32_t* r1, const uint32_t* r0, uint8_t* out, uint64_t n) {
  if (!r1 || !r0 || !out) return SWIM_EINVAL;
  if (n == 0) return SWIM_OK;
  uint32_t *d1 = nullptr, *d0 = nullptr;
  uint8_t* dout = nullptr;
  if (hipMalloc(&d1, n * 4) != hipSuccess || hipMalloc(&d0, n * 4) != hipSuccess || hipMalloc(&dout, n) != hipSuccess)
    return SWIM_EHIP;
  int rc = SWIM_OK;
  if (hipMemcpy(d1, r1, n * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(d0, r0, n * 4, hipMemcpyHostToDevice) != hipSuccess)
    rc = SWIM_EHIP;
  if (rc == SWIM_OK) {
    hipLaunchKernelGGL(k_kat_overrides, dim3(blocks_for(n, 256)), dim3(256), 0, 0, d1, d0, dout, n);
    if (hipMemcpy(out, dout, n, hipMemcpyDeviceToHost) != hipSuccess) rc = SWIM_EHIP;
  }
  (void)hipFree(d1);
  (void)hipFree(d0);
  (void)hipFree(dout);
  return rc;
}

int swim_kat_philox(uint64_t seed, uint32_t kind, const uint32_t* abct, uint32_t* out, uint64_t n) {
  if (!abct || !out) return SWIM_EINVAL;
  if (n == 0) return SWIM_OK;
  uint32_t *din = nullptr, *dout = nullptr;
  if (hipMalloc(&din, n * 16) != hipSuccess || hipMalloc(&dout, n * 4) != hipSuccess) return SWIM_EHIP;
  int rc = SWIM_OK;
  if (hipMemcpy(din, abct, n * 16, hipMemcpyHostToDevice) != hipSuccess) rc = SWIM_EHIP;
  if (rc == SWIM_OK) {
    hipLaunchKernelGGL(k_kat_philox, dim3(blocks_for(n, 256)), dim3(256), 0, 0, seed, kind, din, dout, n);
    if (hipMemcpy(out, dout, n * 4, hipMemcpyDeviceToHost) != hipSuccess) rc = SWIM_EHIP;
  }
  (void)hipFree(din);
  (void)hipFree(dout);
  return rc;
}

int swim_kat_philox4(uint64_t seed, uint32_t kind, const uint32_t* abct, uint32_t* out4, uint64_t n) {
  if (!abct || !out4) return SWIM_EINVAL;
  if (n == 0) return SWIM_OK;
  uint32_t *din = nullptr, *dout = nullptr;
  if (hipMalloc(&din, n * 16) != hipSuccess || hipMalloc(&dout, n * 16) != hipSuccess) return SWIM_EHIP;
  int rc = SWIM_OK;
  if (hipMemcpy(din, abct, n * 16, hipMemcpyHostToDevice) != hipSuccess) rc = SWIM_EHIP;
  if (rc == SWIM_OK) {
    hipLaunchKernelGGL(k_kat_philox4, dim3(blocks_for(n, 256)), dim3(256), 0, 0, seed, kind, din, dout, n);
    if (hipMemcpy(out4, dout, n * 16, hipMemcpyDeviceToHost) != hipSuccess) rc = SWIM_EHIP;
  }
  (void)hipFree(din);
  (void)hipFree(dout);
  return rc;
}

int swim_kat_scan(const uint32_t* in, uint64_t n, uint32_t* wave_excl, uint32_t* wave_tot, uint32_t* block_excl,
                  uint32_t* block_tot) {
  if (!in || !wave_excl || !wave_tot || !block_excl || !block_tot || n % 1024u) return SWIM_EINVAL;
  if (n == 0) return SWIM_OK;
  uint32_t *din = nullptr, *dwe = nullptr, *dwt = nullptr, *dbe = nullptr, *dbt = nullptr;
  int rc = SWIM_OK;
  if (hipMalloc(&din, n * 4) != hipSuccess || hipMalloc(&dwe, n * 4) != hipSuccess ||
      hipMalloc(&dwt, n / 16) != hipSuccess || hipMalloc(&dbe, n * 4) != hipSuccess ||
      hipMalloc(&dbt, n / 256) != hipSuccess)
    rc = SWIM_EHIP;
  if (rc == SWIM_OK && hipMemcpy(din, in, n * 4, hipMemcpyHostToDevice) != hipSuccess) rc = SWIM_EHIP;
  if (rc == SWIM_OK) {
    hipLaunchKernelGGL(k_kat_scan, dim3((uint32_t)(n / 1024)), dim3(1024), 0, 0, din, dwe, dwt, dbe, dbt);
    if (hipMemcpy(wave_excl, dwe, n * 4, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(wave_tot, dwt, n / 16, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(block_excl, dbe, n * 4, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(block_tot, dbt, n / 256, hipMemcpyDeviceToHost) != hipSuccess)
      rc = SWIM_EHIP;
  }
  for (uint32_t* p : {din, dwe, dwt, dbe, dbt})
    if (p) (void)hipFree(p);
  return rc;
}

int swim_debug_holdings(swim_handle* h, uint32_t member, uint32_t* out_hash, uint32_t* out_inf, uint32_t cap,
                        uint32_t* n_out) {
  if (!h || member - h->base.row0 >= h->base.nloc || !n_out) return SWIM_EINVAL;
  const size_t lr = member - h->base.row0;
  Ctl ctl;
  HIPC(h, hipMemcpyAsync(&ctl, h->base.ctl, sizeof ctl, hipMemcpyDeviceToHost, h->stream));
  HIPC(h, hipStreamSynchronize(h->stream));
  const uint32_t GC = h->GC, CC = h->CC;
  std::vector<uint32_t> bits(GC / 32), ch(CC);
  std::vector<uint2> cref(GC);
  std::vector<uint8_t> d(GC);
  HIPC(h, hipMemcpy(bits.data(), h->base.hb + lr * (GC / 32), (size_t)GC / 8, hipMemcpyDeviceToHost));
  if (!h->base.hd4) {
    HIPC(h, hipMemcpy(d.data(), h->base.hd + lr * GC, (size_t)GC, hipMemcpyDeviceToHost));
  } else {  // 4-bit offsets from the slots' creation rounds, 15 = in the escape table
    std::vector<uint8_t> nib(GC / 2), g8(GC);
    std::vector<unsigned long long> hx((size_t)h->base.hxmask + 1);
    HIPC(h, hipMemcpy(nib.data(), h->base.hd + lr * (GC / 2), (size_t)GC / 2, hipMemcpyDeviceToHost));
    HIPC(h, hipMemcpy(g8.data(), h->base.gc8, (size_t)GC, hipMemcpyDeviceToHost));
    HIPC(h, hipMemcpy(hx.data(), h->base.hx, hx.size() * 8, hipMemcpyDeviceToHost));
    for (uint32_t s = 0; s < GC; ++s) {
      const uint32_t o = (nib[s >> 1] >> (4u * (s & 1u))) & 0xFu;
      d[s] = (uint8_t)(g8[s] + o);
      if (o == 15u) {
        const unsigned long long key = 1ull + (unsigned long long)lr * GC + s;
        for (const unsigned long long v : hx)
          if (v != HX_EMPTY && v != HX_TOMB && (v >> 8) == key) d[s] = (uint8_t)(v & 0xFFu);
      }
    }
  }
  HIPC(h, hipMemcpy(cref.data(), h->base.g_cref, (size_t)GC * 8, hipMemcpyDeviceToHost));
  HIPC(h, hipMemcpy(ch.data(), h->base.c_hash, (size_t)CC * 4, hipMemcpyDeviceToHost));
  uint32_t lo = ctl.glo, hi = ctl.gcount, n = 0;
  const uint32_t rnow = (uint32_t)(h->period * h->G);  // next round to run
  if (hi - lo > GC) lo = hi - GC;
  for (uint32_t id = lo; id < hi; ++id) {
    const uint32_t s = id % GC;
    if (!((bits[s >> 5] >> (s & 31)) & 1u)) continue;
    for (uint32_t x = cref[s].x; x != cref[s].y; ++x) {  // every gossip of the slot's batch
      if (n < cap) {
        out_hash[n] = ch[x & (CC - 1)];
        out_inf[n] = rnow - (uint8_t)(rnow - d[s]);  // hd = infection round mod 2^8, age < 2^8
      }
      ++n;
    }
  }
  *n_out = n;
  return SWIM_OK;
}

int swim_debug_member_state(swim_handle* h, uint32_t* out6n, uint32_t n) {
  if (!h || !out6n || n != h->N) return SWIM_EINVAL;
  uint32_t* src[6] = {h->base.fd_epoch, h->base.fd_cursor, h->base.g_epoch, h->base.g_cursor, h->base.gseq,
                      h->base.cnt};
  for (int k = 0; k < 6; ++k)
    HIPC(h, hipMemcpyAsync(out6n + (size_t)k * n, src[k], (size_t)n * 4, hipMemcpyDeviceToHost, h->stream));
  HIPC(h, hipStreamSynchronize(h->stream));
  return SWIM_OK;
}

int swim_debug_sends(swim_handle* h, uint64_t* out2n, uint32_t n) {
  if (!h || !out2n || n != h->N) return SWIM_EINVAL;
  HIPC(h, hipMemcpyAsync(out2n, h->base.dbg_send, (size_t)n * 16, hipMemcpyDeviceToHost, h->stream));
  HIPC(h, hipStreamSynchronize(h->stream));
  if (h->base.dbg_watch != NONE) {  // the watched member's per-round log, to stderr
    std::vector<uint32_t> L(256 * 8);
    HIPC(h, hipMemcpy(L.data(), h->base.dbg_log, L.size() * 4, hipMemcpyDeviceToHost));
    for (uint32_t k = 0; k < 256; ++k)
      if (L[8 * k] || L[8 * k + 3])
        std::fprintf(stderr, "gpu watch r=%u win=%u alive=%u np=%u peers=%d,%d,%d supp=%u\n", L[8 * k], L[8 * k + 1],
                     L[8 * k + 2], L[8 * k + 3], (int)L[8 * k + 4], (int)L[8 * k + 5], (int)L[8 * k + 6], L[8 * k + 7]);
  }
  return SWIM_OK;
}

int swim_shard_buffer_words(swim_handle* h, uint64_t* send_words, uint64_t* recv_words) {
  if (!h || !send_words || !recv_words) return SWIM_EINVAL;
  const uint64_t W32 = h->GC / 32, nloc = h->base.nloc;
  // window records: <= f per local sender, 2 + active words each; SYNC rows: <= scap, 2 + N each;
  // gossip commits: 4 words per staged gossip (x world when gathered); round maxima: W32 + 2
  const uint64_t win = nloc * (uint64_t)h->base.f * (2 + W32);
  const uint64_t rows = (uint64_t)h->scap * (h->base.W + 2ull);
  // commits carry the liveness maxima too, and once members leave a header and the stopped members
  const uint64_t stg = 4ull * h->base.stg_cap + commit_tail(h) + 4 + nloc;
  // The window bounds assume every pair ships every active word; the need bitmaps ship only the
  // words a receiver lacks something in, far fewer (k_gossip_need), so both buffers are capped at
  // 2^31 words (8 GiB): C4's shards (32,768 rows of 262,144) would otherwise reserve ~90 GB for a
  // worst case that never occurs. A round that would exceed the cap fails loudly on every rank
  // (the sender checks its packed volume; swimhip/sharded.py checks every rank's receive volume).
  const uint64_t cap = 1ull << 31;
  *send_words = std::min(cap, std::max({win, rows, stg}));
  *recv_words = std::min(cap, std::max({(uint64_t)(h->N - nloc) * h->base.f * (2 + W32), rows, stg * h->world}));
  if (rows > cap || stg * h->world > cap) return fail(h, SWIM_EINVAL, "shard buffers: SYNC rows or commits exceed 2^31 words");
  return SWIM_OK;
}

int swim_shard_attach(swim_handle* h, void* send_dev, void* recv_dev) {
  if (!h || !send_dev || !recv_dev) return SWIM_EINVAL;
  h->xsend = send_dev;
  h->xrecv = recv_dev;
  uint64_t sw = 0, rw = 0;
  swim_shard_buffer_words(h, &sw, &rw);
  h->xsend_words = sw;
  h->xrecv_words = rw;
  return status_buffers(h);
}

int swim_shard_set_transport(swim_handle* h, const swim_transport* t) {
  if (!h || !t || !t->allgather || !t->alltoallv) return SWIM_EINVAL;
  if (h->pc != PC_FD) return fail(h, SWIM_EINVAL, "swim_shard_set_transport: a period is in flight");
  h->tr = *t;
  h->has_tr = true;
  h->sharded = true;  // (world 1: every exchange goes through the transport to this rank alone)
  return tr_buffers(h);
}

int swim_rccl_unique_id(uint8_t unique_id[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId");
  if (!unique_id) return SWIM_EINVAL;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return SWIM_ERCCL;
  std::memcpy(unique_id, &id, sizeof id);
  return SWIM_OK;
}

int swim_shard_comm_init(swim_handle* h, const uint8_t unique_id[128], uint32_t rank, uint32_t world) {
  if (!h || !unique_id || world != h->world || rank != h->rank) return SWIM_EINVAL;
  if (h->pc != PC_FD) return fail(h, SWIM_EINVAL, "swim_shard_comm_init: a period is in flight");
  if (hipSetDevice(h->cfg.device) != hipSuccess) return fail(h, SWIM_EHIP, "hipSetDevice");
  ncclUniqueId id;
  std::memcpy(&id, unique_id, sizeof id);
  if (h->comm) (void)ncclCommDestroy(h->comm);
  h->comm = nullptr;
  const ncclResult_t r = ncclCommInitRank(&h->comm, (int)world, id, (int)rank);
  if (r != ncclSuccess) return fail(h, SWIM_ERCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  swim_transport t{};
  t.ctx = h;
  t.host_staged = 0;
  t.allgather = rccl_allgather;
  t.alltoallv = rccl_alltoallv;
  h->tr = t;
  h->has_tr = true;
  h->sharded = true;
  return tr_buffers(h);
}

int swim_shard_step(swim_handle* h, swim_xchg* x) {
  if (!h || !x) return SWIM_EINVAL;
  if (h->sharded && (!h->xsend || !h->xrecv)) return fail(h, SWIM_EINVAL, "swim_shard_attach first");
  int rc = period_resume(h, x);
  if (rc) return rc;
  if (x->op == SWIM_X_DONE) {  // end of period: surface overflows like swim_step
    HIPC(h, hipStreamSynchronize(h->stream));
    resolve_timing(h);
    return check_overflow(h);
  }
  return SWIM_OK;
}

int swim_kernel_time(swim_handle* h, uint32_t idx, double* ms, uint64_t* launches) {
  if (!h || idx >= (uint32_t)NCLASS) return SWIM_EINVAL;
  if (ms) *ms = h->acc_ms[idx];
  if (launches) *launches = h->acc_n[idx];
  return SWIM_OK;
}

int swim_kernel_time_reset(swim_handle* h, int enable) {
  if (!h) return SWIM_EINVAL;
  (void)hipStreamSynchronize(h->stream);
  resolve_timing(h);
  for (int i = 0; i < NCLASS; ++i) {
    h->acc_ms[i] = 0;
    h->acc_n[i] = 0;
  }
  h->timing = enable != 0;
  h->tmask = enable == 1 ? ~0u : (uint32_t)enable;  // (a class mask: only those launches get events)
  return SWIM_OK;
}

}  // extern "C"


// swim_oracle.cpp — CPU oracle for the SWIM hot path. TEST INFRASTRUCTURE ONLY.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
// and only as the checker. It is a sequential, single-threaded restatement of the reference's
// protocol logic (scalecube-cluster @ /root/reference), written member-by-member the way the
// Java code runs on each member's single-threaded scheduler (ClusterImpl.java:178), under the
// discrete replay semantics fixed in DESIGN.md §3. Every function cites the reference lines
// it restates. Abbreviations:
//   MPI = cluster/src/main/java/io/scalecube/cluster/membership/MembershipProtocolImpl.java
//   FDI = cluster/src/main/java/io/scalecube/cluster/fdetector/FailureDetectorImpl.java
//   GPI = cluster/src/main/java/io/scalecube/cluster/gossip/GossipProtocolImpl.java
//   MR  = cluster/src/main/java/io/scalecube/cluster/membership/MembershipRecord.java
//   CM  = cluster/src/main/java/io/scalecube/cluster/ClusterMath.java
//   NE  = cluster-testlib/src/main/java/io/scalecube/cluster/utils/NetworkEmulator.java
//   NET = cluster-testlib/src/main/java/io/scalecube/cluster/utils/NetworkEmulatorTransport.java
//
// Parity: isOverrides is pinned by MembershipRecordTest (the reference's only bit-exact
// golden); everything RNG-driven is pinned by behavioural scenario restatements and
// self-consistency fixtures (the reference cannot run here: no JVM). See DESIGN.md §6.

#include "swim_oracle.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <new>
#include <unordered_map>
#include <vector>

namespace {

// ---------------------------------------------------------------------------------------
// Counter-based RNG: Philox4x32-10 (Salmon et al., SC'11). Replaces every JDK RNG call site
// on the path: Collections.shuffle (FDI:346,360; GPI:260), ThreadLocalRandom (FDI:326;
// MPI:420,424; NE:350).
// ---------------------------------------------------------------------------------------
struct U4 {
  uint32_t v[4];
};

inline void mulhilo(uint32_t a, uint32_t b, uint32_t* hi, uint32_t* lo) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  *hi = (uint32_t)(p >> 32);
  *lo = (uint32_t)p;
}

U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    if (r > 0) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    uint32_t hi0, lo0, hi1, lo1;
    mulhilo(0xD2511F53u, c.v[0], &hi0, &lo0);
    mulhilo(0xCD9E8D57u, c.v[2], &hi1, &lo1);
    U4 n;
    n.v[0] = hi1 ^ c.v[1] ^ k0;
    n.v[1] = lo1;
    n.v[2] = hi0 ^ c.v[3] ^ k1;
    n.v[3] = lo0;
    c = n;
  }
  return c;
}

inline uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

inline uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xFF51AFD7ED558CCDull;
  k ^= k >> 33;
  k *= 0xC4CEB9FE1A85EC53ull;
  k ^= k >> 33;
  return k;
}

// Message kinds and selection purposes.
enum Kind : uint32_t {
  K_PING = 1,
  K_ACK = 2,
  K_PING_REQ = 3,
  K_PROXY_PING = 4,
  K_PROXY_ACK = 5,
  K_FWD_ACK = 6,
  K_GOSSIP = 7,
  K_SYNC = 8,
  K_SYNC_ACK = 9,
  K_MREQ = 10,
  K_MRESP = 11,
  K_FD_PERM = 16,
  K_GOSSIP_PERM = 17,
  K_PROXY_PERM = 18,
  K_SYNC_PICK = 19,
};

inline U4 draw4(uint64_t seed, uint32_t kind, uint32_t a, uint32_t b, uint32_t c, uint32_t tick) {
  U4 ctr = {{a, b, c, tick}};
  return philox4x32_10(ctr, (uint32_t)seed ^ (kind * 0x9E3779B9u), (uint32_t)(seed >> 32));
}

inline uint32_t draw(uint64_t seed, uint32_t kind, uint32_t a, uint32_t b, uint32_t c, uint32_t tick) {
  return draw4(seed, kind, a, b, c, tick).v[0];
}

// Keyed bijection on [0, n): 4-round balanced Feistel on the next even power of two with
// cycle walking. Stands in for a Collections.shuffle'd member list (FDI:340-349,355-360;
// GPI:253-274): position p of the shuffled list = perm(p).
uint32_t perm(uint32_t x, uint32_t n, const uint32_t* k) {
  uint32_t bits = 2;
  while ((1ull << bits) < (uint64_t)n) ++bits;
  if (bits & 1) ++bits;
  const uint32_t half = bits / 2;
  const uint32_t mask = (1u << half) - 1u;
  do {
    uint32_t L = x >> half, R = x & mask;
    for (int r = 0; r < 4; ++r) {
      uint32_t F = fmix32(R ^ k[r]) & mask;
      uint32_t nl = R;
      R = L ^ F;
      L = nl;
    }
    x = (L << half) | R;
  } while (x >= n);
  return x;
}

// ---------------------------------------------------------------------------------------
// ClusterMath (CM:23-135).
// ---------------------------------------------------------------------------------------
inline int32_t ceil_log2(int32_t num) {  // CM:133-135: 32 - numberOfLeadingZeros(num)
  return num <= 0 ? (num == 0 ? 0 : 32) : 32 - __builtin_clz((uint32_t)num);
}
inline int32_t periods_to_spread(int32_t rm, int32_t n) { return rm * ceil_log2(n); }              // CM:111-113
inline int32_t periods_to_sweep(int32_t rm, int32_t n) { return 2 * (periods_to_spread(rm, n) + 1); }  // CM:99-102
inline int32_t suspicion_periods(int32_t mult, int32_t n) { return mult * ceil_log2(n); }            // CM:123-125 / pingInterval

// ---------------------------------------------------------------------------------------
// MembershipRecord.isOverrides (MR:66-84) on the packed encoding of include/swimhip.h.
// ---------------------------------------------------------------------------------------
inline uint32_t code_of(uint32_t r) { return r & 3u; }
inline uint32_t inc_of(uint32_t r) { return r >> 2; }
inline bool is_overrides(uint32_t r1, uint32_t r0) {
  if (r0 == SWIM_ABSENT) return r1 != SWIM_DEAD && code_of(r1) == SWIM_ALIVE;  // MR:67-69
  if (r0 == SWIM_DEAD) return false;                                              // MR:73-75
  if (r1 == SWIM_DEAD) return true;                                               // MR:76-78
  if (inc_of(r1) == inc_of(r0))                                                   // MR:79-80
    return code_of(r1) != code_of(r0) && code_of(r1) == SWIM_SUSPECT;
  return inc_of(r1) > inc_of(r0);                                                 // MR:82
}

// ---------------------------------------------------------------------------------------
// Simulation state.
// ---------------------------------------------------------------------------------------
struct Gossip {  // Gossip.java:7-49 + GossipRequest payload (MembershipRecord)
  uint32_t origin, seq, subject, record, hash;
  int64_t create;
  int32_t holders;  // members whose gossips map currently holds it
  int32_t inflight; // delayed GossipRequests of it still travelling (keep its id live)
};

// GossipProtocolImpl.gossips (GPI:49): gossipId -> GossipState (infectionPeriod,
// GossipState.java:14). Gossip ids (origin, seq) are numbered globally in creation order (gid);
// a member's map is a bitset over the id ring (slot = gid mod rc, rc at least twice the live id
// range, so live ids never share a slot) plus the infection round per slot, and the held ids in
// order of infection round, which is non-decreasing (every new state gets the gossip module's
// next round): the send window is a suffix of that order and the sweep a prefix.
struct GossipMap {
  std::vector<uint64_t> held;                        // rc bits
  std::vector<int64_t> inf;                          // rc slots
  std::deque<std::pair<uint32_t, int64_t>> order;    // (gid, infectionPeriod), oldest first
  // selectGossipsToSend's age filter as a bitset (rc bits): the window is the run of `order`
  // with infectionPeriod in [r - spread, r], positions [w_lo, w_end) counted from the first
  // entry ever held (`popped` entries have left the front), kept up to date round by round
  std::vector<uint64_t> win;
  uint64_t popped = 0, w_lo = 0, w_end = 0;
  int32_t w_spread = -1;
};

// GossipState.infected (GossipState.java:17; addToInfected GossipProtocolImpl.java:181): the
// members a gossip was received from during its current GossipState. Kept per receiver as the
// message batches each sender delivered: {round t, the gossips sent in t (a bitset over gid
// words from w0)}. Member p is in infected(g) iff a batch from p of a round t >= the round the
// current state of g was created (infectionPeriod - 1) carries g and that message was not lost —
// exactly the set the reference accumulates (a fresh state starts empty, every later delivery
// adds its sender). Loss draws of messages the receiver already held are evaluated only when a
// suppression query needs them (the draw is a pure function of the message). A batch of round t
// can only matter while the receiver may still send those gossips: rounds <= t + 1 + spread.
struct Batch {
  int64_t t;
  uint32_t tick;
  uint32_t dmean;  // the mean delay its messages were sent under (their arrival rounds)
  uint32_t w0;
  std::vector<uint64_t> bits;
};

struct Member {
  std::vector<uint32_t> table;          // MPI:87 membershipTable (+ MPI:88 members: cell != 0)
  std::vector<uint32_t> meta;           // MetadataStoreImpl.membersMetadata: the version of each member's
                                        // metadata this member fetched last (MetadataStoreImpl.java:112-135)
  uint32_t others = 0;                  // members.size() - 1 == pingMembers == remoteMembers
  int32_t delta = 0;                    // deferred member-count change of the current phase
  std::map<uint32_t, uint64_t> timers;  // MPI:101 suspicionTimeoutTasks: subject -> fire period
  uint32_t fd_epoch = 0, fd_cursor = 0; // FDI:49-50 pingMembers order + pingMemberIndex
  uint32_t g_epoch = 0, g_cursor = 0;   // GPI:52-53 remoteMembers order + remoteMembersIndex
  GossipMap gossips;                    // GPI:49 gossips
  std::unordered_map<uint32_t, std::vector<Batch>> recv;  // sender -> batches (infected sets)
  uint32_t gossip_seq = 0;              // GPI:48 gossipCounter
  uint32_t foreign_seq = 0;             // gossips forwarded for real nodes (their own id namespace)
  uint32_t sync_fd = 0xFFFFFFFFu;       // FD-triggered SYNC target of this period (MPI:385-397)
  bool alive = true;
  // graceful leave (MPI:203-212): the gossip of its own DEAD record; the member shuts down once
  // its own sweep drops it (GossipProtocolImpl.spread completes at sweep, :299-302, and
  // ClusterImpl.doShutdown then disposes and stops the transport, ClusterImpl.java:376-388)
  bool leaving = false, stop = false;
  uint32_t leave_gid = 0;
};

struct SyncReq {
  // kind 0 = periodic doSync (MPI:304-320), 1 = FD-triggered (MPI:389-397), 2 = a joining member's
  // initial SYNC to a seed (start0, MPI:222-257). `to` = the member addressed (for a seed: the member
  // id that owns the seed address), the process at its address receives it.
  uint32_t from, to, kind;
};

// the metadata-fetch attempt id of a SYNC / SYNC_ACK merge (distinct per request)
inline uint32_t sync_attempt(uint32_t peer, uint32_t kind) { return kind == 2 ? 0x80000000u | peer : (peer << 1) | kind; }

}  // namespace

struct oracle_handle {
  swim_config cfg;
  uint32_t N;
  uint32_t G, S, TPP;
  int32_t sweepmax;
  uint64_t seed;
  uint64_t period = 0;
  uint32_t loss_bp = 0;
  // NetworkEmulator.OutboundSettings.meanDelay (NE:309-368) of every link, in ms (0 = none), and
  // its exponential draw as a threshold table: dthr[k] = the smallest 32-bit uniform whose delay
  // -ln(1 - u/2^32) * mean (NE:358-368) is >= k ms, for every k a 32-bit draw can reach
  uint32_t delay_mean = 0;
  std::map<uint32_t, std::vector<uint32_t>> dthr;  // per mean ever set (batches keep their own)
  uint32_t dmax_rounds = 0;  // the longest gossip delay any mean set so far can give, in rounds
  // GossipRequests delayed past their round: delivered at the start of round
  // `arrive`'s onGossipReq step to process `to`, if it still runs
  struct Flight {
    int64_t arrive;
    uint32_t to, from, gid;
  };
  std::vector<Flight> flights;
  std::vector<uint8_t> group;
  uint64_t part_t0 = 0, part_t1 = 0;
  std::vector<uint8_t> link;    // outbound block src->dst (send error), lazily allocated
  std::vector<uint8_t> inlink;  // inbound block at dst of messages from src (silent drop)
  std::vector<Member> m;
  // Addresses: member id x is reached at address addr[x]; occ[a] is the running
  // member at address a (NONE when its transport is stopped). A restart on the same address gives
  // the address to a new member id, so messages sent to the old id reach the new member.
  std::vector<uint32_t> addr, occ;
  std::vector<std::vector<uint32_t>> movers;  // per address: the members restarted on it
  std::vector<uint8_t> started, joining;
  std::vector<Gossip> registry;  // by gid
  uint32_t gbase = 0;            // every gid below is held by nobody
  uint32_t rc = 256;             // slots of each member's GossipMap (power of two)
  int32_t hzn = 0;               // gossipPeriodsToSpread(N) + 1: rounds a batch can matter
  std::vector<swim_event> events;
  swim_stats st;
  std::vector<uint32_t> pres, last_removed;
  std::vector<uint32_t> meta_cur;  // each member's own metadata version (MetadataStoreImpl.updateMetadata, :107-110)
  uint32_t trace = 0;              // swim_trace mask (SWIM_TRACE_FD: FailureDetectorEvents into the ring)
  std::vector<uint64_t> dbg_send;  // debug: per sender, GossipRequests to alive peers before / by infectedFrom
  uint32_t dbg_watch = 0xFFFFFFFFu;
  // pending gossip-delivered records per receiver: subject -> lattice max
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>> inbox;
};

namespace {

inline uint32_t ghash(uint32_t origin, uint32_t seq) { return fmix32(origin ^ fmix32(seq + 0x9E3779B9u)); }

inline uint32_t tick_of(const oracle_handle* h, uint32_t phase) { return (uint32_t)(h->period * h->TPP + phase); }

inline bool bit_set(const std::vector<uint8_t>& bm, uint64_t bit) {
  return !bm.empty() && (bm[bit >> 3] & (1u << (bit & 7)));
}

constexpr uint32_t NONE = 0xFFFFFFFFu;

// The member whose transport receives what is sent to member x (TransportImpl sends to
// member.address(), NET:44-70): the running member at x's address, or NONE.
inline uint32_t route(const oracle_handle* h, uint32_t x) { return h->occ[h->addr[x]]; }

// The sender side of NetworkEmulatorTransport.send/requestResponse (NET:44-70): tryFailOutbound
// (NE:166-180) fails the send immediately — a NETWORK_BREAK error the sender sees — on a
// loss draw (NE:348-351, nextInt(100) < lossPercent) or a blocked destination (loss 100 %,
// NE:105-119; the partition cut is a blockOutbound on both sides). A stopped transport
// (crash) neither sends nor accepts connections, which the sender also sees as an error.
// src and dst are the member ids the message is addressed from / to; the processes at their
// addresses send and receive it (route), partition groups and blocks are per address, and the loss
// draw is keyed by the two processes.
bool out_ok(const oracle_handle* h, uint32_t kind, uint32_t src, uint32_t dst, uint32_t c, uint32_t tick) {
  const uint32_t rs = route(h, src), rd = route(h, dst);
  if (rs == NONE || rd == NONE) return false;
  const uint32_t as = h->addr[src], ad = h->addr[dst];
  if (h->period >= h->part_t0 && h->period < h->part_t1 && h->group[as] != h->group[ad]) return false;
  if (bit_set(h->link, (uint64_t)as * h->N + ad)) return false;
  if (h->loss_bp == 0) return true;      // NE:349 lossPercent > 0
  if (h->loss_bp >= 10000) return false; // NE:350 lossPercent >= 100
  uint32_t thr = (uint32_t)(((uint64_t)h->loss_bp << 32) / 10000u);
  return draw(h->seed, kind, rs, rd, c, tick) >= thr;  // NE:350 nextInt(100) < loss => lost
}

// The receiver side: NET:73-77 (listen) and NET:64-68 (responses) drop a message whose sender
// the receiver blocks inbound (NE:255-269), silently — the sender saw a successful send.
bool in_ok(const oracle_handle* h, uint32_t dst, uint32_t src) {
  return !bit_set(h->inlink, (uint64_t)h->addr[dst] * h->N + h->addr[src]);
}

// Everything of delivered() but the loss draw: both transports up, no partition cut, no block.
bool link_ok(const oracle_handle* h, uint32_t src, uint32_t dst) {
  if (route(h, src) == NONE || route(h, dst) == NONE) return false;
  const uint32_t as = h->addr[src], ad = h->addr[dst];
  if (h->period >= h->part_t0 && h->period < h->part_t1 && h->group[as] != h->group[ad]) return false;
  return !bit_set(h->link, (uint64_t)as * h->N + ad) && in_ok(h, dst, src);
}

// Is message src->dst delivered to dst's protocol handlers?
bool delivered(const oracle_handle* h, uint32_t kind, uint32_t src, uint32_t dst, uint32_t c, uint32_t tick) {
  return out_ok(h, kind, src, dst, c, tick) && in_ok(h, dst, src);
}

// NetworkEmulator.tryDelayOutbound / evaluateDelay (NE:189-201,358-368) of message src->dst: its
// delay in whole ms, from the second word of the message's draw (the first is its loss draw, so one
// Philox block decides both): (long)(-ln(1 - x) * meanDelay) with x = u / 2^32, read from the
// threshold table (exact integer compares, no floating point per message).
uint32_t delay_of_draw(const oracle_handle* h, uint32_t mean, uint32_t u) {
  if (mean == 0) return 0;
  const std::vector<uint32_t>& t = h->dthr.at(mean);
  return (uint32_t)(std::upper_bound(t.begin(), t.end(), u) - t.begin()) - 1u;
}
uint32_t msg_delay(const oracle_handle* h, uint32_t kind, uint32_t src, uint32_t dst, uint32_t c, uint32_t tick) {
  if (h->delay_mean == 0) return 0;
  const uint32_t rs = route(h, src), rd = route(h, dst);
  if (rs == NONE || rd == NONE) return 0;  // not sent at all (out_ok fails)
  return delay_of_draw(h, h->delay_mean, draw4(h->seed, kind, rs, rd, c, tick).v[1]);
}

void perm_keys(const oracle_handle* h, uint32_t kind, uint32_t member, uint32_t epoch, uint32_t* k) {
  U4 r = draw4(h->seed, kind, member, epoch, 0, 0);
  for (int i = 0; i < 4; ++i) k[i] = r.v[i];
}

void emit_event(oracle_handle* h, uint32_t obs, uint32_t subj, uint32_t type, uint32_t reason, uint32_t phase,
                uint32_t record) {
  if (type == SWIM_EV_ADDED) h->st.events_added++;
  if (type == SWIM_EV_REMOVED) h->st.events_removed++;
  if (type == SWIM_EV_UPDATED) h->st.events_updated++;
  if (h->cfg.event_capacity == 0) return;
  swim_event e;
  std::memset(&e, 0, sizeof e);
  e.period = h->period;
  e.observer = obs;
  e.subject = subj;
  e.record = record;
  e.type = (uint8_t)type;
  e.reason = (uint8_t)reason;
  e.phase = (uint8_t)phase;
  h->events.push_back(e);
}

inline bool gossip_held(const oracle_handle* h, const Member& me, uint32_t gid) {
  const uint32_t sl = gid & (h->rc - 1);
  return (me.gossips.held[sl >> 6] >> (sl & 63)) & 1u;
}

// infectionPeriod of a held gossip of the live id range, or -1
int64_t gossip_find(const oracle_handle* h, const Member& me, uint32_t gid) {
  return gossip_held(h, me, gid) ? me.gossips.inf[gid & (h->rc - 1)] : -1;
}

// the held bits of absolute id word w (ids 64w .. 64w+63); the ring has no aliasing words
inline uint64_t held_word(const oracle_handle* h, const Member& me, uint32_t w) {
  return me.gossips.held[w & ((h->rc >> 6) - 1)];
}

// Grow the ring until it holds twice the live id range plus a word of slack on each side.
void gossip_reserve(oracle_handle* h, uint32_t gend) {
  if (2ull * (gend - h->gbase) + 256 <= h->rc) return;
  uint32_t nrc = h->rc;
  while (2ull * (gend - h->gbase) + 256 > nrc) nrc *= 2;
  for (auto& mm : h->m) {
    GossipMap& g = mm.gossips;
    std::vector<uint64_t> nh(nrc / 64, 0), nw(nrc / 64, 0);
    std::vector<int64_t> ni(nrc, 0);
    for (size_t k = 0; k < g.order.size(); ++k) {
      const auto& e = g.order[k];
      const uint32_t sl = e.first & (nrc - 1);
      nh[sl >> 6] |= 1ull << (sl & 63);
      ni[sl] = e.second;
      if (g.popped + k >= g.w_lo && g.popped + k < g.w_end) nw[sl >> 6] |= 1ull << (sl & 63);
    }
    g.held.swap(nh);
    g.inf.swap(ni);
    g.win.swap(nw);
  }
  h->rc = nrc;
}

// gossips.put(id, new GossipState(gossip, inf)) (GossipProtocolImpl.java:166-167,177-178) for a
// gossip the member does not hold (the ring already has room for gid)
void gossip_put(oracle_handle* h, Member& me, uint32_t gid, int64_t inf) {
  const uint32_t sl = gid & (h->rc - 1);
  me.gossips.held[sl >> 6] |= 1ull << (sl & 63);
  me.gossips.inf[sl] = inf;
  me.gossips.order.push_back({gid, inf});
  h->registry[gid].holders++;
}

// gossips.remove(id) of the oldest held gossip (sweepGossips, GossipProtocolImpl.java:297-298)
void gossip_pop_oldest(oracle_handle* h, Member& me) {
  GossipMap& g = me.gossips;
  const uint32_t gid = g.order.front().first;
  const uint32_t sl = gid & (h->rc - 1);
  g.held[sl >> 6] &= ~(1ull << (sl & 63));
  if (g.popped >= g.w_lo && g.popped < g.w_end) {  // still in the window bitset
    g.win[sl >> 6] &= ~(1ull << (sl & 63));
    g.w_lo = g.popped + 1;
  }
  g.order.pop_front();
  g.popped++;
  g.w_lo = std::max(g.w_lo, g.popped);
  g.w_end = std::max(g.w_end, g.w_lo);
  h->registry[gid].holders--;
}

// transport.stop(): the member stops sending, receiving, answering and firing timers.
void stop_member(oracle_handle* h, uint32_t c) {
  Member& me = h->m[c];
  if (!me.alive) return;
  me.alive = false;
  if (h->occ[h->addr[c]] == c) h->occ[h->addr[c]] = NONE;
  me.timers.clear();  // its scheduler is gone
  while (!me.gossips.order.empty()) gossip_pop_oldest(h, me);
  me.recv.clear();
  for (uint32_t j = 0; j < h->N; ++j)
    if (j != c && me.table[j] != SWIM_ABSENT) h->pres[j]--;
}

// Bring the window bitset to round r: gossips with infectionPeriod in [r - spread, r] (GPI:247).
void window_update(oracle_handle* h, GossipMap& g, int64_t r, int32_t spread) {
  auto flip = [&](uint64_t pos) {
    const uint32_t sl = g.order[pos - g.popped].first & (h->rc - 1);
    g.win[sl >> 6] ^= 1ull << (sl & 63);
  };
  if (spread != g.w_spread) {  // view size changed ClusterMath's spread: rebuild
    for (uint64_t k = g.w_lo; k < g.w_end; ++k) flip(k);
    g.w_lo = g.w_end = g.popped;
    g.w_spread = spread;
  }
  const uint64_t end = g.popped + g.order.size();
  while (g.w_end < end && g.order[g.w_end - g.popped].second <= r) flip(g.w_end++);
  while (g.w_lo < g.w_end && g.order[g.w_lo - g.popped].second + spread < r) flip(g.w_lo++);
}

// GossipProtocolImpl.spread -> createAndPutGossip (GPI:124-128,163-169,211-213): the new
// gossip's infectionPeriod is the gossip module's *next* round (`currentPeriod`).
// foreign: a real node's gossip the member forwards (SWIM_DELIVER_FORWARD): onGossipReq puts it under
// its own gossipId (GPI:171-183) and the member's gossipCounter does not move; it gets an id of the
// member's foreign namespace (0x80000000 | k) instead
void spread_gossip(oracle_handle* h, uint32_t origin, uint32_t subject, uint32_t record, int64_t create_round,
                   bool foreign = false) {
  Member& o = h->m[origin];
  uint32_t seq = foreign ? (0x80000000u | o.foreign_seq++) : o.gossip_seq++;
  const uint32_t gid = (uint32_t)h->registry.size();
  h->registry.push_back(Gossip{origin, seq, subject, record, ghash(origin, seq), create_round, 0, 0});
  gossip_reserve(h, gid + 1);
  gossip_put(h, o, gid, create_round);
  h->st.gossips_created++;
}

// MetadataStoreImpl.fetchMetadata (core/metadata/MetadataStoreImpl.java:151-193) as a
// liveness round trip: GET_METADATA_REQ obs->subj and GET_METADATA_RESP subj->obs delivered
// and the subject serving: the process at its address must be the subject itself (onMetadataRequest
// answers only requests for its own id, :216-223; otherwise the fetch times out).
// With message delays the round trip must come back within metadataTimeout (:170).
bool fetch_ok(const oracle_handle* h, uint32_t obs, uint32_t subj, uint32_t attempt, uint32_t tick) {
  return route(h, subj) == subj && delivered(h, K_MREQ, obs, subj, attempt, tick) &&
         delivered(h, K_MRESP, subj, obs, attempt, tick) &&
         msg_delay(h, K_MREQ, obs, subj, attempt, tick) + msg_delay(h, K_MRESP, subj, obs, attempt, tick) <
             (uint32_t)h->cfg.metadata_timeout_ms;
}

// MembershipProtocolImpl.updateMembership (MPI:481-547) with its callees onSelfMemberDetected
// (MPI:549-569), onDeadMemberDetected (MPI:571-587), onAliveMemberDetected (MPI:589-610),
// scheduleSuspicionTimeoutTask (MPI:620-635), cancelSuspicionTimeoutTask (MPI:612-618),
// spreadMembershipGossipUnlessGossiped (MPI:649-656).
//   others_snap: the observer's member count at phase start
void update_membership(oracle_handle* h, uint32_t obs, uint32_t subj, uint32_t r1, uint32_t reason, uint32_t phase,
                       uint32_t attempt, uint32_t tick, uint32_t others_snap, int64_t create_round) {
  Member& me = h->m[obs];
  uint32_t& cell = me.table[subj];
  const uint32_t r0 = cell;
  if (!is_overrides(r1, r0)) return;  // MPI:489-496 (equal records never override)
  if (subj != obs && h->addr[subj] == h->addr[obs]) return;  // MPI:499-505: another id at my address
  const bool spread = reason != SWIM_R_MEMBERSHIP_GOSSIP && reason != SWIM_R_INITIAL_SYNC;  // MPI:652-653
  if (subj == obs) {  // MPI:499-501 -> onSelfMemberDetected MPI:549-569
    uint32_t inc1 = (r1 == SWIM_DEAD) ? inc_of(r0) : inc_of(r1);
    uint32_t r2 = SWIM_PACK(std::max(inc_of(r0), inc1) + 1u, code_of(r0));
    cell = r2;
    h->st.records_accepted++;
    h->st.refutations++;
    spread_gossip(h, obs, obs, r2, create_round);  // MPI:567 (always spread)
    return;
  }
  if (r1 == SWIM_DEAD) {  // MPI:507-509 -> onDeadMemberDetected MPI:571-587
    me.timers.erase(subj);
    cell = SWIM_ABSENT;  // r0 != null guaranteed by isOverrides
    me.delta -= 1;
    h->st.records_accepted++;
    if (me.alive && subj != obs) {
      h->pres[subj]--;
      h->last_removed[subj] = std::max<uint32_t>(h->last_removed[subj], (uint32_t)h->period + 1u);
    }
    emit_event(h, obs, subj, SWIM_EV_REMOVED, reason, phase, r0);
    return;
  }
  if (code_of(r1) == SWIM_SUSPECT) {  // MPI:511-516
    cell = r1;
    h->st.records_accepted++;
    if (me.timers.find(subj) == me.timers.end())  // computeIfAbsent (MPI:627-634)
      me.timers[subj] = h->period + (uint64_t)suspicion_periods(h->cfg.suspicion_mult, (int32_t)others_snap + 1);
    if (spread) spread_gossip(h, obs, subj, r1, create_round);
    return;
  }
  // ALIVE with r0 == null or r0.inc < r1.inc (MPI:518-542)
  if (!fetch_ok(h, obs, subj, attempt, tick)) return;  // MPI:540 failed fetch silently skipped
  me.timers.erase(subj);                               // MPI:534
  if (spread) spread_gossip(h, obs, subj, r1, create_round);  // MPI:535
  // the fetched metadata (the subject's current version) replaces the stored one (MPI:537)
  const uint32_t m1 = h->meta_cur[subj], m0 = me.meta[subj];
  me.meta[subj] = m1;
  cell = r1;                                                  // MPI:604
  h->st.records_accepted++;
  if (r0 == SWIM_ABSENT) {  // MPI:597-598 ADDED
    me.delta += 1;
    if (me.alive && subj != obs) h->pres[subj]++;
    emit_event(h, obs, subj, SWIM_EV_ADDED, reason, phase, r1);
  } else if (m1 != m0) {  // MPI:599-600 UPDATED: metadata differs from the stored one
    emit_event(h, obs, subj, SWIM_EV_UPDATED, reason, phase, r1);
  }
}

void finish_phase(oracle_handle* h) {
  for (auto& mm : h->m) {
    mm.others = (uint32_t)((int32_t)mm.others + mm.delta);
    mm.delta = 0;
  }
}

// ---------------------------------------------------------------------------------------
// FailureDetectorImpl (FDI).
// ---------------------------------------------------------------------------------------
// selectPingMember (FDI:340-349): round robin over a shuffled list; reshuffle on wrap.
uint32_t select_ping_member(oracle_handle* h, uint32_t i) {
  Member& me = h->m[i];
  uint32_t k[4];
  perm_keys(h, K_FD_PERM, i, me.fd_epoch, k);
  for (;;) {
    if (me.fd_cursor >= h->N) {
      me.fd_cursor = 0;
      me.fd_epoch++;
      perm_keys(h, K_FD_PERM, i, me.fd_epoch, k);
    }
    uint32_t x = perm(me.fd_cursor++, h->N, k);
    if (x != i && me.table[x] != SWIM_ABSENT) return x;
  }
}

// selectPingReqMembers (FDI:351-363): first k of shuffle(pingMembers \ {target}).
std::vector<uint32_t> select_ping_req_members(oracle_handle* h, uint32_t i, uint32_t j) {
  std::vector<uint32_t> out;
  const int32_t kreq = h->cfg.ping_req_members;
  if (kreq <= 0) return out;
  uint32_t k[4];
  perm_keys(h, K_PROXY_PERM, i, (uint32_t)h->period, k);
  const Member& me = h->m[i];
  for (uint32_t pos = 0; pos < h->N && (int32_t)out.size() < kreq; ++pos) {
    uint32_t x = perm(pos, h->N, k);
    if (x != i && x != j && me.table[x] != SWIM_ABSENT) out.push_back(x);
  }
  return out;
}

// MembershipProtocolImpl.onFailureDetectorEvent (MPI:376-404).
void on_fd_event(oracle_handle* h, uint32_t i, uint32_t j, uint32_t status, uint32_t tick) {
  Member& me = h->m[i];
  const uint32_t r0 = me.table[j];
  if (r0 == SWIM_ABSENT) return;          // MPI:378-380
  if (code_of(r0) == status) return;      // MPI:381-383
  if (status == SWIM_ALIVE) {             // MPI:385-397: SYNC to the member instead
    me.sync_fd = j;
    return;
  }
  // MPI:399-402 (status SUSPECT, or DEAD from a DEST_GONE ack: the packed DEAD cell)
  update_membership(h, i, j, status == SWIM_DEAD ? SWIM_DEAD : SWIM_PACK(inc_of(r0), status),
                    SWIM_R_FAILURE_DETECTOR_EVENT, 0, 0, tick, me.others, (int64_t)h->period * h->G);
}

// doPing (FDI:126-170) + doPingReq (FDI:172-209) + responder handlers onPing (FDI:226-252),
// onPingReq (FDI:255-277), onTransitPingAck (FDI:283-305), with TransportImpl's cid-only
// response matching (TransportImpl.java:236-238): all ping-req subscriptions share the cid,
// so the first transit ack completes every one still pending.
void do_ping(oracle_handle* h, uint32_t i) {
  Member& me = h->m[i];
  if (me.others == 0) return;  // FDI:132-134 pingMembers empty
  const uint32_t tick = tick_of(h, 0);
  const uint32_t j = select_ping_member(h, i);
  h->st.fd_probes++;
  std::vector<uint32_t> evs;
  // onPing (FDI:226-252) at the process on j's address answers DEST_GONE unless it is j itself;
  // computeMemberStatus (FDI:370-391) turns that ack into DEAD
  const uint32_t acked = route(h, j) == j ? SWIM_ALIVE : SWIM_DEAD;
  // round trip of the direct ping (its delays, NE:189-201); the ack counts if it is back within
  // pingTimeout (FDI:145 .timeout), otherwise it arrives late (handled with the ping-req below)
  const uint32_t t_direct = msg_delay(h, K_PING, i, j, 0, tick) + msg_delay(h, K_ACK, j, i, 0, tick);
  const bool ping_in = delivered(h, K_PING, i, j, 0, tick);
  if (ping_in && delivered(h, K_ACK, j, i, 0, tick) && (!h->delay_mean || t_direct < (uint32_t)h->cfg.ping_timeout_ms)) {  // FDI:143-150
    h->st.fd_direct_ok++;
    evs.push_back(acked);
  } else {
    const int32_t time_left = h->cfg.ping_interval_ms - h->cfg.ping_timeout_ms;  // FDI:160
    std::vector<uint32_t> proxies = select_ping_req_members(h, i, j);           // FDI:161
    if (time_left <= 0 || proxies.empty()) {                                     // FDI:163-165
      evs.push_back(SWIM_SUSPECT);
    } else {
      h->st.fd_ping_req++;
      uint32_t unsent = 0, sent = 0;
      // the ack that reaches i's transport first, and when (ms from the direct ping's send). The
      // PING_REQs go out when the direct ping times out (FDI:152-168) and wait time_left (FDI:183).
      // The direct ping's own ack, when late, shares their correlation id (FDI:174-178) and is
      // taken the same way if it comes back before they time out.
      uint32_t first = 0xFFFFFFFFu, t_first = 0xFFFFFFFFu;
      const uint32_t pto = (uint32_t)h->cfg.ping_timeout_ms, pint = (uint32_t)h->cfg.ping_interval_ms;
      for (uint32_t p : proxies) {
        if (!out_ok(h, K_PING_REQ, i, p, j, tick)) {  // tryFailOutbound: immediate error -> SUSPECT
          ++unsent;
          continue;
        }
        ++sent;
        // onPingReq (FDI:255-277) -> transit PING -> onPing at j -> ACK to the proxy ->
        // onTransitPingAck (FDI:283-305) forwards it to i. Each hop is a send that the next
        // receiver's inbound filter may drop; the last hop reaches i's TransportImpl.
        if (in_ok(h, p, i) && delivered(h, K_PROXY_PING, p, j, i, tick) && delivered(h, K_PROXY_ACK, j, p, i, tick) &&
            out_ok(h, K_FWD_ACK, p, i, j, tick)) {
          const uint32_t hops = msg_delay(h, K_PING_REQ, i, p, j, tick) + msg_delay(h, K_PROXY_PING, p, j, i, tick) +
                                msg_delay(h, K_PROXY_ACK, j, p, i, tick) + msg_delay(h, K_FWD_ACK, p, i, j, tick);
          if (hops < (uint32_t)time_left && pto + hops < t_first) {  // earliest; ties: selection order
            first = p;
            t_first = pto + hops;
          }
        }
      }
      // the late direct ack (sender j) wins ties: it is compared first
      if (h->delay_mean && sent && ping_in && out_ok(h, K_ACK, j, i, 0, tick) && t_direct >= pto && t_direct < pint &&
          t_direct <= t_first) {
        first = j;
        t_first = t_direct;
      }
      // TransportImpl.requestResponse matches responses by correlation id only (:236-238) and
      // every PING_REQ of this probe carries the same cid (FDI:174-178), so the first ack to
      // arrive (without delays: the first proxy in selection order whose relay got through) is
      // taken by every pending subscription; NET:64-68 then checks i's inbound filter against
      // that ack's sender: blocked -> Mono.never() -> every subscription times out.
      const bool ok = first != 0xFFFFFFFFu && in_ok(h, i, first);
      for (uint32_t u = 0; u < unsent; ++u) evs.push_back(SWIM_SUSPECT);
      for (uint32_t s = 0; s < sent; ++s) evs.push_back(ok ? acked : SWIM_SUSPECT);  // FDI:190-207
    }
  }
  for (uint32_t k = 0; k < evs.size(); ++k)  // FailureDetector.listen() (FDI:365-368), when traced
    if (h->trace & SWIM_TRACE_FD) emit_event(h, i, j, SWIM_EV_FD, k, 0, evs[k]);
  for (uint32_t ev : evs) {  // publishPingResult (FDI:365-368) -> MPI:376
    if (ev == SWIM_ALIVE)
      h->st.fd_alive_events++;
    else if (ev == SWIM_DEAD)
      h->st.fd_dead_events++;
    else
      h->st.fd_suspect_events++;
    on_fd_event(h, i, j, ev, tick);
  }
}

// ---------------------------------------------------------------------------------------
// GossipProtocolImpl (GPI).
// ---------------------------------------------------------------------------------------
// selectGossipMembers (GPI:253-274): all if size < fanout, else the window [idx, idx+fanout)
// of a shuffled list, reshuffled when the window would run past the end.
std::vector<uint32_t> select_gossip_members(oracle_handle* h, uint32_t g) {
  Member& me = h->m[g];
  const uint32_t f = (uint32_t)h->cfg.gossip_fanout;
  std::vector<uint32_t> out;
  if (me.others < f) {  // GPI:255-256
    for (uint32_t x = 0; x < h->N; ++x)
      if (x != g && me.table[x] != SWIM_ABSENT) out.push_back(x);
    return out;
  }
  for (int attempt = 0; attempt < 2; ++attempt) {
    uint32_t k[4];
    perm_keys(h, K_GOSSIP_PERM, g, me.g_epoch, k);
    out.clear();
    uint32_t pos = me.g_cursor;
    while (pos < h->N && out.size() < f) {
      uint32_t x = perm(pos++, h->N, k);
      if (x != g && me.table[x] != SWIM_ABSENT) out.push_back(x);
    }
    if (out.size() == f) {
      me.g_cursor = pos;
      return out;
    }
    me.g_epoch++;  // GPI:259-262 reshuffle
    me.g_cursor = 0;
  }
  return out;  // unreachable when others >= f
}

// One gossip round r: doSpreadGossip (GPI:139-157) of every member on the
// start-of-round state, then onGossipReq (GPI:171-183) deliveries, then membership apply
// (MPI:407-414 via the inbox lattice max).
void gossip_round(oracle_handle* h, uint32_t q) {
  const int64_t r = (int64_t)h->period * h->G + q;
  const uint32_t phase = 1 + q;
  const uint32_t tick = tick_of(h, phase);
  const int32_t rm = h->cfg.gossip_repeat_mult;
  while (h->gbase < h->registry.size() && h->registry[h->gbase].holders == 0 && h->registry[h->gbase].inflight == 0)
    h->gbase++;
  const uint32_t gend = (uint32_t)h->registry.size();
  const uint32_t wlo = h->gbase >> 6, whi = (gend + 63) >> 6, nw = whi - wlo;
  const uint32_t thr = (uint32_t)(((uint64_t)h->loss_bp << 32) / 10000u);
  // NetworkEmulator.evaluateLoss of one GossipRequest (NE:348-351), the sender side of out_ok
  auto not_lost = [&](uint32_t src, uint32_t dst, uint32_t gid, uint32_t tk) {
    if (h->loss_bp == 0) return true;
    if (h->loss_bp >= 10000) return false;
    return draw(h->seed, K_GOSSIP, src, dst, h->registry[gid].hash, tk) >= thr;
  };
  // NetworkEmulator.evaluateDelay of the same message in whole gossip rounds:
  // sent in round t, it is handled by onGossipReq in round t + delay / gossipInterval
  const uint32_t gint = (uint32_t)h->cfg.gossip_interval_ms;
  auto delay_rounds = [&](uint32_t mean, uint32_t src, uint32_t dst, uint32_t gid, uint32_t tk) -> uint32_t {
    if (mean == 0) return 0;
    return delay_of_draw(h, mean, draw4(h->seed, K_GOSSIP, src, dst, h->registry[gid].hash, tk).v[1]) / gint;
  };
  // GPI:144-146 "gossips.isEmpty()" on the start-of-round state of every member
  std::vector<uint8_t> nonempty(h->N, 0);
  for (uint32_t s = 0; s < h->N; ++s) nonempty[s] = h->m[s].alive && !h->m[s].gossips.order.empty();
  // sweepGossips (GPI:281-304) at the end of each doSpreadGossip(r). A swept gossip is never in
  // its holder's window (spread < sweep), so sweeping first changes no send of round r; it only
  // makes round-r deliveries of it start a new GossipState, as they do in the reference.
  for (uint32_t s = 0; s < h->N; ++s) {
    Member& me = h->m[s];
    if (!me.alive) continue;
    const int32_t sweep = periods_to_sweep(rm, (int32_t)me.others + 1);  // GPI:283-284
    while (!me.gossips.order.empty() && r > me.gossips.order.front().second + sweep) {
      if (me.leaving && me.gossips.order.front().first == me.leave_gid) me.stop = true;  // GPI:299-302
      gossip_pop_oldest(h, me);
    }
  }
  // Every member's doSpreadGossip(r) runs on the start-of-round state (its gossips, their
  // infected sets, its peers); the messages are handled by the receivers' onGossipReq after
  // all of them, with currentPeriod = r + 1.
  struct Delivery {
    uint32_t to, gid;
  };
  struct Sent {
    uint32_t to, from;
    Batch b;
  };
  std::vector<Delivery> deliveries;
  std::vector<Sent> sent;
  std::vector<uint64_t> W(nw), S(nw);
  for (uint32_t s = 0; s < h->N; ++s) {
    Member& me = h->m[s];
    if (!nonempty[s]) continue;  // GPI:144-146 (no peer selection either)
    const int32_t spread = periods_to_spread(rm, (int32_t)me.others + 1);  // GPI:243-244
    // selectGossipsToSend's age filter (GPI:247)
    window_update(h, me.gossips, r, spread);
    const uint32_t rw = (h->rc >> 6) - 1;
    for (uint32_t k = 0; k < nw; ++k) W[k] = me.gossips.win[(wlo + k) & rw];
    std::vector<uint32_t> peers = select_gossip_members(h, s);  // GPI:150
    if (me.gossips.w_lo == me.gossips.w_end) continue;
    for (uint32_t p : peers) {
      const uint32_t rp = route(h, p);  // the process that receives what s sends to p
      Member& pm = h->m[rp == NONE ? p : rp];
      // !isInfected(member.id()) (GPI:248): the window gossips p delivered to s during their
      // current state
      std::fill(S.begin(), S.end(), 0ull);
      uint64_t nsupp = 0;
      const auto fit = me.recv.find(p);
      if (fit != me.recv.end())
        for (const Batch& bt : fit->second)
          for (uint32_t j = 0; j < bt.bits.size(); ++j) {
            const uint32_t w = bt.w0 + j;
            if (w < wlo || w >= whi) continue;
            for (uint64_t c = bt.bits[j] & W[w - wlo] & ~S[w - wlo]; c; c &= c - 1) {
              const uint32_t g = (w << 6) + (uint32_t)__builtin_ctzll(c);
              // the batch counts for the current GossipState only (created in round inf - 1); a
              // delayed message counts from the round it arrived in (before this round's sends)
              if (!not_lost(p, s, g, bt.tick)) continue;
              const int64_t arrive = bt.t + delay_rounds(bt.dmean, p, s, g, bt.tick);
              if (arrive < me.gossips.inf[g & (h->rc - 1)] - 1 || arrive >= r) continue;
              S[w - wlo] |= 1ull << (g & 63);
              ++nsupp;
            }
          }
      uint64_t nsend = 0;
      for (uint32_t k = 0; k < nw; ++k) nsend += (uint64_t)__builtin_popcountll(W[k] & ~S[k]);
      // one GossipRequest message per gossip and peer (GPI:225-239), counted for alive peers
      if (pm.alive) {
        h->st.gossip_sends += nsend;
        h->st.infected_suppressed += nsupp;
        h->dbg_send[2 * s] += nsend + nsupp;
        h->dbg_send[2 * s + 1] += nsupp;
        if (s == h->dbg_watch)
          std::fprintf(stderr, "oracle watch r=%lld peer=%u rp=%d send=%llu supp=%llu\n", (long long)r, p, (int)rp,
                       (unsigned long long)nsend, (unsigned long long)nsupp);
      }
      // the link part of delivered(): both alive, no partition cut, no outbound / inbound block
      if (!nsend || !pm.alive || h->loss_bp >= 10000 || !link_ok(h, s, p)) continue;
      Sent st{rp, s, Batch{r, tick, h->delay_mean, 0, {}}};
      uint32_t k0 = 0, k1 = nw;
      while (k0 < k1 && !(W[k0] & ~S[k0])) ++k0;
      while (k1 > k0 && !(W[k1 - 1] & ~S[k1 - 1])) --k1;
      st.b.w0 = wlo + k0;
      for (uint32_t k = k0; k < k1; ++k) {
        const uint64_t eff = W[k] & ~S[k];
        st.b.bits.push_back(eff);
        // first receipts: messages p lacks the gossip of, each with its own loss draw; with
        // delays every message that is not lost and arrives in a later round travels (p may have
        // swept the gossip by then, and the message adds s to p's infectedFrom when it arrives)
        const uint64_t held = held_word(h, pm, wlo + k);
        for (uint64_t cand = h->delay_mean ? eff : eff & ~held; cand; cand &= cand - 1) {
          const uint32_t g = ((wlo + k) << 6) + (uint32_t)__builtin_ctzll(cand);
          if (!not_lost(s, rp, g, tick)) continue;
          const uint32_t dr = delay_rounds(h->delay_mean, s, rp, g, tick);
          if (dr) {
            h->flights.push_back({r + (int64_t)dr, rp, s, g});
            h->registry[g].inflight++;
          } else if (!((held >> (g & 63)) & 1u)) {
            deliveries.push_back({rp, g});
          }
        }
      }
      sent.push_back(std::move(st));
    }
  }
  // delayed messages arriving this round, at a receiver still running
  if (!h->flights.empty()) {
    size_t o = 0;
    for (size_t k = 0; k < h->flights.size(); ++k) {
      const auto& fl = h->flights[k];
      if (fl.arrive != r) {
        h->flights[o++] = fl;
        continue;
      }
      h->registry[fl.gid].inflight--;
      if (h->m[fl.to].alive) deliveries.push_back({fl.to, fl.gid});
    }
    h->flights.resize(o);
  }
  // onGossipReq (GPI:171-183): a new id starts a GossipState with infectionPeriod = r + 1
  for (const Delivery& d : deliveries) {
    Member& pm = h->m[d.to];
    if (gossip_held(h, pm, d.gid)) continue;  // an earlier message of this round brought it
    gossip_put(h, pm, d.gid, r + 1);
    h->st.gossip_first_receipts++;
    const Gossip& g = h->registry[d.gid];
    if (g.subject >= h->N) {  // a user gossip (oracle_spread): GossipProtocol.listen() gets it (GPI:176)
      emit_event(h, d.to, g.subject - h->N, SWIM_EV_GOSSIP, SWIM_R_MEMBERSHIP_GOSSIP, phase, g.record);
      continue;
    }
    h->inbox[d.to].push_back({g.subject, g.record});  // sink.next -> onMembershipGossip, batched
  }
  // ... and addToInfected(from) for every message (GPI:181)
  for (Sent& st : sent) h->m[st.to].recv[st.from].push_back(std::move(st.b));
  if (q + 1 == h->G) {  // batches that can no longer suppress a send
    const int64_t keep = r + 1 - h->hzn - (int64_t)h->dmax_rounds;  // a delayed message arrives late
    for (auto& mm : h->m)
      for (auto it = mm.recv.begin(); it != mm.recv.end();) {
        auto& v = it->second;
        v.erase(std::remove_if(v.begin(), v.end(), [&](const Batch& x) { return x.t < keep; }), v.end());
        it = v.empty() ? mm.recv.erase(it) : std::next(it);
      }
  }
  // membership apply of the first receipts (MPI:407-414 -> updateMembership MEMBERSHIP_GOSSIP)
  for (uint32_t p = 0; p < h->N; ++p) {
    if (h->inbox[p].empty()) continue;
    const uint32_t snap = h->m[p].others;
    // the lattice max per subject, subjects in ascending order
    auto& in = h->inbox[p];
    std::sort(in.begin(), in.end());
    size_t o = 0;
    for (size_t k = 0; k < in.size(); ++k) {
      if (o && in[o - 1].first == in[k].first)
        in[o - 1].second = in[k].second;  // sorted: the later record is the larger
      else
        in[o++] = in[k];
    }
    in.resize(o);
    for (auto& kv : in)
      update_membership(h, p, kv.first, kv.second, SWIM_R_MEMBERSHIP_GOSSIP, phase, 0, tick, snap, r + 1);
    h->inbox[p].clear();
  }
  // a leaving member whose DEAD gossip was swept this round shuts down (ClusterImpl.java:376-388)
  for (uint32_t i = 0; i < h->N; ++i)
    if (h->m[i].stop) {
      h->m[i].stop = false;
      stop_member(h, i);
    }
  finish_phase(h);
}

// ---------------------------------------------------------------------------------------
// Suspicion timeouts (MPI:637-647).
// ---------------------------------------------------------------------------------------
void suspicion_phase(oracle_handle* h) {
  const uint32_t phase = h->G + 1;
  const uint32_t tick = tick_of(h, phase);
  for (uint32_t i = 0; i < h->N; ++i) {
    Member& me = h->m[i];
    if (!me.alive) continue;
    std::vector<uint32_t> due;
    for (auto& kv : me.timers)
      if (kv.second <= h->period) due.push_back(kv.first);
    const uint32_t snap = me.others;
    for (uint32_t subj : due) {
      me.timers.erase(subj);  // MPI:638
      if (me.table[subj] != SWIM_ABSENT) {  // MPI:639-645: DEAD with the record's incarnation
        h->st.suspicion_timeouts++;
        update_membership(h, i, subj, SWIM_DEAD, SWIM_R_SUSPICION_TIMEOUT, phase, 0, tick, snap,
                          (int64_t)(h->period + 1) * h->G);
      }
    }
  }
  finish_phase(h);
}

// ---------------------------------------------------------------------------------------
// SYNC anti-entropy: doSync (MPI:304-320), selectSyncAddress (MPI:416-427), onSync
// (MPI:352-373), onSyncAck (MPI:343-349), syncMembership (MPI:463-473).
// ---------------------------------------------------------------------------------------
// selectSyncAddress: uniform over the set of addresses seeds U otherMembers' addresses (MPI:417-425),
// by rejection sampling over address ids (address x = the one of member x; seed addresses are those
// of members [0, n_seeds); the own address is never a seed, MPI:166-172).
bool select_sync_address(oracle_handle* h, uint32_t i, uint32_t tick, uint32_t* out) {
  const Member& me = h->m[i];
  const uint32_t own = h->addr[i];
  const uint32_t nseeds = std::min<uint32_t>(h->cfg.n_seeds, h->N);
  // MPI:421-422: nothing to pick when no other member is known and no seed address is not our own
  if (me.others == 0 && (nseeds == 0 || (nseeds == 1 && own == 0))) return false;
  auto valid = [&](uint32_t x) {
    if (x == own || h->addr[x] != x) return false;  // own address / an id that moved to another address
    if (x < nseeds) return true;
    if (me.table[x] != SWIM_ABSENT) return true;
    for (uint32_t y : h->movers[x])  // members restarted on address x
      if (y != i && me.table[y] != SWIM_ABSENT) return true;
    return false;
  };
  uint32_t x = 0;
  for (uint32_t a = 0; a < 64; ++a) {
    x = (uint32_t)(((uint64_t)draw(h->seed, K_SYNC_PICK, i, a, 0, tick) * h->N) >> 32);
    if (valid(x)) {
      *out = x;
      return true;
    }
  }
  for (uint32_t d = 1; d <= h->N; ++d) {
    uint32_t y = (uint32_t)(((uint64_t)x + d) % h->N);
    if (valid(y)) {
      *out = y;
      return true;
    }
  }
  return false;
}

void sync_phase(oracle_handle* h) {
  const uint32_t ph_sync = h->G + 2, ph_ack = h->G + 3;
  const uint32_t tick_s = tick_of(h, ph_sync), tick_a = tick_of(h, ph_ack);
  const int64_t create_round = (int64_t)(h->period + 1) * h->G;
  std::vector<SyncReq> reqs;
  for (uint32_t i = 0; i < h->N; ++i) {
    Member& me = h->m[i];
    if (!me.alive) {
      me.sync_fd = 0xFFFFFFFFu;
      continue;
    }
    uint32_t peer;
    if (h->joining[i]) {  // start0 (MPI:222-257): SYNC to every seed address; no periodic doSync yet
      for (uint32_t s = 0; s < h->cfg.n_seeds && s < h->N; ++s)
        if (s != h->addr[i]) reqs.push_back({i, s, 2});
    } else if ((uint32_t)(h->period % h->S) == i % h->S && select_sync_address(h, i, tick_s, &peer)) {
      reqs.push_back({i, peer, 0});
    }
    if (me.sync_fd != 0xFFFFFFFFu) reqs.push_back({i, me.sync_fd, 1});
    me.sync_fd = 0xFFFFFFFFu;
  }
  h->st.syncs_sent += reqs.size();
  // prepareSyncDataMsg (MPI:457-461): every SYNC carries its sender's table as of phase start.
  std::map<uint32_t, std::vector<uint32_t>> snap;
  for (auto& rq : reqs)
    if (!snap.count(rq.from)) snap[rq.from] = h->m[rq.from].table;
  // onSync at each receiver, requests in (receiver, sender, kind) order.
  std::vector<size_t> order(reqs.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = i;
  // receivers: the processes at the addressed members' addresses
  std::vector<uint32_t> recv(reqs.size());
  for (size_t k = 0; k < reqs.size(); ++k) recv[k] = route(h, reqs[k].to);
  std::sort(order.begin(), order.end(), [&](size_t a, size_t b) {
    if (recv[a] != recv[b]) return recv[a] < recv[b];
    if (reqs[a].from != reqs[b].from) return reqs[a].from < reqs[b].from;
    return reqs[a].kind < reqs[b].kind;
  });
  struct Ack {
    uint32_t responder, to, kind, seed;
    std::vector<uint32_t> table;
  };
  std::vector<Ack> acks;
  for (size_t oi : order) {
    const SyncReq& rq = reqs[oi];
    if (!delivered(h, K_SYNC, rq.from, rq.to, rq.kind, tick_s)) continue;
    h->st.syncs_delivered++;
    const uint32_t rcv = recv[oi];
    Member& me = h->m[rcv];
    const uint32_t others_snap = me.others;  // phase-start count (delta deferred)
    const std::vector<uint32_t>& data = snap[rq.from];
    const uint32_t attempt = sync_attempt(rq.from, rq.kind);
    for (uint32_t c = 0; c < h->N; ++c)  // syncMembership (MPI:468-471), reason SYNC
      if (data[c] != SWIM_ABSENT)
        update_membership(h, rcv, c, data[c], SWIM_R_SYNC, ph_sync, attempt, tick_s, others_snap, create_round);
    // MPI:357-371: reply SYNC_ACK with the table after the merge (to the sender's address)
    if (delivered(h, K_SYNC_ACK, rcv, rq.from, rq.kind, tick_a)) acks.push_back({rcv, rq.from, rq.kind, rq.to, me.table});
  }
  finish_phase(h);
  // start0 takes the first initial SyncAck only (take(1), MPI:244-247): canonically the lowest seed
  // address whose round trip was delivered; the others are dropped unprocessed (MPI:330-333)
  std::vector<uint32_t> first_seed(h->N, NONE);
  for (auto& ak : acks)
    if (ak.kind == 2) first_seed[ak.to] = std::min(first_seed[ak.to], ak.seed);
  acks.erase(std::remove_if(acks.begin(), acks.end(),
                            [&](const Ack& a) { return a.kind == 2 && a.seed != first_seed[a.to]; }),
             acks.end());
  // onSyncAck at each requester (MPI:343-349), acks in (requester, responder, kind) order.
  std::sort(acks.begin(), acks.end(), [](const Ack& a, const Ack& b) {
    if (a.to != b.to) return a.to < b.to;
    if (a.responder != b.responder) return a.responder < b.responder;
    return a.kind < b.kind;
  });
  for (auto& ak : acks) {
    h->st.sync_acks_delivered++;
    Member& me = h->m[ak.to];
    const uint32_t attempt = sync_attempt(ak.responder, ak.kind);
    const uint32_t reason = ak.kind == 2 ? SWIM_R_INITIAL_SYNC : SWIM_R_SYNC;  // MPI:463-473 (onStart)
    const uint32_t others_snap = me.others;
    for (uint32_t c = 0; c < h->N; ++c)
      if (ak.table[c] != SWIM_ABSENT)
        update_membership(h, ak.to, c, ak.table[c], reason, ph_ack, attempt, tick_a, others_snap, create_round);
  }
  for (uint32_t i = 0; i < h->N; ++i) h->joining[i] = 0;
  finish_phase(h);
}

void step_period(oracle_handle* h) {
  // phase 0: failure detector (FDI:126), one probe per alive member
  for (uint32_t i = 0; i < h->N; ++i)
    if (h->m[i].alive) do_ping(h, i);
  finish_phase(h);
  // phases 1..G: gossip rounds (GPI:139)
  for (uint32_t q = 0; q < h->G; ++q) gossip_round(h, q);
  // phase G+1: suspicion timeouts
  suspicion_phase(h);
  // phases G+2, G+3: SYNC / SYNC_ACK
  sync_phase(h);
  h->period++;
  h->st.period = h->period;
}

}  // namespace

extern "C" {

int oracle_create(const swim_config* cfg, oracle_handle** out) {
  if (!cfg || !out) return SWIM_EINVAL;
  if (cfg->n_members < 1 || cfg->n_members > (1u << 24) || cfg->ping_interval_ms <= 0 || cfg->gossip_interval_ms <= 0 ||
      cfg->gossip_fanout < 1 || cfg->sync_interval_ms <= 0 || cfg->shard_world > 1)  // one unsharded replay
    return SWIM_EINVAL;
  oracle_handle* h = new (std::nothrow) oracle_handle();
  if (!h) return SWIM_ENOMEM;
  h->cfg = *cfg;
  h->N = cfg->n_members;
  h->G = (uint32_t)std::max(1, cfg->ping_interval_ms / cfg->gossip_interval_ms);
  h->S = (uint32_t)std::max(1, cfg->sync_interval_ms / cfg->ping_interval_ms);
  h->TPP = h->G + 4;
  h->sweepmax = periods_to_sweep(cfg->gossip_repeat_mult, (int32_t)cfg->n_members) + 1;  // others + 1 <= N
  h->hzn = periods_to_spread(cfg->gossip_repeat_mult, (int32_t)cfg->n_members) + 1;
  h->seed = cfg->seed;
  h->group.assign(h->N, 0);
  std::memset(&h->st, 0, sizeof h->st);
  const uint32_t n0 = cfg->n_initial ? cfg->n_initial : cfg->n_members;
  if (n0 > h->N || n0 < 1) {
    delete h;
    return SWIM_EINVAL;
  }
  try {
    h->m.resize(h->N);
    for (uint32_t i = 0; i < h->N; ++i) {
      // converged start: members [0, n0) hold each other ALIVE inc 0; spare slots are in no table
      h->m[i].table.assign(h->N, SWIM_ABSENT);
      std::fill(h->m[i].table.begin(), h->m[i].table.begin() + n0, SWIM_PACK(0, SWIM_ALIVE));
      h->m[i].others = n0 - 1;
      h->m[i].alive = i < n0;
      h->m[i].meta.assign(h->N, 0);  // the converged start shares every member's initial metadata
      h->m[i].gossips.held.assign(h->rc / 64, 0);
      h->m[i].gossips.win.assign(h->rc / 64, 0);
      h->m[i].gossips.inf.assign(h->rc, 0);
    }
    h->inbox.resize(h->N);
    h->pres.assign(h->N, 0);
    std::fill(h->pres.begin(), h->pres.begin() + n0, n0 - 1);
    h->last_removed.assign(h->N, 0);
    h->meta_cur.assign(h->N, 0);
    h->dbg_send.assign(2ull * h->N, 0);
    if (const char* w = std::getenv("SWIMHIP_DEBUG_WATCH")) h->dbg_watch = (uint32_t)std::strtoul(w, nullptr, 10);
    h->addr.resize(h->N);
    h->occ.assign(h->N, NONE);
    for (uint32_t i = 0; i < h->N; ++i) h->addr[i] = i;
    for (uint32_t i = 0; i < n0; ++i) h->occ[i] = i;
    h->movers.resize(h->N);
    h->started.assign(h->N, 0);
    std::fill(h->started.begin(), h->started.begin() + n0, 1);
    h->joining.assign(h->N, 0);
  } catch (...) {
    delete h;
    return SWIM_ENOMEM;
  }
  *out = h;
  return SWIM_OK;
}

int oracle_destroy(oracle_handle* h) {
  delete h;
  return SWIM_OK;
}

int oracle_set_loss(oracle_handle* h, uint32_t loss_bp) {
  if (!h || loss_bp > 10000) return SWIM_EINVAL;
  h->loss_bp = loss_bp;
  return SWIM_OK;
}

// NetworkEmulator.setDefaultOutboundSettings(loss, meanDelay) (NE:81-84) of every member: the mean
// delay part. The threshold table: dthr[k] = ceil(2^32 * (1 - exp(-k / mean))).
int oracle_set_delay(oracle_handle* h, uint32_t mean_ms) {
  if (!h || mean_ms > 60000) return SWIM_EINVAL;
  h->delay_mean = mean_ms;  // messages already sent keep their arrival rounds (Batch::dmean, flights)
  if (!mean_ms || h->dthr.count(mean_ms)) return SWIM_OK;
  std::vector<uint32_t>& t = h->dthr[mean_ms];
  for (uint32_t k = 0;; ++k) {
    const double v = std::ceil(std::ldexp(-std::expm1(-(double)k / (double)mean_ms), 32));
    if (v > 4294967295.0) break;
    t.push_back((uint32_t)v);
  }
  h->dmax_rounds = std::max(h->dmax_rounds, (uint32_t)(t.size() - 1) / (uint32_t)h->cfg.gossip_interval_ms);
  return SWIM_OK;
}

int oracle_set_partition(oracle_handle* h, const uint8_t* group, uint32_t n, uint64_t t0, uint64_t t1) {
  if (!h || !group || n != h->N) return SWIM_EINVAL;
  h->group.assign(group, group + n);
  h->part_t0 = t0;
  h->part_t1 = t1;
  return SWIM_OK;
}

int oracle_block_link(oracle_handle* h, uint32_t src, uint32_t dst, int blocked) {
  if (!h || src >= h->N || dst >= h->N) return SWIM_EINVAL;
  if (h->link.empty()) h->link.assign(((uint64_t)h->N * h->N + 7) / 8, 0);
  uint64_t bit = (uint64_t)src * h->N + dst;
  if (blocked)
    h->link[bit >> 3] |= (uint8_t)(1u << (bit & 7));
  else
    h->link[bit >> 3] &= (uint8_t)~(1u << (bit & 7));
  return SWIM_OK;
}

int oracle_block_inbound(oracle_handle* h, uint32_t dst, uint32_t src, int blocked) {
  if (!h || src >= h->N || dst >= h->N) return SWIM_EINVAL;
  if (h->inlink.empty()) h->inlink.assign(((uint64_t)h->N * h->N + 7) / 8, 0);
  uint64_t bit = (uint64_t)dst * h->N + src;
  if (blocked)
    h->inlink[bit >> 3] |= (uint8_t)(1u << (bit & 7));
  else
    h->inlink[bit >> 3] &= (uint8_t)~(1u << (bit & 7));
  return SWIM_OK;
}

int oracle_crash(oracle_handle* h, const uint32_t* ids, uint32_t n) {
  if (!h || (n && !ids)) return SWIM_EINVAL;
  for (uint32_t k = 0; k < n; ++k) {
    if (ids[k] >= h->N) return SWIM_EINVAL;
    stop_member(h, ids[k]);
  }
  return SWIM_OK;
}

// ClusterImpl.shutdown (ClusterImpl.java:370-408) -> MembershipProtocolImpl.leaveCluster
// (MPI:203-212): the member's own record becomes DEAD (incarnation + 1, which the packed DEAD
// cell does not need: a DEAD record overrides every non-DEAD one and nothing overrides it) and
// is spread as a gossip; the member keeps running until that gossip is swept. Takes effect
// before the next period (the gossip's infectionPeriod is the period's first round).
int oracle_leave(oracle_handle* h, const uint32_t* ids, uint32_t n) {
  if (!h || (n && !ids)) return SWIM_EINVAL;
  for (uint32_t k = 0; k < n; ++k) {
    const uint32_t i = ids[k];
    if (i >= h->N) return SWIM_EINVAL;
    Member& me = h->m[i];
    if (!me.alive || me.leaving) continue;
    me.table[i] = SWIM_DEAD;
    me.leaving = true;
    me.leave_gid = (uint32_t)h->registry.size();
    spread_gossip(h, i, i, SWIM_DEAD, (int64_t)h->period * h->G);
  }
  return SWIM_OK;
}

// Cluster.updateMetadata (ClusterImpl.java:364-367): MetadataStoreImpl.updateMetadata (a new local
// version), then MembershipProtocolImpl.updateIncarnation (MPI:184-196): the own record becomes ALIVE
// with incarnation + 1 and is spread (spreadMembershipGossip: always). Before the next period.
int oracle_update_metadata(oracle_handle* h, const uint32_t* ids, uint32_t n) {
  if (!h || (n && !ids)) return SWIM_EINVAL;
  for (uint32_t k = 0; k < n; ++k)
    if (ids[k] >= h->N) return SWIM_EINVAL;
  for (uint32_t k = 0; k < n; ++k) {
    const uint32_t i = ids[k];
    Member& me = h->m[i];
    if (!me.alive || me.leaving) continue;
    h->meta_cur[i]++;
    const uint32_t r = SWIM_PACK(inc_of(me.table[i]) + 1u, SWIM_ALIVE);
    me.table[i] = r;
    spread_gossip(h, i, i, r, (int64_t)h->period * h->G);
  }
  return SWIM_OK;
}

// A new member starts in spare slot x at address a (ClusterImpl.start, ClusterImpl.java:170-227):
// its table holds only itself ALIVE inc 0 (MPI:138-142), every protocol cursor starts afresh, and
// this period's SYNC phase makes its initial SYNC to the seeds (MPI:222-257).
void start_member(oracle_handle* h, uint32_t x, uint32_t a) {
  Member& me = h->m[x];
  std::fill(me.table.begin(), me.table.end(), SWIM_ABSENT);
  std::fill(me.meta.begin(), me.meta.end(), 0u);
  me.table[x] = SWIM_PACK(0, SWIM_ALIVE);
  me.others = 0;
  me.delta = 0;
  me.timers.clear();
  me.alive = true;
  h->started[x] = 1;
  h->joining[x] = 1;
  h->addr[x] = a;
  h->occ[a] = x;
}

int oracle_join(oracle_handle* h, const uint32_t* ids, uint32_t n) {
  if (!h || (n && !ids)) return SWIM_EINVAL;
  for (uint32_t k = 0; k < n; ++k)
    if (ids[k] >= h->N || h->started[ids[k]] || h->occ[ids[k]] != NONE) return SWIM_EINVAL;
  for (uint32_t k = 0; k < n; ++k) start_member(h, ids[k], ids[k]);
  return SWIM_OK;
}

int oracle_restart(oracle_handle* h, const uint32_t* old_ids, const uint32_t* new_ids, uint32_t n) {
  if (!h || (n && (!old_ids || !new_ids))) return SWIM_EINVAL;
  for (uint32_t k = 0; k < n; ++k) {
    const uint32_t o = old_ids[k], x = new_ids[k];
    if (o >= h->N || x >= h->N || !h->started[o] || h->m[o].alive || h->started[x] ||
        h->occ[h->addr[o]] != NONE)
      return SWIM_EINVAL;
    for (uint32_t q = 0; q < k; ++q)
      if (new_ids[q] == x || h->addr[old_ids[q]] == h->addr[o]) return SWIM_EINVAL;
  }
  for (uint32_t k = 0; k < n; ++k) {
    const uint32_t a = h->addr[old_ids[k]];
    h->movers[a].push_back(new_ids[k]);
    start_member(h, new_ids[k], a);
  }
  return SWIM_OK;
}

// GossipProtocolImpl.spread (GPI:124-128) of a user gossip: created before the next period like a
// leave's gossip; its subject is N + origin (no member), its record the tag
int oracle_spread(oracle_handle* h, uint32_t origin, uint32_t tag) {
  if (!h || origin >= h->N || !h->m[origin].alive) return SWIM_EINVAL;
  spread_gossip(h, origin, h->N + origin, tag, (int64_t)h->period * h->G);
  return SWIM_OK;
}

// A message of an external node (a real JVM member over the wire bridge, swimhip/wire.py) handed
// to member `obs` before the next period: its records go through updateMembership one by one, in
// order, with the message's reason (MPI:463-473 syncMembership for SYNC / SYNC_ACK / INITIAL_SYNC,
// MPI:407-414 onMembershipGossip for a membership gossip). Accepted records spread as gossips
// created for the next period's first round (reason SYNC; MPI:649-656); metadata fetches draw
// with attempt SWIM_DELIVER_ATTEMPT | k in that period's FD tick. A stopped member receives nothing.
int oracle_deliver_records(oracle_handle* h, uint32_t obs, const uint32_t* subj, const uint32_t* rec, uint32_t n,
                           uint32_t reason) {
  if (!h || obs >= h->N || (n && (!subj || !rec))) return SWIM_EINVAL;
  // SWIM_DELIVER_FORWARD: each record is a gossip new to obs; GossipProtocolImpl.onGossipReq
  // (GossipProtocolImpl.java:171-183) puts its GossipState (obs forwards it) before membership sees it
  const bool fwd = (reason & SWIM_DELIVER_FORWARD) != 0u;
  reason &= ~SWIM_DELIVER_FORWARD;
  if (reason != SWIM_R_SYNC && reason != SWIM_R_MEMBERSHIP_GOSSIP && reason != SWIM_R_INITIAL_SYNC) return SWIM_EINVAL;
  if (fwd && reason != SWIM_R_MEMBERSHIP_GOSSIP) return SWIM_EINVAL;
  for (uint32_t k = 0; k < n; ++k)
    if (subj[k] >= h->N || rec[k] == SWIM_ABSENT) return SWIM_EINVAL;
  Member& me = h->m[obs];
  if (!me.alive) return SWIM_OK;
  const uint32_t tick = tick_of(h, 0), snap = me.others;
  for (uint32_t k = 0; k < n; ++k) {
    if (fwd) spread_gossip(h, obs, subj[k], rec[k], (int64_t)h->period * h->G, true);
    update_membership(h, obs, subj[k], rec[k], reason, 0, SWIM_DELIVER_ATTEMPT | k, tick, snap,
                      (int64_t)h->period * h->G);
  }
  finish_phase(h);
  return SWIM_OK;
}

int oracle_trace(oracle_handle* h, uint32_t mask) {
  if (!h) return SWIM_EINVAL;
  h->trace = mask;
  return SWIM_OK;
}

int oracle_step(oracle_handle* h, uint32_t periods) {
  if (!h) return SWIM_EINVAL;
  for (uint32_t p = 0; p < periods; ++p) step_period(h);
  return SWIM_OK;
}

int oracle_drain_events(oracle_handle* h, swim_event* buf, uint64_t cap, uint64_t* n_out) {
  if (!h || !n_out) return SWIM_EINVAL;
  std::stable_sort(h->events.begin(), h->events.end(), [](const swim_event& a, const swim_event& b) {
    if (a.period != b.period) return a.period < b.period;
    if (a.observer != b.observer) return a.observer < b.observer;
    if (a.phase != b.phase) return a.phase < b.phase;
    if (a.subject != b.subject) return a.subject < b.subject;
    if (a.type != b.type) return a.type < b.type;
    if (a.reason != b.reason) return a.reason < b.reason;
    return a.record < b.record;
  });
  uint64_t n = std::min<uint64_t>(cap, h->events.size());
  if (n && buf) std::memcpy(buf, h->events.data(), n * sizeof(swim_event));
  *n_out = n;
  int rc = h->events.size() > cap ? SWIM_EOVERFLOW : SWIM_OK;
  h->events.erase(h->events.begin(), h->events.begin() + (long)n);
  return rc;
}

int oracle_read_view(oracle_handle* h, uint32_t observer, uint32_t* row, uint32_t n) {
  if (!h || !row || observer >= h->N || n != h->N) return SWIM_EINVAL;
  std::memcpy(row, h->m[observer].table.data(), (size_t)n * 4);
  return SWIM_OK;
}

int oracle_read_deadlines(oracle_handle* h, uint32_t observer, uint32_t* row, uint32_t n) {
  if (!h || !row || observer >= h->N || n != h->N) return SWIM_EINVAL;
  std::memset(row, 0, (size_t)n * 4);
  for (auto& kv : h->m[observer].timers) row[kv.first] = (uint32_t)kv.second + 1u;
  return SWIM_OK;
}

int oracle_digest(oracle_handle* h, uint64_t* vd, uint64_t* dd) {
  if (!h) return SWIM_EINVAL;
  uint64_t a = 0, b = 0;
  const uint64_t K = 0x9E3779B97F4A7C15ull;
  for (uint32_t i = 0; i < h->N; ++i) {
    const Member& me = h->m[i];
    for (uint32_t j = 0; j < h->N; ++j)
      if (me.table[j]) a += fmix64(((uint64_t)i * h->N + j) * K + me.table[j]);
    for (auto& kv : me.timers) b += fmix64(((uint64_t)i * h->N + kv.first) * K + (uint32_t)(kv.second + 1));
  }
  if (vd) *vd = a;
  if (dd) *dd = b;
  return SWIM_OK;
}

int oracle_read_presence(oracle_handle* h, uint32_t* present, uint32_t* last_removed, uint32_t n) {
  if (!h || n != h->N) return SWIM_EINVAL;
  if (present) std::memcpy(present, h->pres.data(), (size_t)n * 4);
  if (last_removed) std::memcpy(last_removed, h->last_removed.data(), (size_t)n * 4);
  return SWIM_OK;
}

int oracle_stats_get(oracle_handle* h, swim_stats* out) {
  if (!h || !out) return SWIM_EINVAL;
  *out = h->st;
  out->live_gossip_slots = 0;  // storage detail of the device ring, not modelled here
  uint64_t nc = 0;
  for (uint32_t j = 0; j < h->N; ++j)
    if (!h->m[j].alive) nc += h->pres[j];
  out->not_converged = nc;
  return SWIM_OK;
}

int oracle_debug_holdings(oracle_handle* h, uint32_t member, uint32_t* out_hash, uint32_t* out_inf, uint32_t cap,
                          uint32_t* n_out) {
  if (!h || member >= h->N || !n_out) return SWIM_EINVAL;
  uint32_t n = 0;
  for (uint32_t gid = h->gbase; gid < h->registry.size(); ++gid) {
    const int64_t inf = gossip_find(h, h->m[member], gid);
    if (inf < 0) continue;
    if (n < cap) {
      out_hash[n] = h->registry[gid].hash;
      out_inf[n] = (uint32_t)inf;
    }
    ++n;
  }
  *n_out = n;
  return SWIM_OK;
}

int oracle_debug_sends(oracle_handle* h, uint64_t* out2n, uint32_t n) {
  if (!h || !out2n || n != h->N) return SWIM_EINVAL;
  std::copy(h->dbg_send.begin(), h->dbg_send.end(), out2n);
  return SWIM_OK;
}

int oracle_debug_member_state(oracle_handle* h, uint32_t* out6n, uint32_t n) {
  if (!h || !out6n || n != h->N) return SWIM_EINVAL;
  for (uint32_t i = 0; i < n; ++i) {
    const Member& me = h->m[i];
    out6n[0 * (size_t)n + i] = me.fd_epoch;
    out6n[1 * (size_t)n + i] = me.fd_cursor;
    out6n[2 * (size_t)n + i] = me.g_epoch;
    out6n[3 * (size_t)n + i] = me.g_cursor;
    out6n[4 * (size_t)n + i] = me.gossip_seq;
    out6n[5 * (size_t)n + i] = me.others;
  }
  return SWIM_OK;
}

int oracle_is_overrides(uint32_t r1, uint32_t r0) { return is_overrides(r1, r0) ? 1 : 0; }

uint32_t oracle_philox(uint64_t seed, uint32_t kind, uint32_t a, uint32_t b, uint32_t c, uint32_t tick) {
  return draw(seed, kind, a, b, c, tick);
}

void oracle_philox4(uint64_t seed, uint32_t kind, const uint32_t* abct, uint32_t* out4) {
  const U4 v = draw4(seed, kind, abct[0], abct[1], abct[2], abct[3]);
  for (int i = 0; i < 4; ++i) out4[i] = v.v[i];
}

int64_t oracle_cluster_math(int which, int32_t mult, int32_t n, int32_t fanout) {
  switch (which) {
    case 0:
      return ceil_log2(n);
    case 1:
      return periods_to_spread(mult, n);
    case 2:
      return periods_to_sweep(mult, n);
    case 3:
      return suspicion_periods(mult, n);
    case 4:
      return (int64_t)fanout * mult * ceil_log2(n);  // CM:65-67
    default:
      return -1;
  }
}

uint32_t oracle_perm(uint32_t x, uint32_t n, const uint32_t* keys4) { return perm(x, n, keys4); }

}  // extern "C"

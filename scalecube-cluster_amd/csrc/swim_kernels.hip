// swim_kernels.hip — gfx950 kernels of one SWIM protocol period (dense N x N mode).
//
// Phase order per period, all on one HIP stream, no host round trips:
//   k_fd             FailureDetectorImpl.doPing/doPingReq (FailureDetectorImpl.java:126-209)
//                    + onFailureDetectorEvent (MembershipProtocolImpl.java:376-404)
//   G x { k_gossip_prep, k_gossip_select, k_gossip_send, k_gossip_apply, k_finalize }
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
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < P.N) {
    const int32_t d = P.cnt_delta[i];
    if (d) {
      P.cnt[i] = (uint32_t)((int32_t)P.cnt[i] + d);
      P.cnt_delta[i] = 0;
    }
  }
}

// swim_crash: transport.stop() — presence no longer counted, timers dropped.
__global__ void k_crash(KP P, uint32_t c) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < P.N; j += gridDim.x * blockDim.x) {
    if (j != c && P.view[(size_t)c * P.N + j] != 0u) atomicSub(&P.pres[j], 1u);
    P.dl[(size_t)j * P.N + c] = 0u;
  }
}

// ---------------------------------------------------------------------------------------
// Phase 0: failure detector, one thread per observer.
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_fd(KP P) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t probes = 0, direct = 0, preq = 0, sev = 0, aev = 0, created = 0;
  Tally T;
  if (i < P.N && P.alive[i] && P.cnt[i] > 0u) {
    const uint32_t N = P.N;
    const uint32_t half = perm_half_bits(N);
    const uint32_t* row = P.view + (size_t)i * N;
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
      if (x != i && row[x] != 0u) {
        j = x;
        break;
      }
    }
    P.fd_epoch[i] = ep;
    P.fd_cursor[i] = cur;
    if (j == NONE) {  // member count says >0 but the row holds nobody: invariant broken
      atomicOr(&P.ctl->overflow, OV_BUG);
      j = (i + 1) % N;
    }
    probes = 1;
    // outcome as (nA SUSPECT events, then nB events of status stB) — DESIGN.md §3.3
    uint32_t nA = 0, nB = 0, stB = SWIM_SUSPECT;
    if (delivered(P, K_PING, i, j, 0, P.tick) && delivered(P, K_ACK, j, i, 0, P.tick)) {
      direct = 1;
      nB = 1;
      stB = SWIM_ALIVE;
    } else {
      // selectPingReqMembers (FailureDetectorImpl.java:351-363)
      uint32_t proxies[MAXK];
      uint32_t np = 0;
      if (P.kreq > 0u) {
        const PermKey pk = perm_key(P.seed, K_PROXY_PERM, i, P.period);
        for (uint32_t pos = 0; pos < N && np < P.kreq; ++pos) {
          const uint32_t x = perm_apply(pos, N, half, pk);
          if (x != i && x != j && row[x] != 0u) proxies[np++] = x;
        }
      }
      if (!P.time_left_pos || np == 0) {
        nB = 1;  // FailureDetectorImpl.java:163-165
      } else {
        preq = 1;
        bool any_ok = false;
        for (uint32_t q = 0; q < np; ++q) {
          const uint32_t p = proxies[q];
          if (!delivered(P, K_PING_REQ, i, p, j, P.tick)) {
            ++nA;  // NetworkEmulator send error -> immediate SUSPECT
            continue;
          }
          ++nB;
          if (delivered(P, K_PROXY_PING, p, j, i, P.tick) && delivered(P, K_PROXY_ACK, j, p, i, P.tick) &&
              delivered(P, K_FWD_ACK, p, i, j, P.tick))
            any_ok = true;  // first transit ack completes every pending subscription (cid-only match)
        }
        stB = any_ok ? SWIM_ALIVE : SWIM_SUSPECT;
      }
    }
    // publishPingResult -> onFailureDetectorEvent, sequentially (MembershipProtocolImpl.java:376-404)
    const uint32_t snap = P.cnt[i];
    for (uint32_t e = 0; e < nA + nB; ++e) {
      const uint32_t st = e < nA ? (uint32_t)SWIM_SUSPECT : stB;
      if (st == SWIM_ALIVE)
        ++aev;
      else
        ++sev;
      const uint32_t r0 = row[j];
      if (r0 == 0u || rec_code(r0) == st) continue;
      if (st == SWIM_ALIVE) {
        P.sync_fd[i] = j;
        continue;
      }
      const uint32_t rec = apply_record(P, i, j, SWIM_PACK(rec_inc(r0), SWIM_SUSPECT), SWIM_R_FAILURE_DETECTOR_EVENT, 0u,
                                        snap, T);
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
  add_stat(P, ST_GOSSIPS_CREATED, created);
  flush_tally(P, T);
}

// ---------------------------------------------------------------------------------------
// Gossip round.
// ---------------------------------------------------------------------------------------
__global__ void k_gossip_prep(KP P) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  Ctl* c = P.ctl;
  const uint32_t hi = c->gcount;
  uint32_t lo = c->glo;
  while (lo < hi && (hi - lo > P.GC || P.g_expiry[lo & P.gmask] < P.round)) ++lo;
  c->glo = lo;
  c->scan_lo = lo;
  c->scan_hi = hi;
  c->dirty_count = 0u;
}

// One wave per member m, on the start-of-round state (before any delivery of round r):
// doSpreadGossip's "gossips non-empty" test (GossipProtocolImpl.java:144-146), the peer
// choice selectGossipMembers (:253-274) and the previous round's sweepGossips (:281-304;
// entries with r > infectionPeriod + sweep are cleared so round-r receivers see them absent).
// A gossip swept at the end of round r still counts as held at its start (r-1 <= inf+sweep).
__global__ void __launch_bounds__(256) k_gossip_select(KP P) {
  __shared__ uint32_t s_peers[4][MAXF];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t w = threadIdx.x >> 6;
  const uint32_t m = blockIdx.x * 4u + w;
  const uint32_t N = P.N;
  const uint32_t r = P.round;
  const uint32_t lo = P.ctl->scan_lo, hi = P.ctl->scan_hi;
  const bool active = (m < N) && P.alive[m] && lo < hi;
  uint32_t others = 0;
  bool any_l = false;
  if (active) {
    others = P.cnt[m];
    const uint32_t sweep = sweep_rounds(P, others);
    uint32_t* hrow = P.hold + (size_t)m * P.GC;
    for (uint32_t id = lo + lane; id < hi; id += 64u) {
      const uint32_t s = id & P.gmask;
      const uint32_t e = hrow[s];
      if (e == 0u) continue;
      const uint32_t inf = e - 1u;
      if (inf < P.g_create[s]) continue;  // stale entry of a recycled slot
      if (inf <= r && r <= inf + sweep + 1u) any_l = true;
      if (r > inf + sweep) hrow[s] = 0u;  // sweepGossips (swept by the end of round r-1)
    }
  }
  const bool any = __any(any_l);
  uint32_t np = 0;
  if (active && any) {
    // selectGossipMembers, wave-cooperative: lanes test 64 consecutive positions of the
    // keyed shuffle, ballot, take the first members in position order.
    const uint32_t* row = P.view + (size_t)m * N;
    if (others < P.f) {
      for (uint32_t base = 0; base < N; base += 64u) {
        const uint32_t x = base + lane;
        const bool ok = x < N && x != m && row[x] != 0u;
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
            ok = x != m && row[x] != 0u;
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
  if (m < N && lane == 0) P.npeers[m] = np;
  add_stat(P, ST_G_SCANNED, (active && lane == 0) ? hi - lo : 0u);
}

// One wave per sender m: spreadGossipsTo (GossipProtocolImpl.java:215-251) for the peers chosen
// by k_gossip_select. window = gossips with inf <= r <= inf + periodsToSpread; each goes to each
// peer; the receiver adopts it iff it does not hold it (onGossipReq :171-183), and the first
// receipt does an inbox atomicMax for the membership apply.
__global__ void __launch_bounds__(256) k_gossip_send(KP P) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t w = threadIdx.x >> 6;
  const uint32_t m = blockIdx.x * 4u + w;
  const uint32_t N = P.N;
  const uint32_t r = P.round;
  const uint32_t lo = P.ctl->scan_lo, hi = P.ctl->scan_hi;
  uint32_t sends = 0, receipts = 0, probes = 0;
  const uint32_t np = m < N ? P.npeers[m] : 0u;
  if (np > 0u) {
    uint32_t peers[MAXF];
    uint32_t psweep[MAXF];
    for (uint32_t k = 0; k < np; ++k) {
      peers[k] = P.peers[(size_t)m * P.f + k];
      psweep[k] = P.alive[peers[k]] ? sweep_rounds(P, P.cnt[peers[k]]) : NONE;
    }
    const uint32_t spread = spread_rounds(P, P.cnt[m]);
    const uint32_t* hrow = P.hold + (size_t)m * P.GC;
    for (uint32_t id = lo + lane; id < hi; id += 64u) {
      const uint32_t s = id & P.gmask;
      const uint32_t e = hrow[s];
      if (e == 0u) continue;
      const uint32_t inf = e - 1u;
      const uint32_t create = P.g_create[s];
      if (inf < create || inf > r || r > inf + spread) continue;
      const uint32_t gh = P.g_hash[s];
      for (uint32_t k = 0; k < np; ++k) {
        if (psweep[k] == NONE) continue;  // stopped transport: every message to it is lost
        const uint32_t p = peers[k];
        uint32_t* hp = P.hold + (size_t)p * P.GC + s;
        uint32_t v = *hp;
        ++probes;
        {
          const bool held_start = v != 0u && v - 1u >= create && v - 1u <= r && r <= v - 1u + psweep[k];
          if (!held_start) ++sends;
        }
        bool dl_known = false, dl_ok = false;
        for (uint32_t guard = 0; guard < 64u; ++guard) {
          const bool held_now = v != 0u && v - 1u >= create && r <= v - 1u + psweep[k];
          if (held_now) break;
          if (!dl_known) {
            dl_ok = delivered(P, K_GOSSIP, m, p, gh, P.tick);
            dl_known = true;
          }
          if (!dl_ok) break;
          const uint32_t old = atomicCAS(hp, v, r + 2u);
          if (old == v) {
            ++receipts;
            const uint32_t subj = P.g_subject[s];
            const uint32_t prev = atomicMax(&P.inbox[(size_t)p * N + subj], P.g_record[s]);
            if (prev == 0u) {
              const uint32_t d = atomicAdd(&P.ctl->dirty_count, 1u);
              if (d < P.dcap)
                P.dirty[d] = ((unsigned long long)p << 32) | subj;
              else
                atomicOr(&P.ctl->overflow, OV_DIRTY);
            }
            atomicMax(&P.g_expiry[s], r + 1u + P.sweepmax);
            break;
          }
          v = old;
        }
      }
    }
  }
  add_stat(P, ST_GOSSIP_SENDS, sends);
  add_stat(P, ST_GOSSIP_RECEIPTS, receipts);
  add_stat(P, ST_G_PROBES, probes);
  add_stat(P, ST_G_SCANNED, (np > 0u && lane == 0) ? hi - lo : 0u);
}

// Membership apply of a round's first receipts: onMembershipGossip (MPI:407-414) with the
// lattice max of the records that reached the cell this round.
__global__ void __launch_bounds__(256) k_gossip_apply(KP P) {
  Tally T;
  uint32_t created = 0;
  uint32_t n = P.ctl->dirty_count;
  if (n > P.dcap) n = P.dcap;
  const uint32_t stride = gridDim.x * blockDim.x;
  const uint32_t n_pad = (n + 63u) & ~63u;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n_pad; k += stride) {
    if (k < n) {
      const unsigned long long d = P.dirty[k];
      const uint32_t p = (uint32_t)(d >> 32), subj = (uint32_t)d;
      uint32_t* ip = P.inbox + (size_t)p * P.N + subj;
      const uint32_t r1 = *ip;
      *ip = 0u;
      const uint32_t rec = apply_record(P, p, subj, r1, SWIM_R_MEMBERSHIP_GOSSIP, 0u, P.cnt[p], T);
      if (rec) {  // only onSelfMemberDetected spreads here (reason MEMBERSHIP_GOSSIP)
        emit_gossip(P, p, subj, rec, P.gseq[p]++);
        ++created;
      }
    }
  }
  add_stat(P, ST_GOSSIPS_CREATED, created);
  flush_tally(P, T);
}

// ---------------------------------------------------------------------------------------
// Suspicion timeouts: stream due subject columns of the deadline matrix.
// ---------------------------------------------------------------------------------------
__global__ void k_due(KP P) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < P.N && P.colmin[j] <= P.period) {
    const uint32_t idx = atomicAdd(&P.ctl->due_count, 1u);
    P.due[idx] = j;
  }
}

__global__ void __launch_bounds__(256) k_susp_sweep(KP P) {
  __shared__ uint32_t s_min[4];
  Tally T;
  uint32_t fired = 0;
  const uint32_t n = P.ctl->due_count;
  for (uint32_t k = blockIdx.x; k < n; k += gridDim.x) {
    const uint32_t j = P.due[k];
    uint32_t* col = P.dl + (size_t)j * P.N;
    uint32_t mn = NONE;
    for (uint32_t i = threadIdx.x; i < P.N; i += blockDim.x) {
      const uint32_t v = col[i];
      if (v == 0u) continue;
      if (!P.alive[i]) {
        col[i] = 0u;
        continue;
      }
      const uint32_t dl = v - 1u;
      if (dl <= P.period) {  // onSuspicionTimeout (MembershipProtocolImpl.java:637-647)
        col[i] = 0u;
        if (P.view[(size_t)i * P.N + j] != 0u) {
          ++fired;
          apply_record(P, i, j, SWIM_DEAD, SWIM_R_SUSPICION_TIMEOUT, 0u, P.cnt[i], T);
        }
      } else if (dl < mn) {
        mn = dl;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const uint32_t y = __shfl_xor(mn, o, 64);
      mn = y < mn ? y : mn;
    }
    if ((threadIdx.x & 63u) == 0) s_min[threadIdx.x >> 6] = mn;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t b = s_min[0];
      for (uint32_t q = 1; q < blockDim.x / 64u; ++q) b = s_min[q] < b ? s_min[q] : b;
      P.colmin[j] = b;
    }
    __syncthreads();
  }
  add_stat(P, ST_SUSP_TIMEOUTS, fired);
  add_stat(P, ST_SWEEP_CELLS, threadIdx.x == 0 ? ((n + gridDim.x - 1u - blockIdx.x) / gridDim.x) * P.N : 0u);
  flush_tally(P, T);
}

// ---------------------------------------------------------------------------------------
// SYNC / SYNC_ACK.
// ---------------------------------------------------------------------------------------
// selectSyncAddress (MembershipProtocolImpl.java:416-427): uniform over seeds U others.
__device__ uint32_t select_sync_address(const KP& P, uint32_t i) {
  const uint32_t N = P.N;
  const uint32_t* row = P.view + (size_t)i * N;
  uint32_t count = P.cnt[i];
  for (uint32_t s = 0; s < P.n_seeds && s < N; ++s)
    if (s != i && row[s] == 0u) ++count;
  if (count == 0u) return NONE;
  uint32_t x = 0;
  for (uint32_t a = 0; a < 64u; ++a) {
    x = (uint32_t)(((uint64_t)draw1(P.seed, K_SYNC_PICK, i, a, 0, P.tick) * N) >> 32);
    if (x != i && (row[x] != 0u || x < P.n_seeds)) return x;
  }
  for (uint32_t d = 1; d <= N; ++d) {
    const uint32_t y = (uint32_t)(((uint64_t)x + d) % N);
    if (y != i && (row[y] != 0u || y < P.n_seeds)) return y;
  }
  return NONE;
}

__global__ void k_sync_select(KP P) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t sent = 0, dlv = 0;
  if (i < P.N) {
    P.req_to[2 * i] = NONE;
    P.req_to[2 * i + 1] = NONE;
    P.req_stage[2 * i] = NONE;
    P.req_stage[2 * i + 1] = NONE;
    const uint32_t fdt = P.sync_fd[i];
    P.sync_fd[i] = NONE;
    if (P.alive[i]) {
      uint32_t to[2];
      to[0] = (P.period % P.S == i % P.S) ? select_sync_address(P, i) : NONE;  // doSync (:304-320)
      to[1] = fdt;                                                              // MPI:389-397
      for (uint32_t k = 0; k < 2; ++k) {
        if (to[k] == NONE) continue;
        ++sent;
        P.req_to[2 * i + k] = to[k];
        if (!delivered(P, K_SYNC, i, to[k], k, P.tick)) continue;
        ++dlv;
        const uint32_t slot = atomicAdd(&P.ctl->stage_count, 1u);
        if (slot >= P.scap) {
          atomicOr(&P.ctl->overflow, OV_SYNC);
          continue;
        }
        P.req_stage[2 * i + k] = slot;
        P.stage_req[slot] = 2 * i + k;
        atomicAdd(&P.recv_count[to[k]], 1u);
      }
    }
  }
  add_stat(P, ST_SYNCS_SENT, sent);
  add_stat(P, ST_SYNCS_DELIVERED, dlv);
}

// prepareSyncDataMsg (MembershipProtocolImpl.java:457-461): payload = sender's table at phase start.
__global__ void __launch_bounds__(256) k_sync_snapshot(KP P) {
  uint32_t n = P.ctl->stage_count;
  if (n > P.scap) n = P.scap;
  const uint32_t nv = P.N / 4u;
  for (uint32_t k = blockIdx.x; k < n; k += gridDim.x) {
    const uint32_t from = P.stage_req[k] >> 1;
    const uint4* src = reinterpret_cast<const uint4*>(P.view + (size_t)from * P.N);
    uint4* dst = reinterpret_cast<uint4*>(P.stage_sync + (size_t)k * P.N);
    for (uint32_t c = threadIdx.x; c < nv; c += blockDim.x) dst[c] = src[c];
    for (uint32_t c = nv * 4u + threadIdx.x; c < P.N; c += blockDim.x)
      P.stage_sync[(size_t)k * P.N + c] = P.view[(size_t)from * P.N + c];
  }
}

// exclusive scan of recv_count -> recv_off (single workgroup of 1024)
__global__ void __launch_bounds__(1024) k_scan(KP P) {
  __shared__ uint32_t s_part[1024];
  const uint32_t N = P.N;
  const uint32_t per = (N + 1023u) / 1024u;
  const uint32_t b = threadIdx.x * per;
  uint32_t sum = 0;
  for (uint32_t k = 0; k < per; ++k)
    if (b + k < N) sum += P.recv_count[b + k];
  s_part[threadIdx.x] = sum;
  __syncthreads();
  for (uint32_t o = 1; o < 1024u; o <<= 1) {
    const uint32_t y = threadIdx.x >= o ? s_part[threadIdx.x - o] : 0u;
    __syncthreads();
    s_part[threadIdx.x] += y;
    __syncthreads();
  }
  uint32_t run = s_part[threadIdx.x] - sum;
  for (uint32_t k = 0; k < per; ++k)
    if (b + k < N) {
      P.recv_off[b + k] = run;
      run += P.recv_count[b + k];
    }
  if (threadIdx.x == 1023u) P.recv_off[N] = s_part[1023];
}

__global__ void k_sync_scatter(KP P) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q < 2u * P.N && P.req_stage[q] != NONE) {
    const uint32_t to = P.req_to[q];
    const uint32_t pos = P.recv_off[to] + atomicAdd(&P.recv_fill[to], 1u);
    P.bucket[pos] = q;
  }
}

__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t* total, uint32_t* lds4) {
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
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
                                          uint32_t attempt, uint32_t snap, uint32_t& seq, Tally& T, uint32_t& created,
                                          uint32_t* lds4) {
  const uint32_t N = P.N;
  uint32_t* row = P.view + (size_t)obs * N;
  for (uint32_t c0 = 0; c0 < N; c0 += 256u) {
    const uint32_t c = c0 + threadIdx.x;
    uint32_t rec = 0;
    if (c < N) {
      const uint32_t r1 = src[c];
      if (r1 != 0u) rec = apply_record(P, obs, c, r1, SWIM_R_SYNC, attempt, snap, T);
      if (ack_out) ack_out[c] = row[c];
    }
    if (__syncthreads_or(rec != 0u)) {
      uint32_t total;
      const uint32_t off = block_excl_scan256(rec != 0u ? 1u : 0u, &total, lds4);
      if (rec) {
        emit_gossip(P, obs, c, rec, seq + off);
        ++created;
      }
      seq += total;
    }
  }
}

// onSync (MembershipProtocolImpl.java:352-373) at receiver j = blockIdx, requests in
// (sender, kind) order; each SYNC_ACK payload is j's table right after that request's merge.
__global__ void __launch_bounds__(256) k_sync_merge(KP P) {
  __shared__ uint32_t s_list[BUCKET_MAX];
  __shared__ uint32_t s_lds4[4];
  const uint32_t j = blockIdx.x;
  if (j >= P.N) return;
  uint32_t cntj = P.recv_count[j];
  if (cntj == 0u) return;
  if (cntj > (uint32_t)BUCKET_MAX) {
    if (threadIdx.x == 0) atomicOr(&P.ctl->overflow, OV_BUCKET);
    cntj = BUCKET_MAX;
  }
  const uint32_t off = P.recv_off[j];
  for (uint32_t k = threadIdx.x; k < cntj; k += blockDim.x) s_list[k] = P.bucket[off + k];
  __syncthreads();
  if (threadIdx.x == 0) {  // insertion sort: request index q = 2*sender + kind
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
    const uint32_t q = s_list[k];
    const uint32_t slot = P.req_stage[q];
    merge_row(P, j, P.stage_sync + (size_t)slot * P.N, P.stage_ack + (size_t)slot * P.N, q, snap, seq, T, created,
              s_lds4);
  }
  if (threadIdx.x == 0) P.gseq[j] = seq;
  add_stat(P, ST_MERGE_CELLS, threadIdx.x == 0 ? cntj * P.N : 0u);
  add_stat(P, ST_GOSSIPS_CREATED, created);
  flush_tally(P, T);
}

// onSyncAck (MembershipProtocolImpl.java:343-349) at requester i = blockIdx.
__global__ void __launch_bounds__(256) k_sync_ack(KP P) {
  __shared__ uint32_t s_lds4[4];
  const uint32_t i = blockIdx.x;
  if (i >= P.N) return;
  uint32_t q[2], to[2], n = 0;
  for (uint32_t k = 0; k < 2; ++k) {
    const uint32_t qq = 2 * i + k;
    if (P.req_stage[qq] == NONE) continue;
    const uint32_t t = P.req_to[qq];
    if (!delivered(P, K_SYNC_ACK, t, i, k, P.tick)) continue;
    q[n] = qq;
    to[n] = t;
    ++n;
  }
  if (n == 0) return;
  if (n == 2 && to[1] < to[0]) {  // (responder, kind) order
    uint32_t a = q[0];
    q[0] = q[1];
    q[1] = a;
    a = to[0];
    to[0] = to[1];
    to[1] = a;
  }
  Tally T;
  uint32_t created = 0;
  uint32_t seq = P.gseq[i];
  const uint32_t snap = P.cnt[i];
  for (uint32_t k = 0; k < n; ++k) {
    const uint32_t slot = P.req_stage[q[k]];
    const uint32_t attempt = (to[k] << 1) | (q[k] & 1u);
    merge_row(P, i, P.stage_ack + (size_t)slot * P.N, nullptr, attempt, snap, seq, T, created, s_lds4);
  }
  if (threadIdx.x == 0) P.gseq[i] = seq;
  add_stat(P, ST_ACKS_DELIVERED, threadIdx.x == 0 ? n : 0u);
  add_stat(P, ST_ACK_CELLS, threadIdx.x == 0 ? n * P.N : 0u);
  add_stat(P, ST_GOSSIPS_CREATED, created);
  flush_tally(P, T);
}

// ---------------------------------------------------------------------------------------
// Observability.
// ---------------------------------------------------------------------------------------
__global__ void k_digest(const uint32_t* view, const uint32_t* dl, uint32_t N, unsigned long long* out) {
  const uint64_t K = 0x9E3779B97F4A7C15ull;
  unsigned long long a = 0, b = 0;
  const size_t total = (size_t)N * N;
  for (size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x; x < total; x += (size_t)gridDim.x * blockDim.x) {
    const uint32_t v = view[x];
    if (v) a += fmix64((uint64_t)x * K + v);
    const uint32_t d = dl[x];  // x = subject * N + observer
    if (d) {
      const uint64_t subj = x / N, obs = x % N;
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

__global__ void k_kat_philox(uint64_t seed, uint32_t kind, const uint32_t* abct, uint32_t* out, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = draw1(seed, kind, abct[4 * i], abct[4 * i + 1], abct[4 * i + 2], abct[4 * i + 3]);
}

}  // namespace swim

// swim_rng.h — counter-based randomness and keyed permutations for the device path.
//
// Every random choice of the reference's hot path is a JDK RNG call on a per-member
// scheduler: Collections.shuffle (FailureDetectorImpl.java:346,360; GossipProtocolImpl.java:260;
// MembershipProtocolImpl.java:420), ThreadLocalRandom (FailureDetectorImpl.java:326;
// MembershipProtocolImpl.java:424; NetworkEmulator.java:350). On the GPU each is a pure function
// of (seed, kind, a, b, c, tick) so any lane can evaluate any member's draw in any order:
// Philox4x32-10 with counter {a, b, c, tick} and key {seed_lo ^ kind * 0x9E3779B9, seed_hi}.
// Shuffled member lists become a 4-round Feistel bijection on [0, N) (cycle walking).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace swim {

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

struct u32x4 {
  uint32_t x, y, z, w;
};

__host__ __device__ __forceinline__ u32x4 philox10(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    u32x4 n;
    n.x = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
    n.y = (uint32_t)p1;
    n.z = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
    n.w = (uint32_t)p0;
    c = n;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

__host__ __device__ __forceinline__ u32x4 draw4(uint64_t seed, uint32_t kind, uint32_t a, uint32_t b, uint32_t c,
                                                uint32_t tick) {
  u32x4 ctr = {a, b, c, tick};
  return philox10(ctr, (uint32_t)seed ^ (kind * 0x9E3779B9u), (uint32_t)(seed >> 32));
}

__host__ __device__ __forceinline__ uint32_t draw1(uint64_t seed, uint32_t kind, uint32_t a, uint32_t b, uint32_t c,
                                                   uint32_t tick) {
  return draw4(seed, kind, a, b, c, tick).x;
}

__host__ __device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

__host__ __device__ __forceinline__ uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xFF51AFD7ED558CCDull;
  k ^= k >> 33;
  k *= 0xC4CEB9FE1A85EC53ull;
  k ^= k >> 33;
  return k;
}

// gossip identity hash: reference gossipId = memberId + "-" + gossipCounter
// (GossipProtocolImpl.java:211-213), folded to 32 bits for the loss draw counter.
__host__ __device__ __forceinline__ uint32_t gossip_hash(uint32_t origin, uint32_t seq) {
  return fmix32(origin ^ fmix32(seq + 0x9E3779B9u));
}

// Feistel domain for n: half-width in bits (domain = 4^half >= n).
__host__ __device__ __forceinline__ uint32_t perm_half_bits(uint32_t n) {
  uint32_t bits = 2;
  while ((1ull << bits) < (uint64_t)n) ++bits;
  if (bits & 1) ++bits;
  return bits / 2;
}

struct PermKey {
  uint32_t k[4];
};

__host__ __device__ __forceinline__ PermKey perm_key(uint64_t seed, uint32_t kind, uint32_t member, uint32_t epoch) {
  u32x4 r = draw4(seed, kind, member, epoch, 0, 0);
  PermKey p;
  p.k[0] = r.x;
  p.k[1] = r.y;
  p.k[2] = r.z;
  p.k[3] = r.w;
  return p;
}

// position x of the keyed shuffle of [0, n)
__host__ __device__ __forceinline__ uint32_t perm_apply(uint32_t x, uint32_t n, uint32_t half, const PermKey& key) {
  const uint32_t mask = (1u << half) - 1u;
  do {
    uint32_t L = x >> half, R = x & mask;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t F = fmix32(R ^ key.k[r]) & mask;
      const uint32_t nl = R;
      R = L ^ F;
      L = nl;
    }
    x = (L << half) | R;
  } while (x >= n);
  return x;
}

// inverse of perm_apply: the position of member y in the keyed shuffle. The cycle walk of the
// forward map only passes through values >= n, so walking the inverse rounds back from y stops
// exactly at the position that maps to y.
__host__ __device__ __forceinline__ uint32_t perm_inverse(uint32_t y, uint32_t n, uint32_t half, const PermKey& key) {
  const uint32_t mask = (1u << half) - 1u;
  do {
    uint32_t L = y >> half, R = y & mask;
#pragma unroll
    for (int r = 3; r >= 0; --r) {
      const uint32_t pl = R ^ (fmix32(L ^ key.k[r]) & mask);
      R = L;
      L = pl;
    }
    y = (L << half) | R;
  } while (y >= n);
  return y;
}

// ClusterMath.ceilLog2 (ClusterMath.java:133-135): 32 - numberOfLeadingZeros(num)
__host__ __device__ __forceinline__ uint32_t bitlen(uint32_t v) { return v ? 32u - (uint32_t)__builtin_clz(v) : 0u; }

// packed record helpers (include/swimhip.h)
__host__ __device__ __forceinline__ uint32_t rec_code(uint32_t r) { return r & 3u; }
__host__ __device__ __forceinline__ uint32_t rec_inc(uint32_t r) { return r >> 2; }

// MembershipRecord.isOverrides (MembershipRecord.java:66-84) as one unsigned compare:
// the packed word orders (inc, SUSPECT > ALIVE) and DEAD = 0xFFFFFFFF tops the lattice;
// an absent r0 only accepts ALIVE.
__host__ __device__ __forceinline__ bool is_overrides(uint32_t r1, uint32_t r0) {
  return r0 == 0u ? (r1 != 0xFFFFFFFFu && (r1 & 3u) == 1u) : (r1 > r0);
}

}  // namespace swim

/*
 * swim_oracle.h — C ABI of the CPU oracle (TEST INFRASTRUCTURE ONLY).
 *
 * This library is the checker, never the product: only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it. It is a single-threaded, sequential restatement
 * of scalecube-cluster's protocol logic (reference @ /root/reference) under the discrete
 * replay semantics of DESIGN.md §3. Parity status: isOverrides is pinned by the reference's
 * own known-answer test (MembershipRecordTest.java:46-108) and ClusterMath by its formulas
 * (ClusterMath.java:23-135); the RNG-driven period replay cannot be pinned against the
 * reference (no JDK/Maven in this image) and is pinned by behavioural
 * restatements of FailureDetectorTest / MembershipProtocolTest / GossipProtocolTest plus
 * self-consistency golden fixtures (tests/golden/).
 *
 * The entry points mirror include/swimhip.h one for one (oracle_* <-> swim_*), and take the
 * same swim_config / swim_event / swim_stats structs.
 */
#ifndef SWIM_ORACLE_H
#define SWIM_ORACLE_H

#include <stdint.h>

#include "../include/swimhip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_handle oracle_handle;

int oracle_create(const swim_config* cfg, oracle_handle** out);
int oracle_destroy(oracle_handle* h);
int oracle_set_loss(oracle_handle* h, uint32_t loss_bp);
int oracle_set_delay(oracle_handle* h, uint32_t mean_ms);
int oracle_set_partition(oracle_handle* h, const uint8_t* group, uint32_t n, uint64_t t0, uint64_t t1);
int oracle_block_link(oracle_handle* h, uint32_t src, uint32_t dst, int blocked);
int oracle_block_inbound(oracle_handle* h, uint32_t dst, uint32_t src, int blocked);
int oracle_crash(oracle_handle* h, const uint32_t* ids, uint32_t n);
int oracle_leave(oracle_handle* h, const uint32_t* ids, uint32_t n);
int oracle_update_metadata(oracle_handle* h, const uint32_t* ids, uint32_t n);
int oracle_join(oracle_handle* h, const uint32_t* ids, uint32_t n);
int oracle_restart(oracle_handle* h, const uint32_t* old_ids, const uint32_t* new_ids, uint32_t n);
int oracle_spread(oracle_handle* h, uint32_t origin, uint32_t tag);
int oracle_deliver_records(oracle_handle* h, uint32_t obs, const uint32_t* subj, const uint32_t* rec, uint32_t n,
                           uint32_t reason);
int oracle_trace(oracle_handle* h, uint32_t mask);
int oracle_step(oracle_handle* h, uint32_t periods);
int oracle_drain_events(oracle_handle* h, swim_event* buf, uint64_t cap, uint64_t* n_out);
int oracle_read_view(oracle_handle* h, uint32_t observer, uint32_t* row, uint32_t n);
int oracle_read_deadlines(oracle_handle* h, uint32_t observer, uint32_t* row, uint32_t n);
int oracle_digest(oracle_handle* h, uint64_t* view_digest, uint64_t* deadline_digest);
int oracle_read_presence(oracle_handle* h, uint32_t* present, uint32_t* last_removed, uint32_t n);
int oracle_stats_get(oracle_handle* h, swim_stats* out);

int oracle_debug_holdings(oracle_handle* h, uint32_t member, uint32_t* out_hash, uint32_t* out_inf, uint32_t cap,
                          uint32_t* n_out);

int oracle_debug_member_state(oracle_handle* h, uint32_t* out6n, uint32_t n);
int oracle_debug_sends(oracle_handle* h, uint64_t* out2n, uint32_t n);

/* Pure helpers (known-answer tests). */
int oracle_is_overrides(uint32_t r1, uint32_t r0);
uint32_t oracle_philox(uint64_t seed, uint32_t kind, uint32_t a, uint32_t b, uint32_t c, uint32_t tick);
void oracle_philox4(uint64_t seed, uint32_t kind, const uint32_t* abct, uint32_t* out4);
/* ClusterMath (ClusterMath.java): which = 0 ceilLog2, 1 gossipPeriodsToSpread,
 * 2 gossipPeriodsToSweep, 3 suspicionTimeout (periods), 4 maxMessagesPerGossipPerNode. */
int64_t oracle_cluster_math(int which, int32_t mult, int32_t n, int32_t fanout);
uint32_t oracle_perm(uint32_t x, uint32_t n, const uint32_t* keys4);

#ifdef __cplusplus
}
#endif

#endif

// asan_driver.cpp — TEST INFRASTRUCTURE: drives the CPU oracle through every entry point under
// AddressSanitizer + UBSan (`make -C oracle asan-run`), so the checker itself is memory-safe.
// A standalone executable (the sanitizer runtime is linked in; no preloading into a Python host).
// Covers: crash, loss, partition, outbound / inbound blocks, leave, join, restart, metadata
// updates, user gossips, the FD trace, message delays, events, views, deadlines, presence, digests.
#include <cstdio>
#include <cstring>
#include <vector>

#include "swim_oracle.h"

namespace {

int fails = 0;

void check(int rc, const char* what) {
  if (rc != SWIM_OK) {
    std::fprintf(stderr, "asan_driver: %s returned %d\n", what, rc);
    ++fails;
  }
}

swim_config local_config(uint32_t n, uint32_t n_initial, uint64_t seed) {
  swim_config c;
  std::memset(&c, 0, sizeof c);
  c.n_members = n;
  c.seed = seed;
  c.ping_interval_ms = 1000;
  c.ping_timeout_ms = 200;
  c.ping_req_members = 1;
  c.gossip_fanout = 3;
  c.gossip_interval_ms = 100;
  c.gossip_repeat_mult = 2;
  c.sync_interval_ms = 15000;
  c.sync_timeout_ms = 3000;
  c.suspicion_mult = 3;
  c.metadata_timeout_ms = 1000;
  c.n_seeds = 3;
  c.event_capacity = 1u << 16;
  c.n_initial = n_initial;
  return c;
}

void drain_and_read(oracle_handle* h, uint32_t n) {
  std::vector<swim_event> ev(1u << 16);
  uint64_t got = 0;
  check(oracle_drain_events(h, ev.data(), ev.size(), &got), "drain_events");
  std::vector<uint32_t> row(n), pres(n), last(n);
  for (uint32_t i = 0; i < n; i += 7) {
    check(oracle_read_view(h, i, row.data(), n), "read_view");
    check(oracle_read_deadlines(h, i, row.data(), n), "read_deadlines");
  }
  check(oracle_read_presence(h, pres.data(), last.data(), n), "read_presence");
  uint64_t vd = 0, dd = 0;
  check(oracle_digest(h, &vd, &dd), "digest");
  swim_stats st;
  check(oracle_stats_get(h, &st), "stats_get");
}

}  // namespace

int main() {
  const uint32_t n = 96, n0 = 80;
  for (uint32_t delay : {0u, 150u}) {
    swim_config cfg = local_config(n, n0, 7 + delay);
    oracle_handle* h = nullptr;
    check(oracle_create(&cfg, &h), "create");
    if (!h) return 1;
    check(oracle_trace(h, SWIM_TRACE_FD), "trace");
    check(oracle_set_loss(h, 500), "set_loss");
    check(oracle_set_delay(h, delay), "set_delay");
    check(oracle_step(h, 3), "step");
    const uint32_t crash[] = {5, 17, 40};
    check(oracle_crash(h, crash, 3), "crash");
    check(oracle_block_link(h, 1, 2, 1), "block_link");
    check(oracle_block_inbound(h, 9, 3, 1), "block_inbound");
    std::vector<uint8_t> group(n);
    for (uint32_t i = 0; i < n; ++i) group[i] = (uint8_t)(i % 2);
    check(oracle_set_partition(h, group.data(), n, 5, 9), "set_partition");
    check(oracle_spread(h, 0, 0xABCDu), "spread");
    const uint32_t upd[] = {3, 30};
    check(oracle_update_metadata(h, upd, 2), "update_metadata");
    // a real node's SYNC and a forwarded membership gossip (the wire bridge)
    const uint32_t subj[] = {2, 7, 11, 12}, recs[] = {SWIM_PACK(0, SWIM_SUSPECT), SWIM_PACK(2, SWIM_ALIVE), SWIM_DEAD,
                                                      SWIM_PACK(1, SWIM_SUSPECT)};
    check(oracle_deliver_records(h, 12, subj, recs, 4, SWIM_R_SYNC), "deliver_records sync");
    check(oracle_deliver_records(h, 20, subj, recs, 2, SWIM_R_MEMBERSHIP_GOSSIP | SWIM_DELIVER_FORWARD),
          "deliver_records forward");
    check(oracle_step(h, 6), "step");
    const uint32_t leave[] = {60};
    check(oracle_leave(h, leave, 1), "leave");
    const uint32_t old_ids[] = {5}, new_ids[] = {80}, joiners[] = {81, 82};
    check(oracle_restart(h, old_ids, new_ids, 1), "restart");
    check(oracle_join(h, joiners, 2), "join");
    check(oracle_step(h, 25), "step");
    drain_and_read(h, n);
    check(oracle_destroy(h), "destroy");
  }
  std::printf("asan_driver: %s\n", fails ? "FAILED" : "OK");
  return fails ? 1 : 0;
}

// ctl_msan.cpp — TEST HARNESS: a stand-alone driver of ctl_host.cpp (the control step compiled for
// the CPU) for MemorySanitizer, which needs an executable, not a library loaded into Python. It
// runs the step over bootstrap, an election, steady full batches, message loss, isolation and
// membership changes, with and without the fast path and the remote inbox (wire_all), and MSan
// reports any branch, address or store that depends on a value the step never initialised
// (a register that holds whatever the previous code left in it on the GPU).
#include "ctl_host.cpp"

#include <cstdio>
#include <cstdlib>

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint32_t rnd() {
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 7;
  rng_state ^= rng_state << 17;
  return (uint32_t)rng_state;
}

static void scenario(uint32_t G, uint32_t R, uint32_t L, uint32_t P, uint32_t E, uint32_t SE, uint32_t drop_ppm,
                     int fast, int wire, int ticks, int chaos) {
  rg_config c{};
  c.groups = G; c.replicas = R; c.log_capacity = L; c.payload_bytes = P; c.max_entries_per_msg = E;
  c.max_msgs_per_pair = 8; c.num_slabs = 2; c.election_rtt = 10; c.heartbeat_rtt = 1; c.check_quorum = 1;
  c.snapshot_entries = SE; c.compaction_overhead = 5; c.drop_ppm = drop_ppm; c.seed = 0xC3 + R;
  c.ranks = 1; c.wire_all = (uint32_t)wire;
  void* h = ch_create(&c);
  ch_set_fast(h, fast);
  ch_bootstrap(h);
  std::vector<uint8_t> pt(G), camp(G * R), iso(G * R);
  std::vector<uint32_t> pc(G);
  for (int t = 0; t < ticks; ++t) {
    rg_tick_input in{};
    for (uint32_t g = 0; g < G; ++g) {
      pt[g] = t >= 6 ? (chaos ? (uint8_t)(rnd() % (R + 1) == R ? 0xFF : rnd() % R) : 0) : 0xFF;
      pc[g] = chaos ? 1 + rnd() % E : E;
    }
    for (uint32_t i = 0; i < G * R; ++i) {
      camp[i] = (t == 1 && i % R == 0) || (chaos && rnd() % 64 == 0);
      iso[i] = chaos && rnd() % 20 == 0;
    }
    if (chaos && t % 7 == 3 && R > 2)
      for (uint32_t g = 0; g < G; ++g)
        if (rnd() % 4 == 0) ch_config_change(h, g, rnd() % R, rnd() % 2 ? RG_CC_REMOVE : RG_CC_ADD, rnd() % R);
    in.prop_target = pt.data();
    in.prop_count = pc.data();
    in.campaign = camp.data();
    in.isolate = iso.data();
    if (ch_tick(h, &in) != 0) {
      fprintf(stderr, "ch_tick failed\n");
      exit(1);
    }
  }
  rg_replica_view v;
  ch_read_replica(h, 0, &v);
  if (!chaos && v.committed < (uint64_t)(ticks - 8) * E) {  // the steady run replicated every batch
    fprintf(stderr, "R %u fast %d wire %d: committed %llu\n", R, fast, wire, (unsigned long long)v.committed);
    exit(1);
  }
  if (getenv("CTL_MSAN_PROBE")) {  // the sanitizer is live: branch on an uninitialised value
    uint64_t* junk = (uint64_t*)malloc(16);
    if (junk[1] == 42) puts("?");
    free(junk);
  }
  ch_destroy(h);
}

int main() {
  const uint32_t Rs[] = {1, 2, 3, 5, 8};
  for (uint32_t R : Rs)
    for (int fast = 0; fast < 3; ++fast)
      for (int wire = 0; wire < 2; ++wire) {
        scenario(16, R, 512, 256, 64, 200, 0, fast, wire, 40, 0);          // C3's shape, steady
        scenario(8, R, 64, 16, 8, 20, 150000, fast, wire, 120, 1);          // chaos
      }
  printf("MSAN-CLEAN\n");
  return 0;
}

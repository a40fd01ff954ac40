// The LPM flat table (maps.cpp LpmTrie::flat) against the trie walk
// (LpmTrie::lookup, the restatement of lpm_trie_map.cpp:192-264) on random
// IPv4 route sets with updates and logical deletions, every /32 of sampled
// /24s and random addresses.  Host-only: built by tests/test_lpm_flat.py.
#include "../../bpftime_amd/csrc/maps.cpp"

#include <random>

// maps.cpp's only references outside itself (the perf-event attach path)
extern "C" int bpftime_amd_syscall_attach_ex(int, int64_t, int) { return -1; }
extern "C" int bpftime_amd_syscall_detach(int) { return -1; }
extern "C" int bpftime_amd_tracepoint_resolve(int32_t, int64_t *, int *) { return -1; }
void bpftime_amd::syscall_detach_all() {}

using bpftime_amd::LpmTrie;

static uint32_t flat_lookup(const std::vector<uint32_t> &t, uint32_t a) {
  uint32_t e = t[a >> 8];
  if (e & 0x80000000u) e = t[(1u << 24) + 256u * (e & 0x7fffffffu) + (a & 0xff)];
  return e;
}

int main() {
  int bad = 0;
  for (int trial = 0; trial < 12; trial++) {
    std::mt19937_64 rng(1000 + trial);
    LpmTrie t;
    t.dsz = 4;
    t.vsz = 4;
    t.max_entries = 6000;
    t.cap = 2 * t.max_entries + 8;
    std::vector<std::pair<uint32_t, uint32_t>> routes;
    const int nr = trial < 4 ? 40 : 3000;
    for (int i = 0; i < nr; i++) {
      static const uint32_t lens[] = {0, 1, 7, 8, 12, 16, 20, 23, 24, 25, 27, 28, 31, 32};
      const uint32_t plen = trial % 2 ? lens[rng() % 14] : 8 + 4 * (rng() % 7);
      uint32_t net = (uint32_t)rng();
      if (trial % 3 == 0 && plen < 32) net &= ~0u << (32 - plen);  // else stray bits beyond the prefix
      routes.push_back({plen, net});
      uint8_t key[8];
      memcpy(key, &plen, 4);
      const uint32_t be = __builtin_bswap32(net);
      memcpy(key + 4, &be, 4);
      const uint32_t v = i + 1;
      t.update(key, &v, 0);
    }
    for (size_t i = 0; i < routes.size(); i += 5) {  // logical deletions, incl. /32s
      uint8_t key[8];
      memcpy(key, &routes[i].first, 4);
      const uint32_t be = __builtin_bswap32(routes[i].second);
      memcpy(key + 4, &be, 4);
      t.remove(key);
    }
    std::vector<uint32_t> ft;
    if (!t.flat(ft, 1u << 16)) {
      printf("trial %d: flat() failed\n", trial);
      return 1;
    }
    auto check = [&](uint32_t a) {
      uint8_t key[8];
      const uint32_t kp = 32, be = __builtin_bswap32(a);
      memcpy(key, &kp, 4);
      memcpy(key + 4, &be, 4);
      const LpmTrie::Node *n = t.lookup(key);
      const uint32_t want = n ? (uint32_t)(n - t.nodes.data()) + 1 : 0;
      const uint32_t got = flat_lookup(ft, a);
      if (got != want && bad++ < 10) printf("trial %d addr %08x: flat %u walk %u\n", trial, a, got, want);
    };
    for (auto &r : routes) {  // around every route: its ends and neighbours
      const uint32_t span = r.first ? (r.first == 32 ? 0 : (~0u >> r.first)) : ~0u;
      const uint32_t base = r.first ? r.second & (~0u << (32 - r.first)) : 0;
      for (uint32_t a : {base, base + span, base - 1, base + span + 1, r.second, base + (uint32_t)(rng() & span)}) check(a);
    }
    for (int i = 0; i < 200000; i++) check((uint32_t)rng());
    for (int s = 0; s < 64; s++) {  // every address of a few /24s holding routes
      const uint32_t b = routes[rng() % routes.size()].second & ~0xffu;
      for (uint32_t k = 0; k < 256; k++) check(b | k);
    }
  }
  printf(bad ? "FAIL %d\n" : "OK\n", bad);
  return bad ? 1 : 0;
}

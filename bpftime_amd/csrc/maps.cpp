// bpftime_amd: device-resident maps and the prog / link records.
//
// Map semantics (syscall side, from_syscall = true) follow
// runtime/src/handler/map_handler.cpp:109-330 over
//   array_map.cpp:19-81, fix_hash_map.cpp:16-84 + bpftime_hash_map.hpp,
//   per_cpu_array_map.cpp:97-145, per_cpu_hash_map.cpp:141-216,
// with storage in one device arena (HBM) whose layout is described by the
// DMap records the interpreter reads (csrc/common.hpp).  Host-side ops copy
// the touched slots over PCIe: they are control-plane operations and must not
// race a running batch (the reference's syscall path likewise takes the map
// lock, map_handler.hpp:45-62).
#include <errno.h>
#include <sys/mman.h>
#include <stdlib.h>
#include <string.h>
#include <set>

#include <algorithm>
#include <functional>
#include <vector>

#include "../../include/bpftime_amd.h"
#include "runtime.hpp"

namespace bpftime_amd {

Runtime &rt() {
  static Runtime *r = new Runtime();
  return *r;
}

void set_error(const std::string &e) { rt().last_error = e; }

static thread_local std::vector<uint8_t> tl_lookup_buf;

int Runtime::ensure_device() {
  if (d_maptab) return 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    set_error("no HIP device");
    return -1;
  }
  device = dev;
  const char *mb = getenv("BPFTIME_AMD_ARENA_MB");
  arena_size = (uint64_t)(mb ? atoll(mb) : 1024) << 20;  // (288 GB of HBM: two 64-MiB staged rings and more fit)
  if (hipMalloc((void **)&arena, arena_size) != hipSuccess) {
    set_error("hipMalloc(arena) failed");
    arena = nullptr;
    return -1;
  }
  if (hipMemset(arena, 0, arena_size) != hipSuccess) return -1;
  if (hipMalloc((void **)&d_maptab, sizeof(DMap) * kMaxFds) != hipSuccess) {
    set_error("hipMalloc(map table) failed");
    return -1;
  }
  if (hipMemset(d_maptab, 0, sizeof(DMap) * kMaxFds) != hipSuccess) return -1;
  arena_used = 0;
  return 0;
}

uint64_t Runtime::arena_alloc(uint64_t bytes) {
  uint64_t off = (arena_used + 255) & ~255ull;
  if (off + bytes > arena_size) return 0;
  arena_used = off + bytes;
  return (uint64_t)(uintptr_t)arena + off;
}

int Runtime::push_map(int fd) {
  return hipMemcpy(d_maptab + fd, &maps[fd].d, sizeof(DMap), hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}

// bpftime_hash_map.hpp:14-38
static uint64_t next_prime(uint64_t n) {
  auto is_prime = [](uint64_t v) {
    if (v <= 1) return false;
    if (v <= 3) return true;
    if (v % 2 == 0 || v % 3 == 0) return false;
    for (uint64_t i = 5; i * i <= v; i += 6)
      if (v % i == 0 || v % (i + 2) == 0) return false;
    return true;
  };
  while (!is_prime(n)) ++n;
  return n;
}

static uint64_t hash_bytes(const void *key, uint32_t n) {
  uint64_t h = 0;
  for (uint32_t i = 0; i < n; i++) h = h * 31 + ((const uint8_t *)key)[i];
  return h;
}

static MapRec *map_of(int fd) {
  Runtime &r = rt();
  if (fd < 0 || fd >= (int)kMaxFds || r.kind[fd] != HKind::MAP) {
    errno = ENOENT;
    return nullptr;
  }
  return &r.maps[fd];
}

static int alloc_fd(int fd) {
  Runtime &r = rt();
  if (fd < 0) {
    for (fd = 3; fd < (int)kMaxFds && r.kind[fd] != HKind::NONE; fd++) {
    }
  }
  if (fd < 0 || fd >= (int)kMaxFds || r.kind[fd] != HKind::NONE) {
    errno = EBADF;
    return -1;
  }
  return fd;
}

// --- device slot helpers (hash maps) ---
static bool read_slot(const MapRec &m, uint64_t idx, std::vector<uint8_t> &buf) {
  buf.resize(m.d.slot_size);
  return hipMemcpy(buf.data(), (void *)(m.d.data + idx * m.d.slot_size), m.d.slot_size,
                   hipMemcpyDeviceToHost) == hipSuccess;
}
static bool write_slot(const MapRec &m, uint64_t idx, const std::vector<uint8_t> &buf) {
  return hipMemcpy((void *)(m.d.data + idx * m.d.slot_size), buf.data(), m.d.slot_size,
                   hipMemcpyHostToDevice) == hipSuccess;
}
static uint64_t read_count(const MapRec &m) {
  uint64_t c = 0;
  hipMemcpy(&c, (void *)m.d.count_addr, 8, hipMemcpyDeviceToHost);
  return c;
}
static void write_count(const MapRec &m, uint64_t c) {
  hipMemcpy((void *)m.d.count_addr, &c, 8, hipMemcpyHostToDevice);
}

// probe like bpftime_hash_map::elem_lookup; returns bucket or -1
static int64_t host_hash_find(const MapRec &m, const void *key, std::vector<uint8_t> &slot,
                              int64_t *first_empty) {
  const uint64_t nb = m.d.nbuckets;
  uint64_t idx = hash_bytes(key, m.key_size) % nb, start = idx;
  if (first_empty) *first_empty = -1;
  do {
    if (!read_slot(m, idx, slot)) return -1;
    uint32_t st;
    memcpy(&st, slot.data(), 4);
    if (st == 0) {
      if (first_empty) *first_empty = (int64_t)idx;
      return -1;
    }
    if (memcmp(slot.data() + m.d.key_off, key, m.key_size) == 0) return (int64_t)idx;
    idx = (idx + 1) % nb;
  } while (idx != start);
  return -1;
}


// ---- LRU hash (runtime/src/bpf_map/userspace/lru_var_hash_map.cpp) ---------
// Host-side operations on the device table (common.hpp DMap LRU_HASH,
// dev_helpers.hpp lru_*): the same probe, tombstones and stamps, with the
// exact eviction of the reference (the smallest stamp over every bucket).
static constexpr uint32_t kStTomb = 3;

static uint64_t lru_host_stamp() { return (rt().lru_seq.fetch_add(1) + 1) << kLruSeqShift; }
static uint64_t lru_stamp_addr(const MapRec &m, uint64_t i) { return m.d.count_addr + 128 + 8 * i; }
static bool lru_write_stamp(const MapRec &m, uint64_t i, uint64_t st) {
  return hipMemcpy((void *)lru_stamp_addr(m, i), &st, 8, hipMemcpyHostToDevice) == hipSuccess;
}
static uint64_t read_word(const MapRec &m, uint64_t off) {
  uint64_t c = 0;
  hipMemcpy(&c, (void *)(m.d.count_addr + off), 8, hipMemcpyDeviceToHost);
  return c;
}
static void write_word(const MapRec &m, uint64_t off, uint64_t c) {
  hipMemcpy((void *)(m.d.count_addr + off), &c, 8, hipMemcpyHostToDevice);
}

// the FILLED bucket holding key or -1; *free_idx = first tombstone / empty
static int64_t lru_host_probe(const MapRec &m, const void *key, std::vector<uint8_t> &slot, int64_t *free_idx) {
  const uint64_t nb = m.d.nbuckets;
  uint64_t idx = hash_bytes(key, m.key_size) % nb, start = idx;
  *free_idx = -1;
  do {
    if (!read_slot(m, idx, slot)) return -1;
    uint32_t st;
    memcpy(&st, slot.data(), 4);
    if (st == 0 || st == kStTomb) {
      if (*free_idx < 0) *free_idx = (int64_t)idx;
      if (st == 0) return -1;
    } else if (st == 1 && memcmp(slot.data() + m.d.key_off, key, m.key_size) == 0) {
      return (int64_t)idx;
    }
    idx = (idx + 1) % nb;
  } while (idx != start);
  return -1;
}

static bool lru_download(const MapRec &m, std::vector<uint8_t> &tab, std::vector<uint64_t> &stamps) {
  tab.resize(m.bytes);
  stamps.resize(m.d.nbuckets);
  return hipMemcpy(tab.data(), (void *)m.d.data, m.bytes, hipMemcpyDeviceToHost) == hipSuccess &&
         hipMemcpy(stamps.data(), (void *)lru_stamp_addr(m, 0), 8 * m.d.nbuckets, hipMemcpyDeviceToHost) ==
             hipSuccess;
}
static uint32_t tab_state(const MapRec &m, const std::vector<uint8_t> &tab, uint64_t i) {
  uint32_t st;
  memcpy(&st, tab.data() + i * m.d.slot_size, 4);
  return st;
}

// evict the list tail (lru_var_hash_map.cpp:66-71): the smallest stamp
static bool lru_host_evict(const MapRec &m) {
  std::vector<uint8_t> tab;
  std::vector<uint64_t> stamps;
  if (!lru_download(m, tab, stamps)) return false;
  int64_t best = -1;
  for (uint64_t i = 0; i < m.d.nbuckets; i++)
    if (tab_state(m, tab, i) == 1 && (best < 0 || stamps[i] < stamps[(uint64_t)best])) best = (int64_t)i;
  if (best < 0) return false;
  const uint32_t t = kStTomb;
  if (hipMemcpy((void *)(m.d.data + (uint64_t)best * m.d.slot_size), &t, 4, hipMemcpyHostToDevice) != hipSuccess)
    return false;
  write_word(m, 0, read_word(m, 0) - 1);
  write_word(m, 8, read_word(m, 8) + 1);
  return true;
}

// rebuild the table without tombstones (elements keep their stamps); with
// `renumber`, the stamps become their ranks (the recency order, below every
// sequence-stamped use)
static int lru_rebuild(const MapRec &m, bool renumber) {
  std::vector<uint8_t> tab, out(m.bytes, 0);
  std::vector<uint64_t> stamps, os(m.d.nbuckets, 0);
  if (!lru_download(m, tab, stamps)) return -1;
  const uint64_t nb = m.d.nbuckets, ss = m.d.slot_size;
  std::vector<uint64_t> live;
  for (uint64_t i = 0; i < nb; i++)
    if (tab_state(m, tab, i) == 1) live.push_back(i);
  if (renumber) {
    std::vector<uint64_t> ord = live;
    std::sort(ord.begin(), ord.end(), [&](uint64_t a, uint64_t b) { return stamps[a] < stamps[b]; });
    for (uint64_t r = 0; r < ord.size(); r++) stamps[ord[r]] = r + 1;
  }
  for (uint64_t i : live) {
    uint64_t j = hash_bytes(tab.data() + i * ss + m.d.key_off, m.key_size) % nb;
    while (tab_state(m, out, j) != 0) j = (j + 1) % nb;
    memcpy(out.data() + j * ss, tab.data() + i * ss, ss);
    os[j] = stamps[i];
  }
  if (hipMemcpy((void *)m.d.data, out.data(), m.bytes, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy((void *)lru_stamp_addr(m, 0), os.data(), 8 * nb, hipMemcpyHostToDevice) != hipSuccess)
    return -1;
  write_word(m, 0, live.size());
  write_word(m, 8, 0);
  return 0;
}

static const void *lru_host_lookup(MapRec &m, const void *key) {  // :27-41
  std::vector<uint8_t> slot;
  int64_t fi;
  const int64_t idx = key ? lru_host_probe(m, key, slot, &fi) : -1;
  if (idx < 0) {
    errno = ENOENT;
    return nullptr;
  }
  if (!lru_write_stamp(m, (uint64_t)idx, lru_host_stamp())) return nullptr;  // move_to_head
  tl_lookup_buf.assign(slot.begin() + m.d.val_off, slot.begin() + m.d.val_off + m.value_size);
  return tl_lookup_buf.data();
}

static long lru_host_update(MapRec &m, const void *key, const void *value, uint64_t flags) {  // :43-90
  if (flags > 2) {  // is_good_update_flag (:8-11): exactly BPF_ANY / BPF_NOEXIST / BPF_EXIST
    errno = EINVAL;
    return -1;
  }
  std::vector<uint8_t> slot;
  int64_t fi;
  int64_t idx = lru_host_probe(m, key, slot, &fi);
  if (flags == 1 && idx >= 0) {
    errno = EEXIST;
    return -1;
  }
  if (flags == 2 && idx < 0) {
    errno = ENOENT;
    return -1;
  }
  if (idx >= 0) {  // a new value, moved to the head
    memcpy(slot.data() + m.d.val_off, value, m.value_size);
    if (!write_slot(m, (uint64_t)idx, slot) || !lru_write_stamp(m, (uint64_t)idx, lru_host_stamp())) return -1;
    return 0;
  }
  if (read_word(m, 0) >= m.max_entries && !lru_host_evict(m)) {
    errno = ENOMEM;
    return -1;
  }
  if (fi < 0) {  // every bucket on the probe is taken: drop the tombstones
    if (lru_rebuild(m, false) < 0) return -1;
    lru_host_probe(m, key, slot, &fi);
    if (fi < 0) {
      errno = ENOMEM;
      return -1;
    }
  }
  std::vector<uint8_t> s(m.d.slot_size, 0);
  read_slot(m, (uint64_t)fi, slot);
  uint32_t was;
  memcpy(&was, slot.data(), 4);
  const uint32_t st = 1;
  memcpy(s.data(), &st, 4);
  memcpy(s.data() + m.d.key_off, key, m.key_size);
  memcpy(s.data() + m.d.val_off, value, m.value_size);
  if (!lru_write_stamp(m, (uint64_t)fi, lru_host_stamp()) || !write_slot(m, (uint64_t)fi, s)) return -1;
  write_word(m, 0, read_word(m, 0) + 1);
  if (was == kStTomb) write_word(m, 8, read_word(m, 8) - 1);
  return 0;
}

static long lru_host_delete(MapRec &m, const void *key) {  // :92-103
  std::vector<uint8_t> slot;
  int64_t fi;
  const int64_t idx = lru_host_probe(m, key, slot, &fi);
  if (idx < 0) {
    errno = ENOENT;
    return -1;
  }
  const uint32_t t = kStTomb;
  memcpy(slot.data(), &t, 4);
  if (!write_slot(m, (uint64_t)idx, slot)) return -1;
  write_word(m, 0, read_word(m, 0) - 1);
  write_word(m, 8, read_word(m, 8) + 1);
  return 0;
}

// :105-135 walks the unordered_map's order (not part of its contract: the
// reference's tests compare visited sets); this walks buckets.  A key that
// is not present restarts at the first key.
static int lru_host_next_key(const MapRec &m, const void *key, void *next_key) {
  std::vector<uint8_t> tab;
  std::vector<uint64_t> stamps;
  if (!next_key) {
    errno = EINVAL;
    return -1;
  }
  if (!lru_download(m, tab, stamps)) return -1;
  uint64_t from = 0;
  if (key) {
    std::vector<uint8_t> slot;
    int64_t fi;
    const int64_t idx = lru_host_probe(m, key, slot, &fi);
    if (idx >= 0) from = (uint64_t)idx + 1;
  }
  for (uint64_t i = from; i < m.d.nbuckets; i++)
    if (tab_state(m, tab, i) == 1) {
      memcpy(next_key, tab.data() + i * m.d.slot_size + m.d.key_off, m.key_size);
      return 0;
    }
  errno = ENOENT;
  return -1;
}

uint64_t Runtime::prepare_lru() {
  std::lock_guard<std::mutex> g(mu);
  if (!lru_maps.empty()) {
    const bool renumber = lru_seq.load() >= kLruSeqLimit;
    const bool check = renumber || ++lru_launches >= 16;
    if (check) {
      lru_launches = 0;
      // no launch may run while tables move
      if (hipDeviceSynchronize() != hipSuccess) return 0;
      for (int fd : lru_maps) {
        const MapRec &m = maps[fd];
        if (renumber || read_word(m, 8) > (m.d.nbuckets - m.max_entries) / 2)
          if (lru_rebuild(m, renumber) < 0) return 0;
      }
      if (renumber) lru_seq = 1;
    }
  }
  return lru_seq.fetch_add(1) + 1;
}

// ---- LPM trie (runtime/src/bpf_map/userspace/lpm_trie_map.cpp) -------------
// The host keeps the authoritative trie (same node structure and update /
// logical-delete rules as the reference); the device holds a read-only
// replica (common.hpp DMap comment) uploaded before the next launch after a
// change.
struct LpmTrie {
  struct Node {
    uint32_t plen = 0;
    bool inter = false;
    int32_t child[2] = {-1, -1};
    std::vector<uint8_t> data, value;
  };
  uint32_t dsz = 0, vsz = 0, max_entries = 0, cap = 0;
  std::vector<Node> nodes;
  int32_t root = -1;
  uint64_t entries = 0;
  // device flat table of a 4-byte-key trie (flat(); DMap.ix), 0 = none
  void *flat_dev = nullptr;
  uint64_t flat_bytes = 0;
  ~LpmTrie() {
    if (flat_dev) (void)hipFree(flat_dev);
  }

  // DIR-24-8 form of a trie with 4-byte keys (IPv4 routing), for device
  // lookups of full-length keys (prefixlen 32): t[a >> 8] for the top 24
  // address bits holds node + 1 of the node lookup() returns for every
  // address of that /24 (0: none), or 0x80000000 | g when the result
  // depends on the low byte, whose 256 results then sit in group g at
  // t[2^24 + 256 g].  Built by partitioning the address space the way the
  // walk does (lpm_trie_map.cpp:192-264, restated in lookup()): the
  // addresses reaching a node form one prefix block; those its prefix does
  // not match keep the result found above it, the matching ones continue to
  // its children, and a matching 32-bit node ends the walk (a deleted, i.e.
  // intermediate, one with no result: the reference's ENOENT, not the
  // covering prefix).  The blocks are disjoint and cover every address, so
  // each table entry is written by exactly one of them.  False when more
  // than max_groups /24s need a group.
  bool flat(std::vector<uint32_t> &t, uint32_t max_groups) const {
    t.assign(1u << 24, 0);
    uint32_t ng = 0;
    bool ok = true;
    auto top = [](uint32_t a, uint32_t len) { return len ? a & (~0u << (32 - len)) : 0u; };
    auto paint = [&](uint32_t a, uint32_t len, uint32_t v) {
      a = top(a, len);
      if (len <= 24) {
        const uint32_t j = a >> 8;
        std::fill(t.begin() + j, t.begin() + j + (1u << (24 - len)), v);
        return;
      }
      const uint32_t j = a >> 8;
      if (!(t[j] & 0x80000000u)) {
        if (ng >= max_groups) {
          ok = false;
          return;
        }
        t.resize(t.size() + 256, 0);
        t[j] = 0x80000000u | ng++;
      }
      const uint64_t g = (1u << 24) + 256ull * (t[j] & 0x7fffffffu) + (a & 0xff);
      std::fill(t.begin() + g, t.begin() + g + (1u << (32 - len)), v);
    };
    // (node, arrival block (a, len), result found above it)
    std::function<void(int32_t, uint32_t, uint32_t, uint32_t)> visit = [&](int32_t ni, uint32_t a, uint32_t len,
                                                                           uint32_t f) {
      if (!ok) return;
      if (ni < 0) {
        paint(a, len, f);
        return;
      }
      const Node &n = nodes[ni];
      const uint32_t np = n.plen;
      const uint32_t nd = top(((uint32_t)n.data[0] << 24) | ((uint32_t)n.data[1] << 16) |
                                  ((uint32_t)n.data[2] << 8) | n.data[3], np);
      const uint32_t c = std::min(len, np);
      if (top(a, c) != top(nd, c)) {  // no address of the block matches the node
        paint(a, len, f);
        return;
      }
      for (uint32_t i = len; i < np; i++)  // first mismatch at bit i
        paint(top(nd, i) | ((~nd) & (0x80000000u >> i)), i + 1, f);
      const uint32_t ml = std::max(len, np);
      const uint32_t m = len > np ? a : (top(a, len) | nd);  // the matching block (m, ml)
      if (np == 32) {
        paint(m, 32, n.inter ? 0 : (uint32_t)ni + 1);
        return;
      }
      const uint32_t f2 = n.inter ? f : (uint32_t)ni + 1;
      for (uint32_t b = 0; b < 2; b++) {
        const uint32_t bitv = b ? (0x80000000u >> np) : 0;
        if (ml > np && (m & (0x80000000u >> np)) != bitv) continue;
        const uint32_t nl = std::max(ml, np + 1);
        visit(n.child[b], top(top(m, np) | bitv | (m & ~top(~0u, np + 1)), nl), nl, f2);
      }
    };
    visit(root, 0, 0, 0);
    return ok;
  }

  int bit(const uint8_t *d, size_t i) const {  // :88-98
    if (i >= (size_t)dsz * 8) return 0;
    return (d[i / 8] >> (7 - (i % 8))) & 1;
  }
  size_t match(const Node &n, const uint8_t *key) const {  // :101-113
    uint32_t kp;
    memcpy(&kp, key, 4);
    const uint32_t lim = std::min(n.plen, kp);
    size_t i = 0;
    while (i < lim && bit(n.data.data(), i) == bit(key + 4, i)) i++;
    return i;
  }
  int32_t make(const uint8_t *key, uint32_t plen, const void *value, bool inter) {
    if (nodes.size() >= cap) return -1;
    Node n;
    n.plen = plen;
    n.inter = inter;
    n.data.assign(key + 4, key + 4 + dsz);
    n.value.assign(vsz, 0);
    if (!inter && value) memcpy(n.value.data(), value, vsz);
    nodes.push_back(std::move(n));
    return (int32_t)nodes.size() - 1;
  }
  const Node *lookup(const uint8_t *key) const {  // :192-264
    uint32_t kp;
    memcpy(&kp, key, 4);
    const uint32_t maxp = dsz * 8;
    if (kp > maxp) {
      errno = EINVAL;
      return nullptr;
    }
    int32_t node = root;
    const Node *found = nullptr;
    while (node >= 0) {
      const Node &n = nodes[node];
      const size_t ml = match(n, key);
      if (ml == maxp) {
        found = &n;
        break;
      }
      if (ml < n.plen) break;
      if (!n.inter) found = &n;
      if (ml < kp)
        node = n.child[bit(key + 4, n.plen)];
      else
        break;
    }
    if (!found || found->inter) {
      errno = ENOENT;
      return nullptr;
    }
    return found;
  }
  long update(const uint8_t *key, const void *value, uint64_t flags) {  // :266-488
    if (flags != 0 && flags != 1 && flags != 2) {
      errno = EINVAL;
      return -1;
    }
    uint32_t kp;
    memcpy(&kp, key, 4);
    const uint32_t maxp = dsz * 8;
    if (kp > maxp) {
      errno = EINVAL;
      return -1;
    }
    auto need_room = [&]() {
      if (flags == 2) {
        errno = ENOENT;
        return false;
      }
      if (entries >= max_entries) {
        errno = ENOSPC;
        return false;
      }
      if (nodes.size() + 2 > cap) {  // node pool of the device replica
        errno = ENOMEM;
        return false;
      }
      return true;
    };
    if (root < 0) {
      if (!need_room()) return -1;
      root = make(key, kp, value, false);
      entries++;
      return 0;
    }
    int32_t parent = -1, pbit = 0, node = -1;
    int32_t cur = root;
    size_t ml = 0;
    while (cur >= 0) {
      node = cur;
      const Node &n = nodes[cur];
      ml = match(n, key);
      if (n.plen != ml || n.plen == kp || n.plen == maxp) break;
      parent = cur;
      pbit = bit(key + 4, n.plen);
      cur = n.child[pbit];
    }
    auto set_slot = [&](int32_t v) {
      if (parent < 0)
        root = v;
      else
        nodes[parent].child[pbit] = v;
    };
    auto split = [&](int32_t at) {  // intermediate node at the split point
      const int32_t nn = make(key, kp, value, false);
      const int32_t im = make(key, (uint32_t)ml, nullptr, true);
      if (bit(key + 4, ml)) {
        nodes[im].child[0] = at;
        nodes[im].child[1] = nn;
      } else {
        nodes[im].child[0] = nn;
        nodes[im].child[1] = at;
      }
      set_slot(im);
      entries++;
      return 0L;
    };
    if (cur >= 0 && nodes[cur].plen == kp) {  // case 1
      if (match(nodes[cur], key) == kp) {
        Node &n = nodes[cur];
        if (flags == 1) {
          errno = EEXIST;
          return -1;
        }
        if (flags == 2 && n.inter) {
          errno = ENOENT;
          return -1;
        }
        if (n.inter) {
          if (entries >= max_entries) {
            errno = ENOSPC;
            return -1;
          }
          n.inter = false;
          entries++;
        }
        memcpy(n.value.data(), value, vsz);
        return 0;
      }
      if (!need_room()) return -1;
      return split(cur);
    }
    if (cur < 0) {  // case 2
      if (!need_room()) return -1;
      set_slot(make(key, kp, value, false));
      entries++;
      return 0;
    }
    (void)node;
    if (ml == kp) {  // case 3: the new prefix becomes cur's parent
      if (!need_room()) return -1;
      const int32_t nn = make(key, kp, value, false);
      nodes[nn].child[bit(nodes[cur].data.data(), ml)] = cur;
      set_slot(nn);
      entries++;
      return 0;
    }
    if (!need_room()) return -1;  // case 4
    return split(cur);
  }
  long remove(const uint8_t *key) {  // :490-541: logical deletion
    uint32_t kp;
    memcpy(&kp, key, 4);
    if (kp > dsz * 8) {
      errno = EINVAL;
      return -1;
    }
    int32_t cur = root, last = -1;
    while (cur >= 0) {
      last = cur;
      const Node &n = nodes[cur];
      const size_t ml = match(n, key);
      if (n.plen != ml || n.plen == kp) break;
      cur = n.child[bit(key + 4, n.plen)];
      last = cur;
    }
    if (last < 0 || nodes[last].plen != kp || match(nodes[last], key) != kp || nodes[last].inter) {
      errno = ENOENT;
      return -1;
    }
    nodes[last].inter = true;
    std::fill(nodes[last].value.begin(), nodes[last].value.end(), 0);
    if (entries) entries--;
    return 0;
  }
  int first_key(uint8_t *next) const {  // :543-590 (only the first key is implemented there)
    int32_t cur = root;
    while (cur >= 0) {
      const Node &n = nodes[cur];
      if (!n.inter) {
        memcpy(next, &n.plen, 4);
        memcpy(next + 4, n.data.data(), dsz);
        return 0;
      }
      cur = n.child[0] >= 0 ? n.child[0] : n.child[1];
    }
    errno = ENOENT;
    return -1;
  }
  // device replica image (common.hpp DMap comment): header {i32 root,
  // u32 nodes, u32 entries, u32 cap}, then the nodes in pool order
  void image(std::vector<uint8_t> &out, uint32_t slot, uint32_t key_off, uint32_t val_off) const {
    out.assign(16 + (size_t)nodes.size() * slot, 0);
    const uint32_t nn = (uint32_t)nodes.size(), ne = (uint32_t)entries;
    memcpy(out.data(), &root, 4);
    memcpy(out.data() + 4, &nn, 4);
    memcpy(out.data() + 8, &ne, 4);
    memcpy(out.data() + 12, &cap, 4);
    for (size_t i = 0; i < nodes.size(); i++) {
      uint8_t *b = out.data() + 16 + i * slot;
      const Node &n = nodes[i];
      const uint32_t inter = n.inter ? 1 : 0;
      memcpy(b, &n.plen, 4);
      memcpy(b + 4, &inter, 4);
      memcpy(b + 8, n.child, 8);
      memcpy(b + key_off, n.data.data(), dsz);
      memcpy(b + val_off, n.value.data(), vsz);
    }
  }
  // the inverse of image(): the trie an ORDERED batch left in the replica
  // (dev_helpers.hpp lpm_update / lpm_remove append nodes in pool order)
  bool from_image(const uint8_t *img, size_t bytes, uint32_t slot, uint32_t key_off, uint32_t val_off) {
    if (bytes < 16) return false;
    int32_t rt_;
    uint32_t nn, ne;
    memcpy(&rt_, img, 4);
    memcpy(&nn, img + 4, 4);
    memcpy(&ne, img + 8, 4);
    if (nn > cap || 16 + (size_t)nn * slot > bytes || rt_ >= (int32_t)nn) return false;
    nodes.assign(nn, Node{});
    for (uint32_t i = 0; i < nn; i++) {
      const uint8_t *b = img + 16 + (size_t)i * slot;
      Node &n = nodes[i];
      uint32_t inter;
      memcpy(&n.plen, b, 4);
      memcpy(&inter, b + 4, 4);
      n.inter = inter != 0;
      memcpy(n.child, b + 8, 8);
      n.data.assign(b + key_off, b + key_off + dsz);
      n.value.assign(b + val_off, b + val_off + vsz);
    }
    root = rt_;
    entries = ne;
    return true;
  }
};

static void lpm_touch(int fd) { rt().lpm_stale.insert(fd); }

// A bigger node pool for the replica: logical deletions never free a node
// (lpm_trie_map.cpp:490-541), so a trie that keeps learning new prefixes
// outgrows any fixed pool; the reference's allocator just grows.  The
// replica moves to a new arena block (values stay inside the arena, which
// the device's access checks and counter tags rely on; the old block is
// not reused) and is uploaded whole before the next launch.
static int lpm_grow(int fd, uint64_t want_nodes) {
  Runtime &r = rt();
  MapRec &m = r.maps[fd];
  if (lpm_pull(fd) < 0) return -1;
  LpmTrie &t = *m.lpm;
  if (want_nodes <= t.cap) return 0;
  uint64_t cap = t.cap ? t.cap : 8;
  while (cap < want_nodes) cap *= 2;
  if (cap > (1ull << 26)) cap = 1ull << 26;
  if (cap <= t.cap) {
    errno = ENOMEM;
    return -1;
  }
  const uint64_t bytes = 16 + cap * m.d.slot_size;
  if (hipDeviceSynchronize() != hipSuccess) return -1;  // no batch still reading the old replica
  const uint64_t base = r.arena_alloc(bytes);
  if (!base) {
    errno = ENOMEM;
    set_error("map arena exhausted growing an LPM trie (BPFTIME_AMD_ARENA_MB)");
    return -1;
  }
  t.cap = (uint32_t)cap;
  m.d.data = base;
  m.bytes = bytes;
  m.d.ix = 0;
  if (r.push_map(fd) < 0) return -1;
  lpm_touch(fd);
  if (t.dsz == 4) r.lpm_flat_pending.insert(fd);
  return 0;
}

static int lpm_pool_out_error(int fd) {
  set_error("LPM_TRIE map fd " + std::to_string(fd) +
            ": an ORDERED batch's program-side update ran out of the device node pool; the trie keeps its state "
            "from before that batch (bpftime_amd_map_ack_error clears this report)");
  errno = ENOMEM;
  return -1;
}

int lpm_pull(int fd) {
  Runtime &r = rt();
  if (r.kind[fd] == HKind::MAP && r.maps[fd].lpm_pool_out) return lpm_pool_out_error(fd);
  if (!r.lpm_dev_dirty.count(fd)) return 0;
  MapRec &m = r.maps[fd];
  r.lpm_dev_dirty.erase(fd);
  if (r.kind[fd] != HKind::MAP || !m.lpm) return 0;
  if (hipDeviceSynchronize() != hipSuccess) return -1;  // the batch that wrote it
  uint32_t hdr[4];
  if (hipMemcpy(hdr, (void *)m.d.data, 16, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  if (hdr[3] & kLpmPoolOut) {
    // a program's update ran out of the replica's node pool (sized before
    // the launch for two nodes per update site and unit, maps.cpp
    // prepare_ix): the reference's trie would have grown, so the batch's
    // results are not the reference's.  The host keeps its trie (the state
    // before that batch) and reports it
    lpm_touch(fd);
    m.lpm_pool_out = true;
    return lpm_pool_out_error(fd);
  }
  const uint64_t bytes = 16 + (uint64_t)std::min(hdr[1], m.lpm->cap) * m.d.slot_size;
  std::vector<uint8_t> img(bytes);
  if (hipMemcpy(img.data(), (void *)m.d.data, bytes, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  if (!m.lpm->from_image(img.data(), bytes, m.d.slot_size, m.d.key_off, m.d.val_off)) {
    set_error("LPM replica is corrupt");
    return -1;
  }
  // the replica is current; the flat table of the old trie is not
  if (m.d.ix) {
    m.d.ix = 0;
    if (r.push_map(fd) < 0) return -1;
  }
  if (m.lpm->dsz == 4) r.lpm_flat_pending.insert(fd);
  return 0;
}

static int lpm_upload(int fd) {
  Runtime &r = rt();
  MapRec &m = r.maps[fd];
  std::vector<uint8_t> img;
  m.lpm->image(img, m.d.slot_size, m.d.key_off, m.d.val_off);
  if (hipDeviceSynchronize() != hipSuccess) return -1;  // no batch still reading the replica
  if (hipMemcpy((void *)m.d.data, img.data(), img.size(), hipMemcpyHostToDevice) != hipSuccess) return -1;
  r.lpm_stale.erase(fd);
  // device lookups walk the replica until a launch large enough builds the
  // flat table (lpm_flat_build)
  m.d.ix = 0;
  if (m.lpm->dsz == 4) r.lpm_flat_pending.insert(fd);
  return r.push_map(fd);
}

// IPv4 tries also get the flat table (LpmTrie::flat) device lookups of
// full-length keys take in one or two loads instead of the trie walk
static int lpm_flat_build(int fd) {
  Runtime &r = rt();
  MapRec &m = r.maps[fd];
  if (lpm_pull(fd) < 0) return -1;
  r.lpm_flat_pending.erase(fd);
  uint64_t flat = 0;
  std::vector<uint32_t> t;
  if (m.lpm->dsz == 4 && !getenv("BPFTIME_AMD_NO_LPM_FLAT") && m.lpm->flat(t, 1u << 16)) {
    LpmTrie &lt = *m.lpm;
    const uint64_t bytes = 4ull * t.size();
    if (lt.flat_bytes < bytes) {
      if (lt.flat_dev) (void)hipFree(lt.flat_dev);
      lt.flat_dev = nullptr;
      lt.flat_bytes = 0;
      if (hipMalloc(&lt.flat_dev, bytes) == hipSuccess) lt.flat_bytes = bytes;
    }
    if (lt.flat_dev && hipMemcpy(lt.flat_dev, t.data(), bytes, hipMemcpyHostToDevice) == hipSuccess)
      flat = (uint64_t)(uintptr_t)lt.flat_dev;
  }
  m.d.ix = flat;
  return r.push_map(fd);
}

void ix_invalidate(int fd) {
  Runtime &r = rt();
  MapRec &m = r.maps[fd];
  if (!m.ix_addr || !m.ix_valid) return;
  m.ix_valid = false;
  m.d.ix = 0;
  r.push_map(fd);
  r.ix_stale.insert(fd);
}

// Rebuild from the table: index exactly the keys the reference probe
// (bpftime_hash_map.hpp:127-151: from hash % nb, linear, stop at an empty
// bucket) reaches, i.e. a filled bucket whose key's home bucket lies in the
// same run of filled buckets at or before it, first occurrence of a key
// only.  One pass over the runs, starting after an empty bucket; a table
// without an empty bucket keeps no index.
static int ix_rebuild(int fd) {
  Runtime &r = rt();
  MapRec &m = r.maps[fd];
  if (hipDeviceSynchronize() != hipSuccess) return -1;  // no batch still writing the table
  const uint64_t nb = m.d.nbuckets, ss = m.d.slot_size;
  std::vector<uint8_t> t(m.bytes);
  if (hipMemcpy(t.data(), (void *)m.d.data, m.bytes, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  auto state = [&](uint64_t i) {
    uint32_t st;
    memcpy(&st, t.data() + i * ss, 4);
    return st;
  };
  uint64_t e0 = nb;
  for (uint64_t i = 0; i < nb; i++)
    if (state(i) != 1) {
      e0 = i;
      break;
    }
  r.ix_stale.erase(fd);
  if (e0 == nb) return 0;  // full table: no index (lookups take the reference probe)
  const uint64_t isz = (uint64_t)m.d.ix_mask + 1, words = ix_bitmap_words(nb);
  const uint32_t ks = ix_key_stride(m.key_size);  // key bytes per position (keyed indexes)
  // the index (entries, keys), then the bucket bitmap (common.hpp ix_bitmap): one upload
  std::vector<uint32_t> ix(isz * (4 + ks) / 4 + 2 * words, 0);
  uint64_t *bits = (uint64_t *)(ix.data() + isz * (4 + ks) / 4);
  for (uint64_t i = 0; i < nb; i++)
    if (state(i) != 0) bits[i >> 6] |= 1ull << (i & 63);
  if (nb % 64) bits[words - 1] |= ~0ull << (nb % 64);
  std::set<std::string> run_keys;
  uint64_t run_start = 1;  // distance from e0 of the current run's first bucket
  for (uint64_t k = 1; k < nb; k++) {
    const uint64_t i = (e0 + k) % nb;
    if (state(i) != 1) {
      run_keys.clear();
      run_start = k + 1;
      continue;
    }
    const uint8_t *key = t.data() + i * ss + m.d.key_off;
    const uint64_t h = hash_bytes(key, m.key_size);
    const uint64_t home = (h % nb + nb - e0) % nb;  // distance from e0
    if (home < run_start || home > k) continue;       // orphaned by a deletion
    if (!run_keys.insert(std::string((const char *)key, m.key_size)).second) continue;  // shadowed
    uint32_t p = ix_pos(h, m.d.ix_mask);
    while (ix[p]) p = (p + 1) & m.d.ix_mask;
    ix[p] = (uint32_t)i + 1;
    if (ks) memcpy((uint8_t *)ix.data() + 4 * isz + (uint64_t)p * ks, key, m.key_size);
  }
  if (hipMemcpy((void *)m.ix_addr, ix.data(), 4 * ix.size(), hipMemcpyHostToDevice) != hipSuccess) return -1;
  m.ix_valid = true;
  m.d.ix = m.ix_addr;
  return r.push_map(fd);
}

int Runtime::prepare_ix(bool may_delete, uint64_t units, const std::vector<int> &lpm_written,
                        uint32_t lpm_update_sites, bool lpm) {
  std::lock_guard<std::mutex> g(mu);
  // a trie whose device update ran out of its pool fails every launch of a
  // program naming a trie until acknowledged
  // (a trie a writer left on the device: its header's pool flag, 16 bytes)
  for (int fd = 0; lpm && fd < (int)kMaxFds; fd++) {
    if (kind[fd] != HKind::MAP || !maps[fd].lpm) continue;
    if (maps[fd].lpm_pool_out) return lpm_pool_out_error(fd);
    if (!lpm_dev_dirty.count(fd)) continue;
    uint32_t hdr[4];
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(hdr, (void *)maps[fd].d.data, 16, hipMemcpyDeviceToHost) != hipSuccess)
      return -1;
    if ((hdr[3] & kLpmPoolOut) && lpm_pull(fd) < 0) return -1;
  }
  // every launch of a program that names a trie reads the current LPM tries
  while (lpm && !lpm_stale.empty()) {
    const int fd = *lpm_stale.begin();
    if (kind[fd] != HKind::MAP || !maps[fd].lpm) {
      lpm_stale.erase(fd);
      continue;
    }
    if (lpm_upload(fd) < 0) return -1;
  }
  // the flat tables only for launches that pay for their build (a host fill
  // of 2^24 entries and a 64-MiB upload after every change of the trie)
  // tries the program may write keep walking the replica: their flat
  // table is dropped and rebuilt once the host has the trie back; their
  // node pool gets room for two new nodes per update call site and unit
  // (an insert makes at most two), up to 2^22 nodes more
  for (const int fd : lpm_written) {
    if (kind[fd] != HKind::MAP || !maps[fd].lpm) continue;
    if (lpm_pull(fd) < 0) return -1;
    const uint64_t room = std::min<uint64_t>(2 * units * std::max<uint32_t>(lpm_update_sites, 1), 1ull << 22);
    if (maps[fd].lpm->nodes.size() + room > maps[fd].lpm->cap &&
        lpm_grow(fd, maps[fd].lpm->nodes.size() + room) < 0)
      return -1;
    if (lpm_stale.count(fd) && lpm_upload(fd) < 0) return -1;
    if (maps[fd].d.ix) {
      maps[fd].d.ix = 0;
      if (push_map(fd) < 0) return -1;
    }
    if (maps[fd].lpm->dsz == 4) lpm_flat_pending.insert(fd);
  }
  if (lpm && units >= kLpmFlatMinUnits) {
    std::vector<int> pending(lpm_flat_pending.begin(), lpm_flat_pending.end());
    for (const int fd : pending) {
      if (kind[fd] != HKind::MAP || !maps[fd].lpm) {
        lpm_flat_pending.erase(fd);
        continue;
      }
      if (std::find(lpm_written.begin(), lpm_written.end(), fd) != lpm_written.end()) continue;
      if (lpm_flat_build(fd) < 0) return -1;
    }
  }
  if (may_delete) {
    for (int fd = 0; fd < (int)kMaxFds; fd++)
      if (kind[fd] == HKind::MAP && maps[fd].ix_valid) ix_invalidate(fd);
    return 0;
  }
  while (!ix_stale.empty()) {
    const int fd = *ix_stale.begin();
    if (kind[fd] != HKind::MAP || !maps[fd].ix_addr) {
      ix_stale.erase(fd);
      continue;
    }
    if (ix_rebuild(fd) < 0) return -1;
  }
  return 0;
}

}  // namespace bpftime_amd

using namespace bpftime_amd;

extern "C" {

const char *bpftime_amd_last_error(void) { return rt().last_error.c_str(); }

void bpftime_amd_set_ncpu(uint32_t ncpu) { rt().ncpu = ncpu ? ncpu : 1; }
uint32_t bpftime_amd_get_ncpu(void) { return rt().ncpu; }

int bpftime_find_minimal_unused_fd(void) {
  std::lock_guard<std::mutex> g(rt().mu);
  return alloc_fd(-1);
}

int bpftime_maps_create(int fd, const char *name, struct bpf_map_attr attr) {
  Runtime &r = rt();
  std::lock_guard<std::mutex> g(r.mu);
  if (r.ensure_device() < 0) return -1;
  fd = alloc_fd(fd);
  if (fd < 0) return -1;
  MapRec m;
  m.name = name ? name : "";
  m.type = (uint32_t)attr.type;
  m.key_size = attr.key_size;
  m.value_size = attr.value_size;
  m.max_entries = attr.max_ents;
  m.flags = attr.flags;
  m.ifindex = attr.ifindex;
  m.btf_vmlinux_value_type_id = attr.btf_vmlinux_value_type_id;
  m.btf_id = attr.btf_id;
  m.btf_key_type_id = attr.btf_key_type_id;
  m.btf_value_type_id = attr.btf_value_type_id;
  m.kernel_bpf_map_id = attr.kernel_bpf_map_id;
  m.map_extra = attr.map_extra;
  DMap &d = m.d;
  d.type = m.type;
  d.key_size = m.key_size;
  d.value_size = m.value_size;
  d.max_entries = m.max_entries;
  d.ncpu = r.ncpu;
  switch (m.type) {
    case MT_ARRAY:
      m.bytes = (uint64_t)m.value_size * m.max_entries;
      break;
    case MT_PERCPU_ARRAY:
      m.bytes = (uint64_t)m.value_size * m.max_entries * d.ncpu;
      break;
    case MT_HASH:
    case MT_PERCPU_HASH:
    case MT_LRU_HASH: {
      if (m.key_size == 0 || m.value_size == 0 || m.max_entries == 0) {
        errno = EINVAL;
        set_error("hash map needs key/value size and max_entries");
        return -1;
      }
      // LRU: room for the tombstones that evictions and deletions leave
      d.nbuckets = next_prime(m.type == MT_LRU_HASH ? 2ull * m.max_entries + 1 : m.max_entries);
      d.key_off = 8;
      d.val_off = 8 + ((m.key_size + 7) & ~7u);
      uint64_t vbytes = (uint64_t)m.value_size * (m.type == MT_PERCPU_HASH ? d.ncpu : 1);
      // Slots never straddle a 128-B cache line: a power of two up to one
      // line, whole lines beyond.  A lane that loads a FILLED state then
      // reads the key from the same line snapshot (dev_helpers.hpp hash_find).
      uint64_t raw = d.val_off + ((vbytes + 7) & ~7ull);
      uint64_t ss = 16;
      if (raw > 128)
        ss = (raw + 127) & ~127ull;
      else
        while (ss < raw) ss <<= 1;
      d.slot_size = (uint32_t)ss;
      m.bytes = d.nbuckets * d.slot_size;
      break;
    }
    case MT_PROG_ARRAY:
      // prog_array.cpp:101-110: key and value are both 4 bytes
      if (m.key_size != 4 || m.value_size != 4) {
        errno = EINVAL;
        set_error("Key size and value size of prog_array must be 4");
        return -1;
      }
      m.bytes = 4ull * m.max_entries;
      break;
    case MT_RINGBUF:
      // ringbuf_map.cpp: positions + 2 x max_entries data bytes; mask =
      // max_entries - 1 needs a power of two
      if (m.max_entries == 0 || (m.max_entries & (m.max_entries - 1))) {
        errno = EINVAL;
        set_error("ring buffer size must be a power of two");
        return -1;
      }
      m.bytes = 256 + 2ull * m.max_entries;
      break;
    case MT_LPM_TRIE: {
      // lpm_trie_map.cpp:43-81: key = u32 prefixlen + 1..256 data bytes
      if (m.key_size < 5 || m.key_size > 260 || m.value_size == 0 || m.max_entries == 0) {
        errno = EINVAL;
        set_error("LPM trie needs key_size 5..260, value_size > 0, max_entries > 0");
        return -1;
      }
      auto t = std::make_shared<LpmTrie>();
      t->dsz = m.key_size - 4;
      t->vsz = m.value_size;
      t->max_entries = m.max_entries;
      t->cap = (uint32_t)std::min<uint64_t>(2ull * m.max_entries + 8, 1u << 26);
      m.lpm = t;
      d.key_off = 16;
      d.val_off = 16 + ((t->dsz + 7) & ~7u);
      d.slot_size = d.val_off + ((m.value_size + 7) & ~7u);
      m.bytes = 16 + (uint64_t)t->cap * d.slot_size;
      break;
    }
    default:
      errno = EINVAL;
      set_error("unsupported map type " + std::to_string(m.type));
      return -1;
  }
  // hash maps: a 128-B counter line; LRU maps: + a u64 stamp per bucket
  uint64_t extra = (m.type == MT_HASH || m.type == MT_PERCPU_HASH) ? 128
                   : m.type == MT_LRU_HASH                          ? 128 + 8ull * d.nbuckets
                                                                    : 0;
  // PROG_ARRAY: a second copy of the slots after them, where device-side
  // map_lookup_elem hands out the looked-up fd (the reference returns a
  // thread-local copy, prog_array.cpp:113-143: a write through the pointer
  // must not change the array)
  const uint64_t shadow = m.type == MT_PROG_ARRAY ? m.bytes : 0;
  uint64_t base = r.arena_alloc(m.bytes + extra + shadow + 8);
  if (!base) {
    errno = ENOMEM;
    set_error("map arena exhausted (BPFTIME_AMD_ARENA_MB)");
    return -1;
  }
  d.data = base;
  d.count_addr = extra ? base + ((m.bytes + 127) & ~127ull) : 0;
  if (hipMemset((void *)base, 0, m.bytes + extra + shadow + 8) != hipSuccess) return -1;
  if (m.type == MT_PROG_ARRAY) {  // every slot INVALID_ENTRY (-1)
    if (hipMemset((void *)base, 0xff, 2 * m.bytes) != hipSuccess) return -1;
    r.prog_gen++;
  }
  if (m.lpm) {  // empty replica: root = -1, no nodes or entries, the pool's capacity
    const uint32_t hdr[4] = {~0u, 0, 0, m.lpm->cap};
    if (hipMemcpy((void *)base, hdr, 16, hipMemcpyHostToDevice) != hipSuccess) return -1;
  }
  if (extra && m.type != MT_LRU_HASH && !getenv("BPFTIME_AMD_NO_HASH_INDEX")) {
    // lookup index (common.hpp ix_pos): a power of two >= 2 x buckets, so
    // it is at most half full; an empty table's index is empty and valid.
    // After it the bucket bitmap (common.hpp ix_bitmap), the bits past the
    // last bucket set
    // (keyed indexes, common.hpp ix_key_stride: the keys beside the
    // entries; config 3's 65,536 flows take 262,144 positions, 5 MiB with
    // their keys, of which a lookup touches one key line as the reference
    // probe touches one bucket line)
    const uint32_t ks = ix_key_stride(m.key_size);
    uint64_t isz = 64;
    while (isz < 2 * (uint64_t)d.nbuckets) isz <<= 1;
    const uint64_t words = ix_bitmap_words(d.nbuckets);
    uint64_t ix = isz <= (1ull << 32) ? r.arena_alloc((4 + ks) * isz + 8 * words) : 0;
    const uint64_t pad = d.nbuckets % 64 ? ~0ull << (d.nbuckets % 64) : 0;
    if (ix && hipMemset((void *)ix, 0, (4 + ks) * isz + 8 * words) == hipSuccess &&
        hipMemcpy((void *)(ix_bitmap(ix, (uint32_t)(isz - 1), m.key_size) + 8 * (words - 1)), &pad, 8,
                  hipMemcpyHostToDevice) == hipSuccess) {
      m.ix_addr = ix;
      m.ix_valid = true;
      d.ix = ix;
      d.ix_mask = (uint32_t)(isz - 1);
    }
  }
  r.maps[fd] = m;
  r.kind[fd] = HKind::MAP;
  if (m.type == MT_LRU_HASH) r.lru_maps.insert(fd);
  if (m.lpm) r.lpm_maps++;
  if (r.push_map(fd) < 0) return -1;
  return fd;
}

int bpftime_is_map_fd(int fd) { return fd >= 0 && fd < (int)kMaxFds && rt().kind[fd] == HKind::MAP; }
int bpftime_is_prog_fd(int fd) { return fd >= 0 && fd < (int)kMaxFds && rt().kind[fd] == HKind::PROG; }
int bpftime_is_array_map(int fd) {
  MapRec *m = map_of(fd);
  return m && m->type == MT_ARRAY;
}

uint32_t bpftime_map_value_size_from_syscall(int fd) {
  MapRec *m = map_of(fd);
  if (!m) return 0;
  if (m->type == MT_PERCPU_ARRAY || m->type == MT_PERCPU_HASH) return m->value_size * m->d.ncpu;
  return m->value_size;  // map_handler.cpp:69-84
}

// ---- PROG_ARRAY (runtime/src/bpf_map/userspace/prog_array.cpp) -------------
// Slots hold bpftime prog fds (the reference encodes them as -fd-2 beside
// kernel prog ids; kernel programs do not exist here).
static thread_local int32_t tl_prog_fd;

static int32_t prog_array_read(const MapRec &m, int32_t k) {
  int32_t v = -1;
  if (hipMemcpy(&v, (const void *)(m.d.data + 4ull * (uint32_t)k), 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return v;
}

// prog_array.cpp:113-143
static const void *prog_array_lookup(const MapRec &m, const void *key) {
  int32_t k;
  memcpy(&k, key, 4);
  if (k < 0 || (uint32_t)k >= m.max_entries) {
    errno = EINVAL;
    return nullptr;
  }
  const int32_t v = prog_array_read(m, k);
  if (v < 0 || !bpftime_is_prog_fd(v)) {
    errno = ENOENT;
    return nullptr;
  }
  tl_prog_fd = v;
  return &tl_prog_fd;
}

// prog_array.cpp:146-176 (flags are not looked at); a value that is not a
// bpftime prog fd would be asked of the kernel, which has no such fd here
static long prog_array_update(MapRec &m, const void *key, const void *value) {
  int32_t k, v;
  memcpy(&k, key, 4);
  if (k < 0 || (uint32_t)k >= m.max_entries) {
    errno = EINVAL;
    return -1;
  }
  memcpy(&v, value, 4);
  if (!bpftime_is_prog_fd(v)) {
    errno = EBADF;
    return -1;
  }
  if (hipMemcpy((void *)(m.d.data + 4ull * (uint32_t)k), &v, 4, hipMemcpyHostToDevice) != hipSuccess) return -1;
  rt().prog_gen++;
  return 0;
}

// prog_array.cpp:180-189
static long prog_array_delete(MapRec &m, const void *key) {
  int32_t k;
  memcpy(&k, key, 4);
  if (k < 0 || (uint32_t)k >= m.max_entries) {
    errno = EINVAL;
    return -1;
  }
  const int32_t none = -1;
  if (hipMemcpy((void *)(m.d.data + 4ull * (uint32_t)k), &none, 4, hipMemcpyHostToDevice) != hipSuccess) return -1;
  rt().prog_gen++;
  return 0;
}

// prog_array.cpp:191-211: the last key is checked before the range
static int prog_array_next_key(const MapRec &m, const void *key, void *next_key) {
  int32_t out = 0;
  if (key) {
    int32_t k;
    memcpy(&k, key, 4);
    if ((size_t)(k + 1) == m.max_entries) {
      errno = ENOENT;
      return -1;
    }
    if (k < 0 || (uint32_t)k >= m.max_entries) {
      errno = EINVAL;
      return -1;
    }
    out = k + 1;
  }
  memcpy(next_key, &out, 4);
  return 0;
}

const void *bpftime_map_lookup_elem(int fd, const void *key) {
  MapRec *m = map_of(fd);
  if (!m) return nullptr;
  if (m->type == MT_RINGBUF) {  // ringbuf_map.cpp: lookup / update / delete / next key unsupported
    errno = ENOTSUP;
    return nullptr;
  }
  if (m->type == MT_PROG_ARRAY) return prog_array_lookup(*m, key);
  if (m->type == MT_LRU_HASH) return lru_host_lookup(*m, key);
  std::vector<uint8_t> &buf = tl_lookup_buf;
  switch (m->type) {
    case MT_ARRAY:
    case MT_PERCPU_ARRAY: {
      uint32_t k;
      memcpy(&k, key, 4);
      if (k >= m->max_entries) {
        errno = ENOENT;
        return nullptr;
      }
      uint64_t vs = m->type == MT_ARRAY ? m->value_size : (uint64_t)m->value_size * m->d.ncpu;
      buf.resize(vs);
      if (hipMemcpy(buf.data(), (void *)(m->d.data + k * vs), vs, hipMemcpyDeviceToHost) != hipSuccess)
        return nullptr;
      return buf.data();
    }
    case MT_HASH:
    case MT_PERCPU_HASH: {
      std::vector<uint8_t> slot;
      int64_t idx = host_hash_find(*m, key, slot, nullptr);
      if (idx < 0) {
        errno = ENOENT;
        return nullptr;
      }
      uint64_t vs = m->type == MT_HASH ? m->value_size : (uint64_t)m->value_size * m->d.ncpu;
      buf.assign(slot.begin() + m->d.val_off, slot.begin() + m->d.val_off + vs);
      return buf.data();
    }
    case MT_LPM_TRIE: {
      if (!key) {
        errno = EINVAL;
        return nullptr;
      }
      // (the runtime lock: a launch on another thread inserts into
      // lpm_dev_dirty and allocates from the arena under it)
      std::lock_guard<std::mutex> g(rt().mu);
      if (lpm_pull(fd) < 0) return nullptr;
      const LpmTrie::Node *n = m->lpm->lookup((const uint8_t *)key);
      if (!n) return nullptr;
      buf = n->value;  // the reference also hands out a copy (lpm_trie_map.cpp:252-263)
      return buf.data();
    }
  }
  return nullptr;
}

long bpftime_map_update_elem(int fd, const void *key, const void *value, uint64_t flags) {
  MapRec *m = map_of(fd);
  if (!m) return -1;
  if (m->type == MT_RINGBUF) {
    errno = ENOTSUP;
    return -1;
  }
  if (m->type == MT_PROG_ARRAY) return prog_array_update(*m, key, value);
  if (m->type == MT_LRU_HASH) return lru_host_update(*m, key, value, flags);
  uint64_t b = flags & 0xffffffffull;
  bool flags_ok = b == 0 || b == 1 || b == 2;  // map_common_def.hpp:83-94
  if (m->type == MT_LPM_TRIE) {
    if (!key || !value) {
      errno = EINVAL;
      return -1;
    }
    std::lock_guard<std::mutex> g(rt().mu);  // (see bpftime_map_lookup_elem)
    if (lpm_pull(fd) < 0) return -1;
    if (m->lpm->nodes.size() + 2 > m->lpm->cap && lpm_grow(fd, m->lpm->nodes.size() + 2) < 0) return -1;
    const long rc = m->lpm->update((const uint8_t *)key, value, flags);
    if (rc == 0) lpm_touch(fd);
    return rc;
  }
  switch (m->type) {
    case MT_ARRAY:
    case MT_PERCPU_ARRAY: {
      if (!flags_ok) {
        errno = EINVAL;
        return -1;
      }
      uint32_t k;
      memcpy(&k, key, 4);
      if (k < m->max_entries && flags == 1) {
        errno = EEXIST;
        return -1;
      }
      if (k >= m->max_entries) {
        errno = E2BIG;
        return -1;
      }
      uint64_t vs = m->type == MT_ARRAY ? m->value_size : (uint64_t)m->value_size * m->d.ncpu;
      return hipMemcpy((void *)(m->d.data + k * vs), value, vs, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
    }
    case MT_HASH: {
      // fix_hash_map.cpp:34-39 -> bpftime_hash_map::elem_update; returns 0
      ix_invalidate(fd);
      std::vector<uint8_t> slot;
      int64_t empty;
      int64_t idx = host_hash_find(*m, key, slot, &empty);
      if (idx >= 0) {
        memcpy(slot.data() + m->d.val_off, value, m->value_size);
        write_slot(*m, (uint64_t)idx, slot);
      } else if (empty >= 0) {
        uint64_t c = read_count(*m);
        if (c < m->max_entries) {
          std::vector<uint8_t> s(m->d.slot_size, 0);
          uint32_t st = 1;
          memcpy(s.data(), &st, 4);
          memcpy(s.data() + m->d.key_off, key, m->key_size);
          memcpy(s.data() + m->d.val_off, value, m->value_size);
          write_slot(*m, (uint64_t)empty, s);
          write_count(*m, c + 1);
        }
      }
      return 0;
    }
    case MT_PERCPU_HASH: {
      // per_cpu_hash_map.cpp:157-183 (userspace view: ncpu * value_size)
      if (!flags_ok) {
        errno = EINVAL;
        return -1;
      }
      ix_invalidate(fd);
      std::vector<uint8_t> slot;
      int64_t empty;
      int64_t idx = host_hash_find(*m, key, slot, &empty);
      if (flags == 1 && idx >= 0) {
        errno = EEXIST;
        return -1;
      }
      if (flags == 2 && idx < 0) {
        errno = ENOENT;
        return -1;
      }
      uint64_t vs = (uint64_t)m->value_size * m->d.ncpu;
      if (idx >= 0) {
        memcpy(slot.data() + m->d.val_off, value, vs);
        write_slot(*m, (uint64_t)idx, slot);
        return 0;
      }
      uint64_t c = read_count(*m);
      if (c >= m->max_entries || empty < 0) {
        errno = E2BIG;
        return -1;
      }
      std::vector<uint8_t> s(m->d.slot_size, 0);
      uint32_t st = 1;
      memcpy(s.data(), &st, 4);
      memcpy(s.data() + m->d.key_off, key, m->key_size);
      memcpy(s.data() + m->d.val_off, value, vs);
      write_slot(*m, (uint64_t)empty, s);
      write_count(*m, c + 1);
      return 0;
    }
  }
  return -1;
}

long bpftime_map_delete_elem(int fd, const void *key) {
  MapRec *m = map_of(fd);
  if (!m) return -1;
  if (m->type == MT_PROG_ARRAY) return prog_array_delete(*m, key);
  if (m->type == MT_LRU_HASH) return lru_host_delete(*m, key);
  if (m->type == MT_RINGBUF) {
    errno = ENOTSUP;
    return -1;
  }
  if (m->type == MT_LPM_TRIE) {
    if (!key) {
      errno = EINVAL;
      return -1;
    }
    std::lock_guard<std::mutex> g(rt().mu);
    if (lpm_pull(fd) < 0) return -1;
    const long rc = m->lpm->remove((const uint8_t *)key);
    if (rc == 0) lpm_touch(fd);
    return rc;
  }
  switch (m->type) {
    case MT_ARRAY:
    case MT_PERCPU_ARRAY:
      errno = EINVAL;  // array_map.cpp:58-64
      return -1;
    case MT_HASH:
    case MT_PERCPU_HASH: {
      // no launch that trusts its lookup cache may still run (runtime.hpp)
      if (rt().lcache_inflight.load()) {
        if (hipDeviceSynchronize() != hipSuccess) return -1;
        rt().lcache_inflight = false;
        rt().deleter_inflight = false;
      }
      std::vector<uint8_t> slot;
      int64_t idx = host_hash_find(*m, key, slot, nullptr);
      if (idx < 0) {
        if (m->type == MT_PERCPU_HASH) {
          errno = ENOENT;
          return -1;
        }
        return 0;  // fix_hash_map.cpp:41-45 returns 0 regardless
      }
      ix_invalidate(fd);
      uint32_t st = 0;
      memcpy(slot.data(), &st, 4);
      write_slot(*m, (uint64_t)idx, slot);
      write_count(*m, read_count(*m) - 1);
      return 0;
    }
  }
  return -1;
}

int bpftime_map_get_next_key(int fd, const void *key, void *next_key) {
  MapRec *m = map_of(fd);
  if (!m) return -1;
  if (m->type == MT_RINGBUF) {
    errno = ENOTSUP;
    return -1;
  }
  if (m->type == MT_LPM_TRIE) {
    if (!next_key || key) {  // lpm_trie_map.cpp:543-590: only the first key
      errno = next_key ? ENOENT : EINVAL;
      return -1;
    }
    std::lock_guard<std::mutex> g(rt().mu);
    if (lpm_pull(fd) < 0) return -1;
    return m->lpm->first_key((uint8_t *)next_key);
  }
  if (m->type == MT_PROG_ARRAY) return prog_array_next_key(*m, key, next_key);
  if (m->type == MT_LRU_HASH) return lru_host_next_key(*m, key, next_key);
  switch (m->type) {
    case MT_ARRAY:
    case MT_PERCPU_ARRAY: {  // array_map.cpp:66-81
      uint32_t k = 0;
      if (key) memcpy(&k, key, 4);
      if (!key || k >= m->max_entries) {
        uint32_t z = 0;
        memcpy(next_key, &z, 4);
        return 0;
      }
      if (k == m->max_entries - 1) {
        errno = ENOENT;
        return -1;
      }
      k++;
      memcpy(next_key, &k, 4);
      return 0;
    }
    case MT_HASH:
    case MT_PERCPU_HASH: {  // fix_hash_map.cpp:47-84: bucket index order
      if (!next_key) {
        errno = EINVAL;
        return -1;
      }
      std::vector<uint8_t> all(m->bytes);
      if (hipMemcpy(all.data(), (void *)m->d.data, m->bytes, hipMemcpyDeviceToHost) != hipSuccess) return -1;
      uint64_t from = 0;
      if (key) {
        std::vector<uint8_t> slot;
        int64_t idx = host_hash_find(*m, key, slot, nullptr);
        if (idx >= 0) from = (uint64_t)idx + 1;
      }
      for (uint64_t i = from; i < m->d.nbuckets; i++) {
        const uint8_t *s = all.data() + i * m->d.slot_size;
        uint32_t st;
        memcpy(&st, s, 4);
        if (st == 1) {
          memcpy(next_key, s + m->d.key_off, m->key_size);
          return 0;
        }
      }
      errno = ENOENT;
      return -1;
    }
  }
  return -1;
}

static void drop_host_view(Runtime &r, int fd) {
  MapRec &m = r.maps[fd];
  if (m.host_view) munmap(m.host_view, m.host_view_bytes);
  m.host_view = nullptr;
  m.host_view_bytes = 0;
  m.host_shadow.clear();
  r.host_views.erase(fd);
}

void bpftime_close(int fd) {
  Runtime &r = rt();
  int detach = 0;
  {
    std::lock_guard<std::mutex> g(r.mu);
    if (fd < 0 || fd >= (int)kMaxFds) return;
    r.prog_gen++;
    if (r.kind[fd] == HKind::MAP) {
      drop_host_view(r, fd);
      r.lru_maps.erase(fd);
      r.lpm_dev_dirty.erase(fd);
      if (r.maps[fd].lpm) r.lpm_maps--;
      r.maps[fd] = MapRec();
      r.push_map(fd);
    } else if (r.kind[fd] == HKind::PROG) {
      r.progs[fd] = ProgRec();
    } else if (r.kind[fd] == HKind::LINK) {
      detach = r.links[fd].attach_id;
      r.links[fd] = LinkRec();
    } else if (r.kind[fd] == HKind::PERF) {
      r.perfs[fd] = PerfRec();
    }
    r.kind[fd] = HKind::NONE;
  }
  if (detach) bpftime_amd_syscall_detach(detach);  // a perf link: its syscall attachment
}

int bpftime_amd_map_ack_error(int fd) {
  Runtime &r = rt();
  std::lock_guard<std::mutex> g(r.mu);
  if (fd < 0 || fd >= (int)kMaxFds || r.kind[fd] != HKind::MAP) return -1;
  const bool had = r.maps[fd].lpm_pool_out;
  r.maps[fd].lpm_pool_out = false;
  return had ? 1 : 0;
}

void bpftime_amd_reset(void) {
  Runtime &r = rt();
  std::lock_guard<std::mutex> g(r.mu);
  std::vector<int> detach;
  for (uint32_t i = 0; i < kMaxFds; i++) {
    if (r.kind[i] == HKind::MAP) drop_host_view(r, (int)i);
    if (r.kind[i] == HKind::LINK && r.links[i].attach_id) detach.push_back(r.links[i].attach_id);
    r.kind[i] = HKind::NONE;
    r.maps[i] = MapRec();
    r.lru_maps.erase((int)i);
    r.lpm_dev_dirty.erase((int)i);
    r.progs[i] = ProgRec();
    r.links[i] = LinkRec();
    r.perfs[i] = PerfRec();
  }
  r.lpm_maps = 0;
  (void)detach;
  syscall_detach_all();  // the link-made attachments and the direct ones
  if (r.d_maptab) hipMemset(r.d_maptab, 0, sizeof(DMap) * kMaxFds);
  r.arena_used = 0;
  r.prog_gen++;  // tail-call images linked before the reset relink
}

// ---- lddw helpers: bpftime_shm.cpp:637-676 --------------------------------
uint64_t bpftime_amd_map_ptr_by_fd(uint32_t fd) {
  if (!map_of((int)fd)) {
    errno = ENOENT;
    return ~0ull;  // INVALID_MAP_PTR
  }
  return fd;
}

uint64_t bpftime_amd_map_val(uint64_t map_ptr) {
  int fd = (int)map_ptr;
  MapRec *m = map_of(fd);
  if (!m) {
    errno = ENOENT;
    return 0;
  }
  switch (m->type) {
    case MT_ARRAY:
      return m->max_entries ? m->d.data : 0;
    case MT_PERCPU_ARRAY:
      return m->max_entries ? m->d.data : 0;  // cpu 0's slot of key 0
    default: {
      uint8_t key[512];
      if (m->key_size > sizeof(key) || bpftime_map_get_next_key(fd, nullptr, key) < 0) {
        errno = ENOENT;
        return 0;
      }
      std::vector<uint8_t> slot;
      int64_t idx = host_hash_find(*m, key, slot, nullptr);
      return idx < 0 ? 0 : m->d.data + (uint64_t)idx * m->d.slot_size + m->d.val_off;
    }
  }
}

uint64_t bpftime_amd_map_device_ptr(int fd, uint64_t *bytes) {
  MapRec *m = map_of(fd);
  if (!m) return 0;
  if (bytes) *bytes = m->bytes;
  return m->d.data;
}

int bpftime_amd_map_snapshot(int fd, void *out, uint64_t bytes) {
  MapRec *m = map_of(fd);
  if (!m || bytes > m->bytes) return -1;
  return hipMemcpy(out, (void *)m->d.data, bytes, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}

int bpftime_amd_map_restore(int fd, const void *in, uint64_t bytes) {
  MapRec *m = map_of(fd);
  if (!m || bytes > m->bytes) return -1;
  ix_invalidate(fd);
  if (hipMemcpy((void *)m->d.data, in, bytes, hipMemcpyHostToDevice) != hipSuccess) return -1;
  if (m->d.count_addr) {
    uint64_t c = 0;
    for (uint64_t i = 0; i < m->d.nbuckets && (i + 1) * m->d.slot_size <= bytes; i++) {
      uint32_t st;
      memcpy(&st, (const uint8_t *)in + i * m->d.slot_size, 4);
      c += st == 1;
    }
    write_count(*m, c);
  }
  return 0;
}

int bpftime_amd_map_geometry(int fd, uint64_t *nbuckets, uint32_t *slot_size, uint32_t *key_off,
                             uint32_t *val_off, uint32_t *ncpu) {
  MapRec *m = map_of(fd);
  if (!m) return -1;
  if (nbuckets) *nbuckets = m->d.nbuckets;
  if (slot_size) *slot_size = m->d.slot_size;
  if (key_off) *key_off = m->d.key_off;
  if (val_off) *val_off = m->d.val_off;
  if (ncpu) *ncpu = m->d.ncpu;
  return 0;
}

// ringbuf::fetch_data (ringbuf_map.cpp): committed records from the consumer
// position on, stopping at a record still being written; discarded records
// are skipped.  Each delivered record is written to out as [u32 len][bytes].
int64_t bpftime_amd_ringbuf_fetch(int fd, void *out, uint64_t cap, uint64_t *used) {
  MapRec *m = map_of(fd);
  if (used) *used = 0;
  if (!m || m->type != MT_RINGBUF) {
    errno = EINVAL;
    return -1;
  }
  if (hipDeviceSynchronize() != hipSuccess) return -1;  // producers of queued batches first
  uint64_t pos[2];
  std::vector<uint8_t> data(2ull * m->max_entries);
  if (hipMemcpy(&pos[0], (void *)m->d.data, 8, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(&pos[1], (void *)(m->d.data + 128), 8, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(data.data(), (void *)(m->d.data + 256), data.size(), hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  const uint64_t mask = m->max_entries - 1;
  uint64_t cons = pos[0], off = 0;
  int64_t cnt = 0;
  while (cons < pos[1]) {
    uint32_t len;
    memcpy(&len, data.data() + (cons & mask), 4);
    if (len & 0x80000000u) break;  // BUSY
    const uint32_t n = len & 0x3fffffffu;
    if (!(len & 0x40000000u)) {     // not DISCARD
      if (off + 4 + n > cap) break;
      memcpy((uint8_t *)out + off, &n, 4);
      memcpy((uint8_t *)out + off + 4, data.data() + (cons & mask) + 8, n);
      off += 4 + n;
      cnt++;
    }
    cons += ((uint64_t)n + 8 + 7) / 8 * 8;
  }
  if (hipMemcpy((void *)m->d.data, &cons, 8, hipMemcpyHostToDevice) != hipSuccess) return -1;
  if (used) *used = off;
  return cnt;
}

uint64_t bpftime_amd_map_count(int fd) {
  MapRec *m = map_of(fd);
  if (m && m->lpm) {
    std::lock_guard<std::mutex> g(rt().mu);
    return lpm_pull(fd) < 0 ? 0 : m->lpm->entries;
  }
  if (!m || !m->d.count_addr) return 0;
  return read_count(*m);
}

// ---- prog / link records ---------------------------------------------------
int bpftime_progs_create(int fd, const void *insns, size_t insn_cnt, const char *prog_name, int prog_type) {
  Runtime &r = rt();
  std::lock_guard<std::mutex> g(r.mu);
  fd = alloc_fd(fd);
  if (fd < 0) return -1;
  ProgRec p;
  p.name = prog_name ? prog_name : "";
  p.insns.assign((const uint8_t *)insns, (const uint8_t *)insns + insn_cnt * 8);
  p.type = prog_type;
  r.progs[fd] = std::move(p);
  r.kind[fd] = HKind::PROG;
  r.prog_gen++;
  return fd;
}

static int link_perf(int fd, int prog_fd, int perf_fd, int bad_errno);

// bpftime_shm_internal.cpp:566-607: only prog_fd is validated; the target of
// an XDP link is an ifindex.
int bpftime_link_create(int fd, struct bpf_link_create_args *args) {
  Runtime &r = rt();
  if (args && args->attach_type == BPFTIME_AMD_BPF_PERF_EVENT) {
    // :578-600: a perf-event link's target must be a perf event (libbpf
    // probes with target_fd -1 and expects EBADF); it attaches like
    // BPF_PROG_ATTACH (both fds checked under the runtime lock, link_perf)
    return link_perf(fd, (int)args->prog_fd, (int)args->target_fd, EBADF);
  }
  std::lock_guard<std::mutex> g(r.mu);
  if (!args) {
    errno = EINVAL;
    return -1;
  }
  if (args->prog_fd >= kMaxFds || r.kind[args->prog_fd] != HKind::PROG) {
    errno = EBADF;
    return -1;
  }
  fd = alloc_fd(fd);
  if (fd < 0) return -1;
  LinkRec l;
  l.prog_fd = args->prog_fd;
  l.target = args->target_fd;
  l.attach_type = args->attach_type;
  l.flags = args->flags;
  r.links[fd] = l;
  r.kind[fd] = HKind::LINK;
  return fd;
}

int bpftime_amd_xdp_links(int *link_fds, int *prog_fds, uint32_t *ifindexes, int max) {
  Runtime &r = rt();
  std::lock_guard<std::mutex> g(r.mu);
  int n = 0;
  for (uint32_t i = 0; i < kMaxFds; i++) {
    if (r.kind[i] != HKind::LINK || r.links[i].attach_type != BPFTIME_AMD_BPF_XDP) continue;
    if (n < max) {
      if (link_fds) link_fds[n] = (int)i;
      if (prog_fds) prog_fds[n] = (int)r.links[i].prog_fd;
      if (ifindexes) ifindexes[n] = r.links[i].target;
    }
    n++;
  }
  return n;
}

// ---- map info (bpftime_shm.cpp:287-306) -------------------------------------
int bpftime_map_get_info(int fd, struct bpf_map_attr *out_attr, const char **out_name, int *type) {
  MapRec *m = map_of(fd);
  if (!m) {
    errno = ENOENT;
    return -1;
  }
  if (out_attr) {
    memset(out_attr, 0, sizeof(*out_attr));
    out_attr->type = (int)m->type;
    out_attr->key_size = m->key_size;
    out_attr->value_size = m->value_size;
    out_attr->max_ents = m->max_entries;
    out_attr->flags = m->flags;
    out_attr->ifindex = m->ifindex;
    out_attr->btf_vmlinux_value_type_id = m->btf_vmlinux_value_type_id;
    out_attr->btf_id = m->btf_id;
    out_attr->btf_key_type_id = m->btf_key_type_id;
    out_attr->btf_value_type_id = m->btf_value_type_id;
    out_attr->map_extra = m->map_extra;
  }
  if (out_name) *out_name = m->name.c_str();
  if (type) *type = (int)m->type;
  return 0;
}

// ---- host views of ARRAY maps (bpftime_shm.cpp:347-353 via the mocked
// mmap64, syscall_context.cpp:915-920) ---------------------------------------
// The reference hands a loader the array's bytes in its shared-memory
// segment.  Here they live in HBM: the view is page-aligned host memory
// holding the same bytes, exchanged with the device at batch boundaries --
// what a host write changed reaches the device before the next launch, what
// a batch changed reaches the view when a synchronous batch returns or on
// bpftime_amd_map_msync.
void *bpftime_get_array_map_raw_data(int fd) {
  Runtime &r = rt();
  std::lock_guard<std::mutex> g(r.mu);
  MapRec *m = map_of(fd);
  if (!m || m->type != MT_ARRAY) {
    errno = EINVAL;
    return nullptr;
  }
  if (m->host_view) return m->host_view;
  const uint64_t pg = 4096, len = std::max<uint64_t>(pg, (m->bytes + pg - 1) / pg * pg);
  void *p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) {
    errno = ENOMEM;
    return nullptr;
  }
  m->host_shadow.resize(m->bytes);
  if (m->bytes && hipMemcpy(m->host_shadow.data(), (void *)m->d.data, m->bytes, hipMemcpyDeviceToHost) != hipSuccess) {
    munmap(p, len);
    errno = EIO;
    return nullptr;
  }
  memcpy(p, m->host_shadow.data(), m->bytes);
  m->host_view = (uint8_t *)p;
  m->host_view_bytes = len;
  r.host_views.insert(fd);
  return p;
}

// host writes -> device: exactly the bytes that differ from the last
// exchange, run by run.  A byte the host did not write is never uploaded,
// so a counter a batch advanced since the last exchange survives a host
// write next to it; batches still running on any stream finish first (they
// may be writing the same map).
static int view_push(MapRec &m) {
  bool synced = false;
  for (uint64_t i = 0; i < m.bytes;) {
    if (m.host_view[i] == m.host_shadow[i]) {
      i++;
      continue;
    }
    uint64_t j = i + 1;
    while (j < m.bytes && m.host_view[j] != m.host_shadow[j]) j++;
    if (!synced) {
      if (hipDeviceSynchronize() != hipSuccess) return -1;
      synced = true;
    }
    if (hipMemcpy((void *)(m.d.data + i), m.host_view + i, j - i, hipMemcpyHostToDevice) != hipSuccess) return -1;
    memcpy(m.host_shadow.data() + i, m.host_view + i, j - i);
    i = j;
  }
  return 0;
}

static int view_pull(MapRec &m) {
  if (hipMemcpy(m.host_shadow.data(), (void *)m.d.data, m.bytes, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  memcpy(m.host_view, m.host_shadow.data(), m.bytes);
  return 0;
}

int Runtime::host_views_push() {
  std::lock_guard<std::mutex> g(mu);
  for (int fd : host_views)
    if (view_push(maps[fd]) < 0) return -1;
  return 0;
}

int Runtime::host_views_pull() {
  std::lock_guard<std::mutex> g(mu);
  for (int fd : host_views)
    if (view_pull(maps[fd]) < 0) return -1;
  return 0;
}

int bpftime_amd_map_msync(int fd) {
  Runtime &r = rt();
  std::lock_guard<std::mutex> g(r.mu);
  MapRec *m = map_of(fd);
  if (!m || !m->host_view) {
    errno = EINVAL;
    return -1;
  }
  if (hipDeviceSynchronize() != hipSuccess) return -1;  // batches still running first
  return view_push(*m) < 0 || view_pull(*m) < 0 ? -1 : 0;
}

// ---- perf events + BPF_PROG_ATTACH (bpftime_shm.cpp:227-253,
// bpftime_shm_internal.cpp:212-315) ------------------------------------------
static int perf_create(int fd, const PerfRec &p) {
  Runtime &r = rt();
  std::lock_guard<std::mutex> g(r.mu);
  fd = alloc_fd(fd);
  if (fd < 0) return -1;
  r.perfs[fd] = p;
  r.kind[fd] = HKind::PERF;
  return fd;
}

int bpftime_amd_perf_event_syscall(int fd, int64_t sys_nr) {
  if (sys_nr < -1) {
    errno = EINVAL;
    return -1;
  }
  PerfRec p;
  p.sys_nr = sys_nr;
  return perf_create(fd, p);
}

// add_tracepoint (:254-264): the id is resolved when a program attaches
int bpftime_tracepoint_create(int fd, int pid, int32_t tp_id) {
  PerfRec p;
  p.pid = pid;
  p.tracepoint_id = tp_id;
  return perf_create(fd, p);
}

// add_uprobe / add_uprobe_override (:212-252): records only, nothing on this
// path probes a process
int bpftime_uprobe_create(int fd, int pid, const char *name, uint64_t offset, bool retprobe, size_t ref_ctr_off) {
  PerfRec p;
  p.type = retprobe ? 7 : 6;
  p.pid = pid;
  p.module = name ? name : "";
  p.offset = offset;
  p.ref_ctr_off = ref_ctr_off;
  return perf_create(fd, p);
}

int bpftime_amd_perf_event_record(int fd, const struct bpftime_amd_perf_event *e) {
  if (!e) {
    errno = EINVAL;
    return -1;
  }
  PerfRec p;
  p.type = e->type;
  p.pid = e->pid;
  p.enabled = e->enabled != 0;
  p.tracepoint_id = e->tracepoint_id;
  p.sys_nr = e->sys_nr;
  p.offset = e->offset;
  p.ref_ctr_off = e->ref_ctr_off;
  p.module = e->module_name ? e->module_name : "";
  p.cpu = e->cpu;
  p.sample_type = e->sample_type;
  p.config = e->config;
  return perf_create(fd, p);
}

int bpftime_amd_perf_event_get(int fd, struct bpftime_amd_perf_event *e) {
  Runtime &r = rt();
  std::lock_guard<std::mutex> g(r.mu);
  if (fd < 0 || fd >= (int)kMaxFds || r.kind[fd] != HKind::PERF || !e) {
    errno = ENOENT;
    return -1;
  }
  const PerfRec &p = r.perfs[fd];
  e->type = p.type;
  e->pid = p.pid;
  e->enabled = p.enabled;
  e->tracepoint_id = p.tracepoint_id;
  e->sys_nr = p.sys_nr;
  e->offset = p.offset;
  e->ref_ctr_off = p.ref_ctr_off;
  e->module_name = p.module.c_str();  // valid until the record changes
  e->cpu = p.cpu;
  e->sample_type = p.sample_type;
  e->config = p.config;
  return 0;
}

static int perf_enable(int fd, bool on) {  // :317-337
  Runtime &r = rt();
  std::lock_guard<std::mutex> g(r.mu);
  if (fd < 0 || fd >= (int)kMaxFds || r.kind[fd] != HKind::PERF) {
    errno = ENOENT;
    return -1;
  }
  r.perfs[fd].enabled = on;
  return 0;
}
int bpftime_perf_event_enable(int fd) { return perf_enable(fd, true); }
int bpftime_perf_event_disable(int fd) { return perf_enable(fd, false); }

int bpftime_is_perf_event_fd(int fd) { return fd >= 0 && fd < (int)kMaxFds && rt().kind[fd] == HKind::PERF; }

// What a link to perf event p drives: 1 + the sys_enter dispatch slot for a
// syscall enter tracepoint (the global one: sys_nr -1), 0 for a record that
// runs nothing on this path (sys_exit tracepoints: the replay holds enter
// records only; uprobes, software events), -1 for a tracepoint id that does
// not resolve (the reference's attach fails there too,
// syscall_trace_attach_private_data.cpp:51-62); *enter: the sys_enter (1) or
// sys_exit (0) tracepoint
static int perf_drives(const PerfRec &p, int64_t *nr, int *enter) {
  if (p.type != 2) return 0;
  *enter = 1;
  *nr = p.sys_nr;
  if (p.tracepoint_id >= 0 && bpftime_amd_tracepoint_resolve(p.tracepoint_id, nr, enter) < 0) return -1;
  return 1;
}

// A link from prog_fd to perf_fd at `fd` (-1: a fresh one).  A link to a
// sys_enter or sys_exit tracepoint attaches the program to the syscall
// dispatch (it is instantiated: a program the device cannot load fails the
// link); any other perf target, and a tracepoint id that does not resolve
// here, gives a link record that runs nothing: the reference's
// add_bpf_link / add_bpf_prog_attach_target (bpftime_shm_internal.cpp:293-315,
// :566-607) check only the handler kinds and resolve the id when its agent
// attaches.  bad_errno: what a non-perf perf_fd or non-program prog_fd sets
// (ENOENT for BPF_PROG_ATTACH, EBADF for BPF_LINK_CREATE).
static int link_perf(int fd, int prog_fd, int perf_fd, int bad_errno) {
  Runtime &r = rt();
  int64_t nr = -1;
  int drives, enter = 1;
  {
    std::lock_guard<std::mutex> g(r.mu);
    if (perf_fd < 0 || perf_fd >= (int)kMaxFds || r.kind[perf_fd] != HKind::PERF) {  // "Fd is not a perf fd"
      errno = bad_errno;
      return -1;
    }
    if (prog_fd < 0 || prog_fd >= (int)kMaxFds || r.kind[prog_fd] != HKind::PROG) {
      errno = bad_errno;
      return -1;
    }
    if (fd >= 0 && (fd >= (int)kMaxFds || r.kind[fd] != HKind::NONE)) {
      errno = EBADF;
      return -1;
    }
    drives = perf_drives(r.perfs[perf_fd], &nr, &enter);
  }
  int id = 0;
  if (drives > 0) {
    id = bpftime_amd_syscall_attach_ex(prog_fd, nr, enter);  // instantiates the program (outside the lock)
    if (id < 0) return -1;
  }
  std::lock_guard<std::mutex> g(r.mu);
  fd = alloc_fd(fd);
  if (fd < 0) {
    if (id) bpftime_amd_syscall_detach(id);
    return -1;
  }
  LinkRec l;
  l.prog_fd = (uint32_t)prog_fd;
  l.target = (uint32_t)perf_fd;
  l.attach_type = BPFTIME_AMD_BPF_PERF_EVENT;
  l.perf = true;
  l.attach_id = id;
  r.links[fd] = l;
  r.kind[fd] = HKind::LINK;
  return fd;
}

int bpftime_attach_perf_to_bpf(int perf_fd, int bpf_fd) { return link_perf(-1, bpf_fd, perf_fd, ENOENT); }

int bpftime_amd_link_perf(int fd, int prog_fd, int perf_fd) { return link_perf(fd, prog_fd, perf_fd, ENOENT); }

int bpftime_amd_link_attached(int fd) {
  Runtime &r = rt();
  std::lock_guard<std::mutex> g(r.mu);
  if (fd < 0 || fd >= (int)kMaxFds || r.kind[fd] != HKind::LINK) return -1;
  return r.links[fd].attach_id ? 1 : 0;
}

// ---- host merge ------------------------------------------------------------
// final = init + sum(shard - init), counter by counter at the map's counter
// width (a u32 counter's combined delta wraps at 2^32 instead of carrying
// into its neighbour)
#define MERGE_DELTA(T)                                                     \
  do {                                                                     \
    T *a = (T *)acc;                                                       \
    const T *i0 = (const T *)init, *s = (const T *)shard;                  \
    for (uint64_t k = 0; k < bytes / sizeof(T); k++) a[k] = (T)(a[k] + (T)(s[k] - i0[k])); \
  } while (0)

int bpftime_amd_merge_delta(void *acc, const void *init, const void *shard, uint64_t bytes, uint32_t width) {
  if (!acc || !init || !shard || !width || bytes % width) return -1;
  switch (width) {
    case 1: MERGE_DELTA(uint8_t); return 0;
    case 2: MERGE_DELTA(uint16_t); return 0;
    case 4: MERGE_DELTA(uint32_t); return 0;
    case 8: MERGE_DELTA(uint64_t); return 0;
  }
  return -1;
}
#undef MERGE_DELTA

int bpftime_amd_merge_delta_u64(void *acc, const void *init, const void *shard, uint64_t bytes) {
  return bpftime_amd_merge_delta(acc, init, shard, bytes, 8);
}

}  // extern "C"

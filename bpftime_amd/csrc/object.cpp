// bpftime_amd: eBPF ELF object loader.
//
// The reference opens objects with libbpf (runtime/object/bpf_object.cpp:
// 149-173, bpf_object__open) and, on its LD_PRELOAD path, lets libbpf's
// bpf_object__load create the maps and relocate the programs before the
// BPF_MAP_CREATE / BPF_PROG_LOAD records reach its syscall server
// (runtime/syscall-server/syscall_context.cpp:429-668).  libbpf is absent
// here, so this file does that work itself for the subset an XDP / tracing
// object built by clang + libbpf headers uses:
//
//   * ELF64 little-endian EM_BPF objects: program sections (SHF_EXECINSTR,
//     one program per global function symbol; .text holds subprograms);
//   * maps: BTF-defined (`SEC(".maps")`, __uint / __type members decoded
//     from .BTF) and legacy `SEC("maps")` struct bpf_map_def records;
//   * global data: .bss / .data* / .rodata* become one-element ARRAY maps
//     (libbpf's internal maps), initialised from the section bytes;
//   * relocations (.rel<sec>, R_BPF_64_64 on lddw): a map symbol gives
//     BPF_PSEUDO_MAP_FD (src 1, imm = fd), a data symbol gives
//     BPF_PSEUDO_MAP_VALUE (src 2, imm = fd, next imm = addend + symbol
//     offset), exactly the instruction form libbpf hands to BPF_PROG_LOAD;
//   * CO-RE field relocations (.BTF.ext core_relo: field byte offset / size
//     / existence, type existence / size), resolved by member name against
//     a target BTF (libbpf's btf_custom_path; e.g. the reference's
//     example/xdp-counter/base.btf, where xdp_md has u64 data / data_end as
//     in runtime/extension/userspace_xdp.h:6-17), including the load-size
//     change libbpf makes when the target field is wider.  Without a target
//     BTF the built-in one describes xdp_md as the runtime lays it out.
//
// BPF-to-BPF calls are rejected: the reference VM patches every call as a
// helper call (vm/compat/ubpf-vm/compat_ubpf.cpp:75-95), so they cannot run
// there either.  Host-only code: no device work until bpftime_object_load.
#include <ctype.h>
#include <elf.h>
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <string>
#include <vector>

#include "../../include/bpftime_amd.h"

#ifndef EM_BPF
#define EM_BPF 247
#endif

namespace {

// ---------------------------------------------------------------- BTF ----
enum : uint32_t {
  K_INT = 1, K_PTR, K_ARRAY, K_STRUCT, K_UNION, K_ENUM, K_FWD, K_TYPEDEF, K_VOLATILE, K_CONST,
  K_RESTRICT, K_FUNC, K_FUNC_PROTO, K_VAR, K_DATASEC, K_FLOAT, K_DECL_TAG, K_TYPE_TAG, K_ENUM64
};

struct BMember {
  std::string name;
  uint32_t type = 0;
  uint32_t bit_off = 0;
  uint32_t bit_size = 0;  // bitfield (kind_flag), 0 otherwise
};

struct BType {
  uint32_t kind = 0;
  std::string name;
  uint32_t size = 0;  // INT / STRUCT / UNION / ENUM / DATASEC / FLOAT
  uint32_t type = 0;  // PTR / TYPEDEF / modifiers / VAR / FUNC; ARRAY element
  uint32_t nelems = 0;
  uint32_t enc = 0;   // INT encoding word (bit 24: signed)
  std::vector<BMember> members;                          // STRUCT / UNION
  std::vector<std::pair<uint32_t, uint32_t>> secinfo;    // DATASEC: (var type, offset)
};

struct Btf {
  std::vector<BType> t;  // t[0] = void

  bool parse(const uint8_t *p, size_t n, std::string &err) {
    t.assign(1, BType());
    if (n < 24) return (err = "BTF too short", false);
    uint16_t magic;
    uint32_t hdr_len, type_off, type_len, str_off, str_len;
    memcpy(&magic, p, 2);
    memcpy(&hdr_len, p + 4, 4);
    memcpy(&type_off, p + 8, 4);
    memcpy(&type_len, p + 12, 4);
    memcpy(&str_off, p + 16, 4);
    memcpy(&str_len, p + 20, 4);
    if (magic != 0xeb9f) return (err = "bad BTF magic", false);
    if ((uint64_t)hdr_len + type_off + type_len > n || (uint64_t)hdr_len + str_off + str_len > n)
      return (err = "BTF sections out of range", false);
    const uint8_t *ty = p + hdr_len + type_off, *st = p + hdr_len + str_off;
    auto str = [&](uint32_t o) -> std::string {
      if (o >= str_len) return "";
      return std::string((const char *)st + o, strnlen((const char *)st + o, str_len - o));
    };
    size_t off = 0;
    auto u32 = [&](size_t at) {
      uint32_t v;
      memcpy(&v, ty + at, 4);
      return v;
    };
    while (off + 12 <= type_len) {
      BType b;
      const uint32_t name_off = u32(off), info = u32(off + 4), su = u32(off + 8);
      off += 12;
      b.kind = (info >> 24) & 0x1f;
      const uint32_t vlen = info & 0xffff;
      const bool kflag = (info >> 31) & 1;
      b.name = str(name_off);
      b.size = su;
      b.type = su;
      size_t extra = 0;
      switch (b.kind) {
        case K_INT:
          if (off + 4 > type_len) return (err = "truncated BTF int", false);
          b.enc = u32(off);
          extra = 4;
          break;
        case K_ARRAY:
          if (off + 12 > type_len) return (err = "truncated BTF array", false);
          b.type = u32(off);
          b.nelems = u32(off + 8);
          extra = 12;
          break;
        case K_STRUCT:
        case K_UNION:
          if (off + 12ull * vlen > type_len) return (err = "truncated BTF struct", false);
          for (uint32_t i = 0; i < vlen; i++) {
            BMember m;
            m.name = str(u32(off + 12 * i));
            m.type = u32(off + 12 * i + 4);
            const uint32_t o = u32(off + 12 * i + 8);
            m.bit_off = kflag ? (o & 0xffffff) : o;
            m.bit_size = kflag ? (o >> 24) : 0;
            b.members.push_back(m);
          }
          extra = 12ull * vlen;
          break;
        case K_ENUM: extra = 8ull * vlen; break;
        case K_FUNC_PROTO: extra = 8ull * vlen; break;
        case K_VAR: extra = 4; break;
        case K_DATASEC:
          if (off + 12ull * vlen > type_len) return (err = "truncated BTF datasec", false);
          for (uint32_t i = 0; i < vlen; i++) b.secinfo.emplace_back(u32(off + 12 * i), u32(off + 12 * i + 4));
          extra = 12ull * vlen;
          break;
        case K_DECL_TAG: extra = 4; break;
        case K_ENUM64: extra = 12ull * vlen; break;
        case K_PTR: case K_FWD: case K_TYPEDEF: case K_VOLATILE: case K_CONST: case K_RESTRICT:
        case K_FUNC: case K_FLOAT: case K_TYPE_TAG:
          break;
        default:
          return (err = "unknown BTF kind " + std::to_string(b.kind), false);
      }
      off += extra;
      t.push_back(std::move(b));
    }
    return true;
  }

  const BType *at(uint32_t id) const { return id < t.size() ? &t[id] : nullptr; }
  // strip typedefs and qualifiers
  uint32_t skip(uint32_t id) const {
    for (int guard = 0; guard < 64; guard++) {
      const BType *b = at(id);
      if (!b) return 0;
      if (b->kind == K_TYPEDEF || b->kind == K_VOLATILE || b->kind == K_CONST || b->kind == K_RESTRICT ||
          b->kind == K_TYPE_TAG)
        id = b->type;
      else
        return id;
    }
    return 0;
  }
  uint64_t size_of(uint32_t id) const {
    id = skip(id);
    const BType *b = at(id);
    if (!b) return 0;
    switch (b->kind) {
      case K_INT: case K_STRUCT: case K_UNION: case K_ENUM: case K_ENUM64: case K_DATASEC: case K_FLOAT:
        return b->size;
      case K_PTR: return 8;
      case K_ARRAY: return (uint64_t)b->nelems * size_of(b->type);
      default: return 0;
    }
  }
  std::vector<uint32_t> find(const std::string &name, uint32_t kind) const {
    std::vector<uint32_t> r;
    for (uint32_t i = 1; i < t.size(); i++)
      if (t[i].kind == kind && t[i].name == name) r.push_back(i);
    return r;
  }
};

// The runtime's own context types as BTF (used as the CO-RE target when no
// target BTF is given): xdp_md as runtime/extension/userspace_xdp.h:6-17 and
// example/xdp-counter/base.btf lay it out.
static void builtin_target(Btf &b) {
  b.t.assign(1, BType());
  auto add = [&](BType x) {
    b.t.push_back(std::move(x));
    return (uint32_t)(b.t.size() - 1);
  };
  BType u32t; u32t.kind = K_INT; u32t.name = "unsigned int"; u32t.size = 4;
  BType u64t; u64t.kind = K_INT; u64t.name = "long long unsigned int"; u64t.size = 8;
  const uint32_t i32 = add(u32t), i64 = add(u64t);
  BType x; x.kind = K_STRUCT; x.name = "xdp_md"; x.size = 48;
  const char *names[] = {"data", "data_end", "data_meta", "ingress_ifindex", "rx_queue_index",
                         "egress_ifindex", "buffer_start", "buffer_end"};
  const uint32_t types[] = {i64, i64, i32, i32, i32, i32, i64, i64};
  const uint32_t offs[] = {0, 8, 16, 20, 24, 28, 32, 40};
  for (int i = 0; i < 8; i++) {
    BMember m;
    m.name = names[i];
    m.type = types[i];
    m.bit_off = offs[i] * 8;
    x.members.push_back(m);
  }
  add(x);
}

// CO-RE access resolution: the access string "a:b:c" on type `root`;
// returns byte offset, byte size of the final field, and its type.
struct Access {
  bool ok = false;
  int64_t off = 0;
  uint64_t size = 0;
  uint32_t type = 0;
  bool bitfield = false;
  std::vector<std::string> names;  // member names along the path ("" for array steps)
};

static Access walk_local(const Btf &b, uint32_t root, const std::vector<int64_t> &spec) {
  Access a;
  if (spec.empty()) return a;
  uint32_t cur = b.skip(root);
  a.off = spec[0] * (int64_t)b.size_of(cur);
  for (size_t i = 1; i < spec.size(); i++) {
    const BType *t = b.at(cur);
    if (!t) return a;
    if (t->kind == K_STRUCT || t->kind == K_UNION) {
      if (spec[i] < 0 || (size_t)spec[i] >= t->members.size()) return a;
      const BMember &m = t->members[spec[i]];
      if (m.bit_size || m.bit_off % 8) a.bitfield = true;
      a.off += m.bit_off / 8;
      a.names.push_back(m.name);
      cur = b.skip(m.type);
    } else if (t->kind == K_ARRAY) {
      a.off += spec[i] * (int64_t)b.size_of(t->type);
      a.names.push_back("");
      cur = b.skip(t->type);
    } else {
      return a;
    }
  }
  a.ok = true;
  a.type = cur;
  a.size = b.size_of(cur);
  return a;
}

// the same path in a target type, members matched by name
static Access walk_target(const Btf &b, uint32_t root, const std::vector<int64_t> &spec,
                          const std::vector<std::string> &names) {
  Access a;
  uint32_t cur = b.skip(root);
  a.off = spec[0] * (int64_t)b.size_of(cur);
  for (size_t i = 1; i < spec.size(); i++) {
    const BType *t = b.at(cur);
    if (!t) return a;
    const std::string &want = names[i - 1];
    if ((t->kind == K_STRUCT || t->kind == K_UNION) && !want.empty()) {
      const BMember *hit = nullptr;
      for (const BMember &m : t->members)
        if (m.name == want) hit = &m;
      if (!hit) return a;
      if (hit->bit_size || hit->bit_off % 8) a.bitfield = true;
      a.off += hit->bit_off / 8;
      cur = b.skip(hit->type);
    } else if (t->kind == K_ARRAY && want.empty()) {
      if (spec[i] >= (int64_t)t->nelems && t->nelems) return a;
      a.off += spec[i] * (int64_t)b.size_of(t->type);
      cur = b.skip(t->type);
    } else {
      return a;
    }
  }
  a.ok = true;
  a.type = cur;
  a.size = b.size_of(cur);
  return a;
}

static std::string essential_name(const std::string &n) {
  const size_t p = n.find("___");
  return p == std::string::npos ? n : n.substr(0, p);
}

// ---------------------------------------------------------------- ELF ----
struct Section {
  std::string name;
  Elf64_Shdr h{};
  const uint8_t *data = nullptr;
};

struct MapDef {
  std::string name;
  bpf_map_attr attr{};
  int sec = -1;             // ELF section the map lives in
  uint64_t sec_off = 0;     // offset of its symbol (BTF / legacy maps)
  std::vector<uint8_t> init;  // initial value of key 0 (data sections)
  bool internal = false;    // .bss / .data / .rodata
};

struct Reloc {
  size_t insn;       // index inside the program
  int map = -1;      // map index
  int src = 0;       // BPF_PSEUDO_MAP_FD (1) or BPF_PSEUDO_MAP_VALUE (2)
  int64_t addend = 0;
};

struct Prog {
  std::string name, secname;
  int type = 0;
  std::vector<uint8_t> insns;  // CO-RE relocated, lddw imms still map indices
  std::vector<Reloc> relocs;
  int fd = -1;
};

constexpr uint8_t LDDW = 0x18, CALL = 0x85;

static int prog_type_of(const std::string &sec) {
  // libbpf section_defs (the common ones): BPF_PROG_TYPE_* from linux/bpf.h
  struct P { const char *pfx; int type; };
  static const P tab[] = {
      {"xdp", 6},        {"tracepoint/", 5}, {"tp/", 5},        {"raw_tracepoint/", 17}, {"raw_tp/", 17},
      {"kprobe/", 2},    {"kretprobe/", 2},  {"uprobe", 2},     {"uretprobe", 2},        {"socket", 1},
      {"tc", 3},         {"classifier", 3},  {"perf_event", 7}, {"fentry/", 26},         {"fexit/", 26},
  };
  for (const P &p : tab)
    if (sec.compare(0, strlen(p.pfx), p.pfx) == 0) return p.type;
  return 0;
}

}  // namespace

struct bpftime_object {
  std::string name;
  std::vector<uint8_t> buf;
  std::vector<Section> secs;
  std::vector<Elf64_Sym> syms;
  std::vector<std::string> sym_names;
  Btf btf, target;
  bool has_btf = false, has_target = false;
  std::vector<MapDef> maps;
  std::vector<Prog> progs;
  std::vector<int> map_fds;
  std::string license, error;
  bool loaded = false;

  int fail(const std::string &e) {
    error = e;
    errno = EINVAL;
    return -1;
  }

  int sec_by_name(const std::string &n) const {
    for (size_t i = 0; i < secs.size(); i++)
      if (secs[i].name == n) return (int)i;
    return -1;
  }

  int parse() {
    const uint8_t *p = buf.data();
    const size_t n = buf.size();
    if (n < sizeof(Elf64_Ehdr) || memcmp(p, ELFMAG, SELFMAG) != 0) return fail("not an ELF file");
    Elf64_Ehdr eh;
    memcpy(&eh, p, sizeof eh);
    if (eh.e_ident[EI_CLASS] != ELFCLASS64 || eh.e_ident[EI_DATA] != ELFDATA2LSB)
      return fail("not a little-endian ELF64 object");
    if (eh.e_machine != EM_BPF) return fail("not a BPF object (e_machine " + std::to_string(eh.e_machine) + ")");
    if (eh.e_shentsize != sizeof(Elf64_Shdr) || eh.e_shoff + (uint64_t)eh.e_shnum * sizeof(Elf64_Shdr) > n)
      return fail("bad section header table");
    secs.resize(eh.e_shnum);
    for (size_t i = 0; i < eh.e_shnum; i++) {
      memcpy(&secs[i].h, p + eh.e_shoff + i * sizeof(Elf64_Shdr), sizeof(Elf64_Shdr));
      const Elf64_Shdr &h = secs[i].h;
      if (h.sh_type != SHT_NOBITS && h.sh_type != SHT_NULL) {
        if (h.sh_offset + h.sh_size > n) return fail("section " + std::to_string(i) + " out of range");
        secs[i].data = p + h.sh_offset;
      }
    }
    if (eh.e_shstrndx >= secs.size()) return fail("bad shstrndx");
    const Section &shs = secs[eh.e_shstrndx];
    for (Section &s : secs) {
      if (s.h.sh_name < shs.h.sh_size)
        s.name = std::string((const char *)shs.data + s.h.sh_name,
                             strnlen((const char *)shs.data + s.h.sh_name, shs.h.sh_size - s.h.sh_name));
    }
    // symbols
    for (const Section &s : secs) {
      if (s.h.sh_type != SHT_SYMTAB) continue;
      const size_t cnt = s.h.sh_size / sizeof(Elf64_Sym);
      if (s.h.sh_link >= secs.size()) return fail("bad symtab link");
      const Section &strs = secs[s.h.sh_link];
      for (size_t i = 0; i < cnt; i++) {
        Elf64_Sym sym;
        memcpy(&sym, s.data + i * sizeof(Elf64_Sym), sizeof sym);
        syms.push_back(sym);
        sym_names.push_back(sym.st_name < strs.h.sh_size
                                ? std::string((const char *)strs.data + sym.st_name,
                                              strnlen((const char *)strs.data + sym.st_name,
                                                      strs.h.sh_size - sym.st_name))
                                : "");
      }
      break;
    }
    if (syms.empty()) return fail("object has no symbol table");
    const int bi = sec_by_name(".BTF");
    if (bi >= 0) {
      if (!btf.parse(secs[bi].data, secs[bi].h.sh_size, error)) return fail(".BTF: " + error);
      has_btf = true;
    }
    const int li = sec_by_name("license");
    if (li >= 0 && secs[li].data)
      license.assign((const char *)secs[li].data, strnlen((const char *)secs[li].data, secs[li].h.sh_size));
    if (collect_maps() < 0 || collect_progs() < 0) return -1;
    return 0;
  }

  // ---- maps ----
  int collect_maps() {
    const int mi = sec_by_name(".maps");
    if (mi >= 0) {
      if (!has_btf) return fail(".maps section without .BTF");
      const BType *ds = nullptr;
      for (const BType &t : btf.t)
        if (t.kind == K_DATASEC && t.name == ".maps") ds = &t;
      if (!ds) return fail("no .maps DATASEC in BTF");
      for (auto &vi : ds->secinfo) {
        const BType *var = btf.at(vi.first);
        if (!var || var->kind != K_VAR) return fail("bad .maps variable");
        MapDef m;
        m.name = var->name;
        m.sec = mi;
        m.sec_off = vi.second;
        for (size_t s = 0; s < syms.size(); s++)  // symbol offset (libbpf fixes DATASEC offsets the same way)
          if (sym_names[s] == m.name && syms[s].st_shndx == (unsigned)mi) m.sec_off = syms[s].st_value;
        const BType *def = btf.at(btf.skip(var->type));
        if (!def || def->kind != K_STRUCT) return fail("map " + m.name + ": definition is not a struct");
        for (const BMember &mem : def->members) {
          const BType *ptr = btf.at(btf.skip(mem.type));
          if (!ptr || ptr->kind != K_PTR) return fail("map " + m.name + ": member " + mem.name + " is not __uint/__type");
          const uint32_t pointee = btf.skip(ptr->type);
          const BType *arr = btf.at(pointee);
          auto uint_val = [&](uint32_t &dst) -> bool {
            if (!arr || arr->kind != K_ARRAY) return false;
            dst = arr->nelems;
            return true;
          };
          bool ok = true;
          if (mem.name == "type") {
            uint32_t v = 0;
            ok = uint_val(v);
            m.attr.type = (int)v;
          } else if (mem.name == "max_entries") {
            ok = uint_val(m.attr.max_ents);
          } else if (mem.name == "map_flags") {
            uint32_t v = 0;
            ok = uint_val(v);
            m.attr.flags = v;
          } else if (mem.name == "key_size") {
            ok = uint_val(m.attr.key_size);
          } else if (mem.name == "value_size") {
            ok = uint_val(m.attr.value_size);
          } else if (mem.name == "key") {
            m.attr.key_size = (uint32_t)btf.size_of(pointee);
          } else if (mem.name == "value") {
            m.attr.value_size = (uint32_t)btf.size_of(pointee);
          } else if (mem.name == "numa_node" || mem.name == "pinning" || mem.name == "map_extra") {
            uint32_t v = 0;
            ok = uint_val(v);
          } else {
            return fail("map " + m.name + ": unsupported definition member '" + mem.name + "'");
          }
          if (!ok) return fail("map " + m.name + ": member " + mem.name + " is not a __uint");
        }
        maps.push_back(m);
      }
    }
    const int lm = sec_by_name("maps");
    if (lm >= 0) {  // legacy struct bpf_map_def {type, key_size, value_size, max_entries, map_flags}
      std::vector<size_t> ms;
      for (size_t s = 0; s < syms.size(); s++)
        if (syms[s].st_shndx == (unsigned)lm && ELF64_ST_TYPE(syms[s].st_info) != STT_SECTION &&
            ELF64_ST_TYPE(syms[s].st_info) != STT_FILE && !sym_names[s].empty())
          ms.push_back(s);
      if (ms.empty()) return fail("legacy maps section without map symbols");
      const uint64_t dsz = secs[lm].h.sh_size / ms.size();
      if (dsz < 16) return fail("legacy map definitions too small");
      for (size_t s : ms) {
        MapDef m;
        m.name = sym_names[s];
        m.sec = lm;
        m.sec_off = syms[s].st_value;
        if (m.sec_off + 16 > secs[lm].h.sh_size) return fail("legacy map " + m.name + " out of range");
        uint32_t w[5] = {0, 0, 0, 0, 0};
        memcpy(w, secs[lm].data + m.sec_off, dsz >= 20 ? 20 : 16);
        m.attr.type = (int)w[0];
        m.attr.key_size = w[1];
        m.attr.value_size = w[2];
        m.attr.max_ents = w[3];
        m.attr.flags = w[4];
        maps.push_back(m);
      }
    }
    // global data (libbpf internal maps): one-element ARRAYs named
    // <first 8 chars of the object>.<section>
    for (size_t i = 0; i < secs.size(); i++) {
      const Section &s = secs[i];
      const bool bss = s.name.compare(0, 4, ".bss") == 0, data = s.name.compare(0, 5, ".data") == 0,
                 ro = s.name.compare(0, 7, ".rodata") == 0;
      if (!(bss || data || ro) || s.h.sh_size == 0 || !(s.h.sh_flags & SHF_ALLOC)) continue;
      // libbpf internal_map_name(): suffix of at least 7 chars, the object
      // name's prefix in the rest of the 15, [^A-Za-z0-9_.] -> '_'
      MapDef m;
      const size_t sfx = std::max<size_t>(7, s.name.size());
      const size_t pfx = std::min<size_t>(sfx < 15 ? 15 - sfx : 0, name.size());
      m.name = (name.substr(0, pfx) + s.name.substr(0, sfx)).substr(0, 15);
      for (char &c : m.name)
        if (!isalnum((unsigned char)c) && c != '_' && c != '.') c = '_';
      m.sec = (int)i;
      m.internal = true;
      m.attr.type = 2;  // BPF_MAP_TYPE_ARRAY
      m.attr.key_size = 4;
      m.attr.value_size = (uint32_t)s.h.sh_size;
      m.attr.max_ents = 1;
      m.attr.flags = ro ? 0x80 /* BPF_F_RDONLY_PROG */ : 0x400 /* BPF_F_MMAPABLE */;
      if (!bss && s.h.sh_type != SHT_NOBITS) m.init.assign(s.data, s.data + s.h.sh_size);
      maps.push_back(m);
    }
    return 0;
  }

  int map_for_symbol(const Elf64_Sym &sym, int *src) const {
    for (size_t i = 0; i < maps.size(); i++) {
      const MapDef &m = maps[i];
      if ((int)sym.st_shndx != m.sec) continue;
      if (m.internal) {
        *src = 2;
        return (int)i;
      }
      if (m.sec_off == sym.st_value) {
        *src = 1;
        return (int)i;
      }
    }
    return -1;
  }

  // ---- programs ----
  int collect_progs() {
    for (size_t si = 0; si < secs.size(); si++) {
      const Section &s = secs[si];
      if (s.h.sh_type != SHT_PROGBITS || !(s.h.sh_flags & SHF_EXECINSTR) || s.name == ".text") continue;
      if (s.h.sh_size % 8) return fail("section " + s.name + " is not a whole number of instructions");
      std::vector<size_t> fs;
      for (size_t k = 0; k < syms.size(); k++)
        if (syms[k].st_shndx == si && ELF64_ST_TYPE(syms[k].st_info) == STT_FUNC &&
            ELF64_ST_BIND(syms[k].st_info) == STB_GLOBAL)
          fs.push_back(k);
      if (fs.empty()) return fail("program section " + s.name + " has no global function symbol");
      for (size_t k : fs) {
        Prog pr;
        pr.name = sym_names[k];
        pr.secname = s.name;
        pr.type = prog_type_of(s.name);
        uint64_t lo = syms[k].st_value, sz = syms[k].st_size ? syms[k].st_size : s.h.sh_size - lo;
        if (lo % 8 || sz % 8 || lo + sz > s.h.sh_size) return fail("function " + pr.name + " out of its section");
        pr.insns.assign(s.data + lo, s.data + lo + sz);
        // relocations of this section that fall inside the function
        for (const Section &r : secs) {
          if (r.h.sh_type != SHT_REL || r.h.sh_info != si) continue;
          const size_t cnt = r.h.sh_size / sizeof(Elf64_Rel);
          for (size_t j = 0; j < cnt; j++) {
            Elf64_Rel rel;
            memcpy(&rel, r.data + j * sizeof rel, sizeof rel);
            if (rel.r_offset < lo || rel.r_offset >= lo + sz) continue;
            const size_t ii = (rel.r_offset - lo) / 8;
            const uint32_t symi = (uint32_t)ELF64_R_SYM(rel.r_info), type = (uint32_t)ELF64_R_TYPE(rel.r_info);
            if (symi >= syms.size()) return fail("relocation against a bad symbol");
            const Elf64_Sym &sym = syms[symi];
            uint8_t *in = &pr.insns[ii * 8];
            if (in[0] == CALL || type == R_BPF_64_32)
              return fail("program " + pr.name + ": BPF-to-BPF call at insn " + std::to_string(ii) +
                          " (the reference VM patches every call as a helper, compat_ubpf.cpp:75-95)");
            if (type != R_BPF_64_64 || in[0] != LDDW || (ii + 1) * 8 >= pr.insns.size())
              return fail("program " + pr.name + ": unsupported relocation type " + std::to_string(type) +
                          " at insn " + std::to_string(ii));
            if (sym.st_shndx == SHN_UNDEF)
              return fail("program " + pr.name + ": extern symbol '" + sym_names[symi] + "' is not supported");
            Reloc rc;
            rc.insn = ii;
            rc.map = map_for_symbol(sym, &rc.src);
            if (rc.map < 0)
              return fail("program " + pr.name + ": relocation against '" + sym_names[symi] +
                          "' which is neither a map nor global data");
            int32_t imm;
            memcpy(&imm, in + 4, 4);
            rc.addend = (int64_t)imm + (rc.src == 2 ? (int64_t)sym.st_value : 0);
            pr.relocs.push_back(rc);
          }
        }
        progs.push_back(std::move(pr));
      }
    }
    if (progs.empty()) return fail("object has no programs");
    return 0;
  }

  // ---- CO-RE (.BTF.ext core_relo) ----
  int core_relocate() {
    const int ei = sec_by_name(".BTF.ext");
    if (ei < 0 || !has_btf) return 0;
    const uint8_t *p = secs[ei].data;
    const size_t n = secs[ei].h.sh_size;
    if (n < 32) return 0;
    uint32_t hdr_len, core_off, core_len;
    memcpy(&hdr_len, p + 4, 4);
    if (hdr_len < 32) return 0;  // no core_relo part
    memcpy(&core_off, p + 24, 4);
    memcpy(&core_len, p + 28, 4);
    if (!core_len) return 0;
    if ((uint64_t)hdr_len + core_off + core_len > n) return fail(".BTF.ext core_relo out of range");
    const uint8_t *c = p + hdr_len + core_off, *end = c + core_len;
    uint32_t rec;
    memcpy(&rec, c, 4);
    c += 4;
    if (rec < 16) return fail(".BTF.ext: bad core_relo record size");
    // strings of .BTF (access strings and section names)
    const int bi = sec_by_name(".BTF");
    uint32_t bh, s_off, s_len;
    memcpy(&bh, secs[bi].data + 4, 4);
    memcpy(&s_off, secs[bi].data + 16, 4);
    memcpy(&s_len, secs[bi].data + 20, 4);
    const char *bs = (const char *)secs[bi].data + bh + s_off;
    auto bstr = [&](uint32_t o) { return o < s_len ? std::string(bs + o, strnlen(bs + o, s_len - o)) : std::string(); };
    const Btf &tgt = has_target ? target : target_builtin();
    while (c + 8 <= end) {
      uint32_t sec_name_off, num;
      memcpy(&sec_name_off, c, 4);
      memcpy(&num, c + 4, 4);
      c += 8;
      const std::string sec = bstr(sec_name_off);
      for (uint32_t k = 0; k < num; k++, c += rec) {
        if (c + 16 > end) return fail(".BTF.ext: truncated core_relo");
        uint32_t insn_off, type_id, acc_off, kind;
        memcpy(&insn_off, c, 4);
        memcpy(&type_id, c + 4, 4);
        memcpy(&acc_off, c + 8, 4);
        memcpy(&kind, c + 12, 4);
        if (apply_core(sec, insn_off, type_id, bstr(acc_off), kind, tgt) < 0) return -1;
      }
    }
    return 0;
  }

  static const Btf &target_builtin() {
    static Btf b;
    static bool init = false;
    if (!init) {
      builtin_target(b);
      init = true;
    }
    return b;
  }

  int apply_core(const std::string &sec, uint32_t insn_off, uint32_t type_id, const std::string &acc,
                 uint32_t kind, const Btf &tgt) {
    // programs of this section containing the instruction
    Prog *pr = nullptr;
    uint64_t base = 0;
    const int si = sec_by_name(sec);
    for (Prog &q : progs) {
      if (q.secname != sec) continue;
      for (size_t k = 0; k < syms.size(); k++)
        if ((int)syms[k].st_shndx == si && sym_names[k] == q.name &&
            insn_off >= syms[k].st_value && insn_off < syms[k].st_value + q.insns.size()) {
          pr = &q;
          base = syms[k].st_value;
        }
    }
    if (!pr) return 0;  // relocation in a subprogram no program uses
    uint8_t *in = &pr->insns[insn_off - base];
    std::vector<int64_t> spec;
    {
      size_t i = 0;
      while (i < acc.size()) {
        size_t j = acc.find(':', i);
        if (j == std::string::npos) j = acc.size();
        spec.push_back(strtoll(acc.substr(i, j - i).c_str(), nullptr, 10));
        i = j + 1;
      }
    }
    const uint32_t lroot = btf.skip(type_id);
    const BType *lt = btf.at(lroot);
    if (!lt) return fail("CO-RE: bad local type id " + std::to_string(type_id));
    const std::string ename = essential_name(lt->name);
    int64_t val = 0;
    uint64_t new_sz = 0, old_sz = 0;
    bool found = false, sized_field = false, int_field = false;
    if (kind <= 5) {  // field relocations
      const Access la = walk_local(btf, lroot, spec);
      if (!la.ok) return fail("CO-RE: bad access string '" + acc + "' on " + lt->name);
      if (la.bitfield && kind <= 1) return fail("CO-RE: bitfield access " + lt->name + " '" + acc + "' unsupported");
      Access ta;
      auto cands = tgt.find(ename, lt->kind);
      for (uint32_t cand : cands) {
        ta = walk_target(tgt, cand, spec, la.names);
        if (ta.ok) break;
      }
      if (cands.empty()) ta = la;  // type unknown to the target: keep the object's own layout
      found = ta.ok;
      old_sz = la.size;
      new_sz = ta.size;
      const BType *ft = tgt.at(ta.type);
      int_field = ft && (ft->kind == K_INT || ft->kind == K_ENUM || ft->kind == K_ENUM64 || ft->kind == K_PTR);
      sized_field = true;
      switch (kind) {
        case 0: val = ta.off; break;                         // FIELD_BYTE_OFFSET
        case 1: val = (int64_t)ta.size; break;               // FIELD_BYTE_SIZE
        case 2: val = found ? 1 : 0; found = true; break;    // FIELD_EXISTS
        case 3: {                                            // FIELD_SIGNED
          const BType *t = tgt.at(ta.type);
          val = t && ((t->kind == K_INT && (t->enc >> 24) & 1) || t->kind == K_ENUM) ? 1 : 0;
          break;
        }
        default:
          return fail("CO-RE: relocation kind " + std::to_string(kind) + " (bitfield shifts) unsupported");
      }
    } else if (kind == 8 || kind == 9 || kind == 12) {  // TYPE_EXISTS / TYPE_SIZE / TYPE_MATCHES
      auto cands = tgt.find(ename, lt->kind);
      const bool have = !cands.empty() || !has_target;
      const uint32_t tid = cands.empty() ? lroot : cands[0];
      const Btf &src = cands.empty() ? btf : tgt;
      val = kind == 9 ? (int64_t)src.size_of(tid) : (have ? 1 : 0);
      found = true;
    } else {
      return fail("CO-RE: relocation kind " + std::to_string(kind) + " unsupported");
    }
    if (!found) {
      // libbpf poisons an instruction whose field is missing in the target
      // (bpf_core_poison_insn): a call to the invalid helper 0xbad2310
      memset(in, 0, 8);
      in[0] = CALL;
      const int32_t bad = 0xbad2310;
      memcpy(in + 4, &bad, 4);
      return 0;
    }
    const uint8_t cls = in[0] & 7;
    if (cls == 1 || cls == 2 || cls == 3) {  // LDX / ST / STX: offset (and size) of the access
      if (val < -32768 || val > 32767) return fail("CO-RE: field offset out of range");
      const int16_t off = (int16_t)val;
      memcpy(in + 2, &off, 2);
      if (kind == 0 && sized_field && new_sz != old_sz) {
        if (!int_field) return fail("CO-RE: size of non-integer field changed at insn " + std::to_string(insn_off / 8));
        uint8_t szc;
        switch (new_sz) {
          case 1: szc = 0x10; break;
          case 2: szc = 0x08; break;
          case 4: szc = 0x00; break;
          case 8: szc = 0x18; break;
          default: return fail("CO-RE: unsupported target field size");
        }
        in[0] = (uint8_t)((in[0] & 0xe7) | szc);
      }
    } else if ((cls == 4 || cls == 7) && !(in[0] & 0x08)) {  // ALU/ALU64 with an immediate
      const int32_t imm = (int32_t)val;
      memcpy(in + 4, &imm, 4);
    } else if (in[0] == LDDW) {
      const int32_t lo = (int32_t)val, hi = (int32_t)(val >> 32);
      memcpy(in + 4, &lo, 4);
      memcpy(in + 12, &hi, 4);
    } else {
      return fail("CO-RE: cannot patch instruction at byte " + std::to_string(insn_off) + " of " + sec);
    }
    return 0;
  }

  // final instructions for a map fd assignment
  void relocated(const Prog &pr, const int *fds, std::vector<uint8_t> &out) const {
    out = pr.insns;
    for (const Reloc &rc : pr.relocs) {
      uint8_t *in = &out[rc.insn * 8];
      in[1] = (uint8_t)((in[1] & 0x0f) | (rc.src << 4));
      const int32_t fd = fds[rc.map];
      memcpy(in + 4, &fd, 4);
      const int32_t nx = rc.src == 2 ? (int32_t)rc.addend : 0;
      memcpy(in + 12, &nx, 4);
    }
  }
};

extern "C" {

struct bpftime_object *bpftime_object_open_mem(const void *buf, size_t len, const char *name) {
  bpftime_object *o = new bpftime_object();
  o->buf.assign((const uint8_t *)buf, (const uint8_t *)buf + len);
  o->name = name ? name : "obj";
  if (o->parse() < 0 || o->core_relocate() < 0) return o;  // error kept in the object
  return o;
}

struct bpftime_object *bpftime_object_open(const char *obj_path) {
  FILE *f = obj_path ? fopen(obj_path, "rb") : nullptr;
  if (!f) return nullptr;
  std::vector<uint8_t> b;
  uint8_t tmp[65536];
  size_t r;
  while ((r = fread(tmp, 1, sizeof tmp, f)) > 0) b.insert(b.end(), tmp, tmp + r);
  fclose(f);
  std::string base = obj_path;
  const size_t sl = base.rfind('/');
  if (sl != std::string::npos) base = base.substr(sl + 1);
  const size_t dot = base.find('.');
  if (dot != std::string::npos) base = base.substr(0, dot);
  return bpftime_object_open_mem(b.data(), b.size(), base.c_str());
}

const char *bpftime_object_error(const struct bpftime_object *obj) {
  return obj ? obj->error.c_str() : "no object";
}

int bpftime_object_load_relocate_btf_mem(struct bpftime_object *obj, const void *btf, size_t len) {
  if (!obj || !obj->error.empty()) return -1;
  if (obj->loaded) return obj->fail("object already loaded");
  std::string err;
  if (!obj->target.parse((const uint8_t *)btf, len, err)) return obj->fail("target BTF: " + err);
  obj->has_target = true;
  // re-run CO-RE from the original instructions against the new target
  obj->progs.clear();
  obj->maps.clear();
  if (obj->collect_maps() < 0 || obj->collect_progs() < 0 || obj->core_relocate() < 0) return -1;
  return 0;
}

int bpftime_object_load_relocate_btf(struct bpftime_object *obj, const char *btf_path) {
  FILE *f = btf_path ? fopen(btf_path, "rb") : nullptr;
  if (!f) return obj ? obj->fail(std::string("cannot open ") + (btf_path ? btf_path : "(null)")) : -1;
  std::vector<uint8_t> b;
  uint8_t tmp[65536];
  size_t r;
  while ((r = fread(tmp, 1, sizeof tmp, f)) > 0) b.insert(b.end(), tmp, tmp + r);
  fclose(f);
  return bpftime_object_load_relocate_btf_mem(obj, b.data(), b.size());
}

int bpftime_object_map_count(const struct bpftime_object *obj) {
  return obj && obj->error.empty() ? (int)obj->maps.size() : -1;
}

int bpftime_object_map_info(const struct bpftime_object *obj, int idx, const char **name,
                            struct bpf_map_attr *attr) {
  if (!obj || idx < 0 || idx >= (int)obj->maps.size()) return -1;
  if (name) *name = obj->maps[idx].name.c_str();
  if (attr) *attr = obj->maps[idx].attr;
  return 0;
}

int bpftime_object_program_count(const struct bpftime_object *obj) {
  return obj && obj->error.empty() ? (int)obj->progs.size() : -1;
}

int bpftime_object_program_info(const struct bpftime_object *obj, int idx, const char **name,
                                const char **secname, int *prog_type, size_t *insn_cnt) {
  if (!obj || idx < 0 || idx >= (int)obj->progs.size()) return -1;
  const Prog &p = obj->progs[idx];
  if (name) *name = p.name.c_str();
  if (secname) *secname = p.secname.c_str();
  if (prog_type) *prog_type = p.type;
  if (insn_cnt) *insn_cnt = p.insns.size() / 8;
  return 0;
}

int bpftime_object_program_insns(const struct bpftime_object *obj, int idx, const int *map_fds, void *out,
                                 size_t insn_cap) {
  if (!obj || idx < 0 || idx >= (int)obj->progs.size() || !map_fds) return -1;
  std::vector<uint8_t> v;
  obj->relocated(obj->progs[idx], map_fds, v);
  if (v.size() / 8 > insn_cap) return -1;
  memcpy(out, v.data(), v.size());
  return (int)(v.size() / 8);
}

int bpftime_object_load(struct bpftime_object *obj) {
  if (!obj || !obj->error.empty()) return -1;
  if (obj->loaded) return 0;
  obj->map_fds.assign(obj->maps.size(), -1);
  for (size_t i = 0; i < obj->maps.size(); i++) {
    const MapDef &m = obj->maps[i];
    const int fd = bpftime_maps_create(-1, m.name.c_str(), m.attr);
    if (fd < 0) return obj->fail("cannot create map " + m.name + ": " + bpftime_amd_last_error());
    obj->map_fds[i] = fd;
    if (!m.init.empty()) {
      const uint32_t k0 = 0;
      if (bpftime_map_update_elem(fd, &k0, m.init.data(), 0) < 0)
        return obj->fail("cannot initialise map " + m.name);
    }
  }
  for (Prog &p : obj->progs) {
    std::vector<uint8_t> v;
    obj->relocated(p, obj->map_fds.data(), v);
    p.fd = bpftime_progs_create(-1, v.data(), v.size() / 8, p.name.c_str(), p.type);
    if (p.fd < 0) return obj->fail("cannot create program " + p.name);
  }
  obj->loaded = true;
  return 0;
}

int bpftime_object_find_program_by_name(const struct bpftime_object *obj, const char *name) {
  if (!obj || !name || !obj->loaded) return -1;
  for (const Prog &p : obj->progs)
    if (p.name == name) return p.fd;
  return -1;
}

int bpftime_object_find_program_by_secname(const struct bpftime_object *obj, const char *secname) {
  if (!obj || !secname || !obj->loaded) return -1;
  for (const Prog &p : obj->progs)
    if (p.secname == secname) return p.fd;
  return -1;
}

int bpftime_object_find_map_fd_by_name(const struct bpftime_object *obj, const char *name) {
  if (!obj || !name || !obj->loaded) return -1;
  for (size_t i = 0; i < obj->maps.size(); i++)
    if (obj->maps[i].name == name) return obj->map_fds[i];
  return -1;
}

const char *bpftime_object_license(const struct bpftime_object *obj) { return obj ? obj->license.c_str() : ""; }

void bpftime_object_close(struct bpftime_object *obj) { delete obj; }

}  // extern "C"

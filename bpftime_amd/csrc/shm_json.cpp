// bpftime_amd: the reference's handler JSON format.
//
// bpftime moves its shared-memory state between processes and tools as JSON
// (runtime/src/bpftime_shm_json.cpp:103-327, `bpftimetool export/import`):
//
//   { "<fd>": {"type": "bpf_map_handler",  "name": ..., "attr": {map_type,
//              key_size, value_size, max_entries, flags, ifindex, btf_*,
//              map_extra, kernel_bpf_map_id}},
//     "<fd>": {"type": "bpf_prog_handler", "name": ..., "attr": {type,
//              insns: hex bytes, cnt, attach_fds?}},
//     "<fd>": {"type": "bpf_link_handler", "attr": {prog_fd, target_fd}} }
//
// Importing such a file recreates the records at the same fds in this
// runtime's registry (maps in HBM), so state loaded by the reference's
// libbpf path (real clang objects, LD_PRELOAD syscall server) runs on the
// GPU unchanged.  The format does not keep a link's attach type; a link to an
// XDP program (prog type 6) is taken as a BPF_XDP link, since that is the
// only kind this runtime executes.  Handler kinds outside this path (perf
// events, epoll, memfd) are rejected, as the reference rejects the kinds it
// cannot import.  Host-only code.
#include <ctype.h>
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/bpftime_amd.h"
#include "runtime.hpp"

namespace {

// ---- a minimal JSON value / parser / writer --------------------------------
struct J {
  enum K { NUL, BOOL, NUM, STR, ARR, OBJ } k = NUL;
  bool b = false;
  double n = 0;
  bool is_int = false;
  long long i = 0;
  std::string s;
  std::vector<J> a;
  std::vector<std::pair<std::string, J>> o;  // insertion order kept
  const J *get(const std::string &key) const {
    for (auto &kv : o)
      if (kv.first == key) return &kv.second;
    return nullptr;
  }
};

struct Parser {
  const char *p, *e;
  std::string err;
  void ws() {
    while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) p++;
  }
  bool fail(const char *m) {
    if (err.empty()) err = m;
    return false;
  }
  bool str(std::string &out) {
    if (p >= e || *p != '"') return fail("expected string");
    p++;
    while (p < e && *p != '"') {
      if (*p == '\\') {
        if (++p >= e) return fail("bad escape");
        switch (*p) {
          case 'n': out += '\n'; break;
          case 't': out += '\t'; break;
          case 'r': out += '\r'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'u': {
            if (e - p < 5) return fail("bad \\u escape");
            unsigned v = (unsigned)strtoul(std::string(p + 1, 4).c_str(), nullptr, 16);
            if (v < 0x80) {
              out += (char)v;
            } else if (v < 0x800) {
              out += (char)(0xc0 | (v >> 6));
              out += (char)(0x80 | (v & 0x3f));
            } else {
              out += (char)(0xe0 | (v >> 12));
              out += (char)(0x80 | ((v >> 6) & 0x3f));
              out += (char)(0x80 | (v & 0x3f));
            }
            p += 4;
            break;
          }
          default: out += *p;
        }
        p++;
      } else {
        out += *p++;
      }
    }
    if (p >= e) return fail("unterminated string");
    p++;
    return true;
  }
  bool val(J &v, int depth = 0) {
    if (depth > 64) return fail("nesting too deep");
    ws();
    if (p >= e) return fail("unexpected end");
    if (*p == '{') {
      v.k = J::OBJ;
      p++;
      ws();
      if (p < e && *p == '}') {
        p++;
        return true;
      }
      for (;;) {
        ws();
        std::string key;
        if (!str(key)) return false;
        ws();
        if (p >= e || *p != ':') return fail("expected ':'");
        p++;
        J x;
        if (!val(x, depth + 1)) return false;
        v.o.emplace_back(std::move(key), std::move(x));
        ws();
        if (p < e && *p == ',') {
          p++;
          continue;
        }
        if (p < e && *p == '}') {
          p++;
          return true;
        }
        return fail("expected ',' or '}'");
      }
    }
    if (*p == '[') {
      v.k = J::ARR;
      p++;
      ws();
      if (p < e && *p == ']') {
        p++;
        return true;
      }
      for (;;) {
        J x;
        if (!val(x, depth + 1)) return false;
        v.a.push_back(std::move(x));
        ws();
        if (p < e && *p == ',') {
          p++;
          continue;
        }
        if (p < e && *p == ']') {
          p++;
          return true;
        }
        return fail("expected ',' or ']'");
      }
    }
    if (*p == '"') {
      v.k = J::STR;
      return str(v.s);
    }
    if (e - p >= 4 && !strncmp(p, "true", 4)) {
      v.k = J::BOOL;
      v.b = true;
      p += 4;
      return true;
    }
    if (e - p >= 5 && !strncmp(p, "false", 5)) {
      v.k = J::BOOL;
      p += 5;
      return true;
    }
    if (e - p >= 4 && !strncmp(p, "null", 4)) {
      p += 4;
      return true;
    }
    const char *s = p;
    bool frac = false;
    while (p < e && (isdigit((unsigned char)*p) || *p == '-' || *p == '+' || *p == '.' || *p == 'e' || *p == 'E')) {
      if (*p == '.' || *p == 'e' || *p == 'E') frac = true;
      p++;
    }
    if (s == p) return fail("unexpected character");
    std::string t(s, p);
    v.k = J::NUM;
    v.n = strtod(t.c_str(), nullptr);
    if (!frac) {
      v.is_int = true;
      v.i = t[0] == '-' ? strtoll(t.c_str(), nullptr, 10) : (long long)strtoull(t.c_str(), nullptr, 10);
    }
    return true;
  }
};

bool parse(const std::string &text, J &out, std::string &err) {
  Parser ps{text.data(), text.data() + text.size(), ""};
  if (!ps.val(out)) {
    err = ps.err;
    return false;
  }
  ps.ws();
  if (ps.p != ps.e) {
    err = "trailing characters";
    return false;
  }
  return true;
}

long long num(const J *v, bool *ok) {
  if (!v || v->k != J::NUM) {
    *ok = false;
    return 0;
  }
  return v->is_int ? v->i : (long long)v->n;
}

std::string quote(const std::string &s) {
  std::string o = "\"";
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') {
      o += '\\';
      o += (char)c;
    } else if (c < 0x20) {
      char buf[8];
      snprintf(buf, sizeof buf, "\\u%04x", c);
      o += buf;
    } else {
      o += (char)c;
    }
  }
  return o + "\"";
}

// bpftime_shm_json.hpp:17-41 (lowercase hex, two digits per byte)
std::string to_hex(const uint8_t *b, size_t n) {
  static const char *d = "0123456789abcdef";
  std::string s(2 * n, '0');
  for (size_t i = 0; i < n; i++) {
    s[2 * i] = d[b[i] >> 4];
    s[2 * i + 1] = d[b[i] & 15];
  }
  return s;
}

bool from_hex(const std::string &s, std::vector<uint8_t> &out, size_t n) {
  if (s.size() != 2 * n) return false;
  out.resize(n);
  for (size_t i = 0; i < n; i++) {
    char t[3] = {s[2 * i], s[2 * i + 1], 0};
    char *end;
    out[i] = (uint8_t)strtoul(t, &end, 16);
    if (*end) return false;
  }
  return true;
}

int import_handler(int fd, const J &v, std::string &err) {
  using namespace bpftime_amd;
  const J *type = v.get("type");
  const J *attr = v.get("attr");
  if (!type || type->k != J::STR || !attr || attr->k != J::OBJ) {
    err = "handler without type / attr";
    return -1;
  }
  const J *name = v.get("name");
  const std::string nm = name && name->k == J::STR ? name->s : "";
  bool ok = true;
  if (type->s == "bpf_map_handler") {
    bpf_map_attr a{};
    a.type = (int)num(attr->get("map_type"), &ok);
    a.key_size = (uint32_t)num(attr->get("key_size"), &ok);
    a.value_size = (uint32_t)num(attr->get("value_size"), &ok);
    a.max_ents = (uint32_t)num(attr->get("max_entries"), &ok);
    a.flags = (uint64_t)num(attr->get("flags"), &ok);
    bool opt = true;  // fields the reference writes but this runtime does not need
    a.ifindex = (uint32_t)num(attr->get("ifindex"), &opt);
    a.btf_vmlinux_value_type_id = (uint32_t)num(attr->get("btf_vmlinux_value_type_id"), &opt);
    a.btf_id = (uint32_t)num(attr->get("btf_id"), &opt);
    a.btf_key_type_id = (uint32_t)num(attr->get("btf_key_type_id"), &opt);
    a.btf_value_type_id = (uint32_t)num(attr->get("btf_value_type_id"), &opt);
    a.map_extra = (uint64_t)num(attr->get("map_extra"), &opt);
    a.kernel_bpf_map_id = (uint32_t)num(attr->get("kernel_bpf_map_id"), &opt);
    if (!ok) {
      err = "map " + std::to_string(fd) + ": missing attribute";
      return -1;
    }
    if (bpftime_maps_create(fd, nm.c_str(), a) != fd) {
      err = "map " + std::to_string(fd) + ": " + bpftime_amd_last_error();
      return -1;
    }
    return 0;
  }
  if (type->s == "bpf_prog_handler") {
    const int ptype = (int)num(attr->get("type"), &ok);
    const long long cnt = num(attr->get("cnt"), &ok);
    const J *insns = attr->get("insns");
    std::vector<uint8_t> code;
    if (!ok || cnt < 0 || !insns || insns->k != J::STR || !from_hex(insns->s, code, (size_t)cnt * 8)) {
      err = "prog " + std::to_string(fd) + ": bad insns";
      return -1;
    }
    if (bpftime_progs_create(fd, code.data(), (size_t)cnt, nm.c_str(), ptype) != fd) {
      err = "prog " + std::to_string(fd) + ": cannot create";
      return -1;
    }
    return 0;
  }
  if (type->s == "bpf_link_handler") {
    bpf_link_create_args a{};
    a.prog_fd = (uint32_t)num(attr->get("prog_fd"), &ok);
    a.target_fd = (uint32_t)num(attr->get("target_fd"), &ok);
    if (!ok) {
      err = "link " + std::to_string(fd) + ": missing prog_fd / target_fd";
      return -1;
    }
    {
      Runtime &r = rt();
      std::lock_guard<std::mutex> g(r.mu);
      if (a.prog_fd < kMaxFds && r.kind[a.prog_fd] == HKind::PROG && r.progs[a.prog_fd].type == BPFTIME_AMD_PROG_TYPE_XDP)
        a.attach_type = BPFTIME_AMD_BPF_XDP;
    }
    if (bpftime_link_create(fd, &a) != fd) {
      err = "link " + std::to_string(fd) + ": prog fd " + std::to_string(a.prog_fd) + " is not a program";
      return -1;
    }
    return 0;
  }
  err = "unsupported handler type " + type->s;
  return -1;
}

bool read_file(const char *path, std::string &out) {
  FILE *f = path ? fopen(path, "rb") : nullptr;
  if (!f) return false;
  char buf[65536];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) out.append(buf, n);
  fclose(f);
  return true;
}

}  // namespace

extern "C" {

int bpftime_import_shm_handler_from_json(int fd, const char *json_string) {
  J v;
  std::string err;
  if (!json_string || !parse(json_string, v, err) || v.k != J::OBJ) {
    bpftime_amd::set_error("handler json: " + (err.empty() ? std::string("not an object") : err));
    errno = EINVAL;
    return -1;
  }
  if (import_handler(fd, v, err) < 0) {
    bpftime_amd::set_error(err);
    errno = EINVAL;
    return -1;
  }
  return 0;
}

int bpftime_import_global_shm_from_json(const char *filename) {
  std::string text, err;
  J root;
  if (!read_file(filename, text)) {
    bpftime_amd::set_error(std::string("cannot read ") + (filename ? filename : "(null)"));
    errno = ENOENT;
    return -1;
  }
  if (!parse(text, root, err) || root.k != J::OBJ) {
    bpftime_amd::set_error("shm json: " + (err.empty() ? std::string("not an object") : err));
    errno = EINVAL;
    return -1;
  }
  // maps and programs before links (a link names its program's fd)
  for (int pass = 0; pass < 2; pass++)
    for (auto &kv : root.o) {
      const J *t = kv.second.get("type");
      const bool link = t && t->k == J::STR && t->s == "bpf_link_handler";
      if (link != (pass == 1)) continue;
      char *end;
      const long fd = strtol(kv.first.c_str(), &end, 10);
      if (*end || fd < 0) {
        bpftime_amd::set_error("shm json: bad fd key '" + kv.first + "'");
        errno = EINVAL;
        return -1;
      }
      if (import_handler((int)fd, kv.second, err) < 0) {
        bpftime_amd::set_error(err);
        errno = EINVAL;
        return -1;
      }
    }
  return 0;
}

int bpftime_export_global_shm_to_json(const char *filename) {
  using namespace bpftime_amd;
  Runtime &r = rt();
  std::string out = "{";
  bool first = true;
  {
    std::lock_guard<std::mutex> g(r.mu);
    for (uint32_t fd = 0; fd < kMaxFds; fd++) {
      std::string item;
      if (r.kind[fd] == HKind::MAP) {
        const MapRec &m = r.maps[fd];
        char buf[512];
        snprintf(buf, sizeof buf,
                 "{\"attr\": {\"btf_id\": 0, \"btf_key_type_id\": 0, \"btf_value_type_id\": 0, "
                 "\"btf_vmlinux_value_type_id\": 0, \"flags\": %llu, \"ifindex\": 0, \"kernel_bpf_map_id\": 0, "
                 "\"key_size\": %u, \"map_extra\": 0, \"map_type\": %u, \"max_entries\": %u, \"value_size\": %u}, ",
                 (unsigned long long)m.flags, m.key_size, m.type, m.max_entries, m.value_size);
        item = std::string(buf) + "\"name\": " + quote(m.name) + ", \"type\": \"bpf_map_handler\"}";
      } else if (r.kind[fd] == HKind::PROG) {
        const ProgRec &p = r.progs[fd];
        item = "{\"attr\": {\"cnt\": " + std::to_string(p.insns.size() / 8) + ", \"insns\": \"" +
               to_hex(p.insns.data(), p.insns.size()) + "\", \"type\": " + std::to_string(p.type) +
               "}, \"name\": " + quote(p.name) + ", \"type\": \"bpf_prog_handler\"}";
      } else if (r.kind[fd] == HKind::LINK) {
        const LinkRec &l = r.links[fd];
        item = "{\"attr\": {\"prog_fd\": " + std::to_string(l.prog_fd) + ", \"target_fd\": " +
               std::to_string(l.target) + "}, \"type\": \"bpf_link_handler\"}";
      } else {
        continue;
      }
      out += std::string(first ? "\n" : ",\n") + "    \"" + std::to_string(fd) + "\": " + item;
      first = false;
    }
  }
  out += "\n}\n";
  FILE *f = filename ? fopen(filename, "wb") : nullptr;
  if (!f) {
    set_error(std::string("cannot write ") + (filename ? filename : "(null)"));
    return -1;
  }
  const bool ok = fwrite(out.data(), 1, out.size(), f) == out.size();
  fclose(f);
  return ok ? 0 : -1;
}

}  // extern "C"

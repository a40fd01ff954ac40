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
//     "<fd>": {"type": "bpf_perf_event_handler", "enabled": bool, "attr":
//              {type, pid, tracepoint_id | offset, ref_ctr_off, _module_name
//              | cpu, sample_type, config}},
//     "<fd>": {"type": "bpf_link_handler", "attr": {prog_fd, target_fd}} }
//
// Importing such a file recreates the records at the same fds in this
// runtime's registry (maps in HBM), so state loaded by the reference's
// libbpf path (real clang objects, LD_PRELOAD syscall server) runs on the
// GPU unchanged.  The format does not keep a link's attach type: a link
// whose target is a perf event record (and whose program is not XDP) is a
// perf link, and one to a syscall sys_enter tracepoint attaches its program
// to the replay dispatch (tracepoint id -> syscall number as the reference
// resolves it, tracepoints.cpp); a link to an XDP program is a BPF_XDP link.
// A prog's `attach_fds` (:123-125) become links at fresh fds, after every
// record of the file exists.  Perf events that run nothing on this path
// (uprobes, software events, sys_exit tracepoints) are kept as records.
// Handler kinds outside this path (epoll, memfd) are rejected, as the
// reference rejects the kinds it cannot import.  Export writes what the
// reference's export writes (:235-327: attachments as link records, no
// attach_fds -- its comment at :271 has no code behind it, and writing both
// would attach twice on re-import), plus "sys_nr" beside a tracepoint made
// from a syscall number when the tracefs has no id for it.  Host-only code.
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

// attach: where a prog's attach_fds go ({prog fd, perf fd}), linked by the
// caller once the records they name exist
int import_handler(int fd, const J &v, std::string &err, std::vector<std::pair<int, int>> *attach) {
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
    if (const J *af = attr->get("attach_fds")) {
      if (af->k != J::ARR && af->k != J::NUL) {
        err = "prog " + std::to_string(fd) + ": attach_fds is not an array";
        return -1;
      }
      for (const J &x : af->a) {
        bool k = true;
        const long long t = num(&x, &k);
        if (!k) {
          err = "prog " + std::to_string(fd) + ": bad attach fd";
          return -1;
        }
        if (attach) attach->emplace_back(fd, (int)t);
      }
    }
    return 0;
  }
  if (type->s == "bpf_perf_event_handler") {
    bpftime_amd_perf_event e{};
    e.type = (int)num(attr->get("type"), &ok);
    e.pid = (int)num(attr->get("pid"), &ok);
    e.tracepoint_id = -1;
    e.sys_nr = -1;
    std::string module;
    switch (e.type) {
      case 2: {  // PERF_TYPE_TRACEPOINT
        e.tracepoint_id = (int32_t)num(attr->get("tracepoint_id"), &ok);
        bool has = true;
        const long long nr = num(attr->get("sys_nr"), &has);  // (this runtime's export, see above)
        if (has && e.tracepoint_id < 0) e.sys_nr = nr;
        break;
      }
      case 6:  // BPF_TYPE_UPROBE
      case 7:  // BPF_TYPE_URETPROBE
        e.ref_ctr_off = (uint64_t)num(attr->get("ref_ctr_off"), &ok);
        /* fall through */
      case 1008: {  // BPF_TYPE_UPROBE_OVERRIDE
        e.offset = (uint64_t)num(attr->get("offset"), &ok);
        const J *mn = attr->get("_module_name");
        if (!mn || mn->k != J::STR) ok = false;
        else module = mn->s;
        e.module_name = module.c_str();
        break;
      }
      case 1:  // PERF_TYPE_SOFTWARE
        e.cpu = (int)num(attr->get("cpu"), &ok);
        e.sample_type = (int32_t)num(attr->get("sample_type"), &ok);
        e.config = (int64_t)num(attr->get("config"), &ok);
        break;
      default:
        err = "perf event " + std::to_string(fd) + ": Unsupported perf event type " + std::to_string(e.type);
        return -1;
    }
    if (!ok) {
      err = "perf event " + std::to_string(fd) + ": missing attribute";
      return -1;
    }
    const J *en = v.get("enabled");
    e.enabled = en && en->k == J::BOOL && en->b;
    if (bpftime_amd_perf_event_record(fd, &e) != fd) {
      err = "perf event " + std::to_string(fd) + ": cannot create";
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
    bool xdp = false, perf = false;
    {
      Runtime &r = rt();
      std::lock_guard<std::mutex> g(r.mu);
      xdp = a.prog_fd < kMaxFds && r.kind[a.prog_fd] == HKind::PROG && r.progs[a.prog_fd].type == BPFTIME_AMD_PROG_TYPE_XDP;
      perf = a.target_fd < kMaxFds && r.kind[a.target_fd] == HKind::PERF;
    }
    if (xdp) a.attach_type = BPFTIME_AMD_BPF_XDP;
    if (perf && !xdp) {
      if (bpftime_amd_link_perf(fd, (int)a.prog_fd, (int)a.target_fd) != fd) {
        err = "link " + std::to_string(fd) + ": prog fd " + std::to_string(a.prog_fd) + " -> perf event " +
              std::to_string(a.target_fd) + ": " + bpftime_amd_last_error();
        return -1;
      }
      return 0;
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

// add_bpf_prog_attach_target (bpftime_shm_internal.cpp:293-315): a link
// at a fresh fd; the target is not checked there, so a target that is no
// perf event gives a plain link record
int link_attach_fds(const std::vector<std::pair<int, int>> &attach, std::string &err) {
  for (const auto &pa : attach) {
    int rc;
    if (bpftime_is_perf_event_fd(pa.second)) {
      rc = bpftime_amd_link_perf(-1, pa.first, pa.second);
    } else {
      bpf_link_create_args a{};
      a.prog_fd = (uint32_t)pa.first;
      a.target_fd = (uint32_t)pa.second;
      rc = bpftime_link_create(-1, &a);
    }
    if (rc < 0) {
      err = "prog " + std::to_string(pa.first) + ": attach fd " + std::to_string(pa.second) + ": " +
            bpftime_amd_last_error();
      return -1;
    }
  }
  return 0;
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
  std::vector<std::pair<int, int>> attach;
  if (import_handler(fd, v, err, &attach) < 0 || link_attach_fds(attach, err) < 0) {
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
  // maps, programs and perf events before links (a link names its program
  // and its target), a prog's attach_fds last
  std::vector<std::pair<int, int>> attach;
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
      if (import_handler((int)fd, kv.second, err, &attach) < 0) {
        bpftime_amd::set_error(err);
        errno = EINVAL;
        return -1;
      }
    }
  if (link_attach_fds(attach, err) < 0) {
    bpftime_amd::set_error(err);
    errno = EINVAL;
    return -1;
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
                 "{\"attr\": {\"btf_id\": %u, \"btf_key_type_id\": %u, \"btf_value_type_id\": %u, "
                 "\"btf_vmlinux_value_type_id\": %u, \"flags\": %llu, \"ifindex\": %u, \"kernel_bpf_map_id\": %u, "
                 "\"key_size\": %u, \"map_extra\": %llu, \"map_type\": %u, \"max_entries\": %u, \"value_size\": %u}, ",
                 m.btf_id, m.btf_key_type_id, m.btf_value_type_id, m.btf_vmlinux_value_type_id,
                 (unsigned long long)m.flags, m.ifindex, m.kernel_bpf_map_id, m.key_size,
                 (unsigned long long)m.map_extra, m.type, m.max_entries, m.value_size);
        item = std::string(buf) + "\"name\": " + quote(m.name) + ", \"type\": \"bpf_map_handler\"}";
      } else if (r.kind[fd] == HKind::PROG) {
        const ProgRec &p = r.progs[fd];
        item = "{\"attr\": {\"cnt\": " + std::to_string(p.insns.size() / 8) + ", \"insns\": \"" +
               to_hex(p.insns.data(), p.insns.size()) + "\", \"type\": " + std::to_string(p.type) +
               "}, \"name\": " + quote(p.name) + ", \"type\": \"bpf_prog_handler\"}";
      } else if (r.kind[fd] == HKind::PERF) {
        // bpf_perf_event_handler_attr_to_json (:66-95), keys in its order
        const PerfRec &p = r.perfs[fd];
        std::string a;
        if (p.type == 6 || p.type == 7 || p.type == 1008) {
          a = "\"_module_name\": " + quote(p.module) + ", \"data_type\": \"uprobe_perf_event_data\", \"offset\": " +
              std::to_string(p.offset) + ", \"pid\": " + std::to_string(p.pid) + ", \"ref_ctr_off\": " +
              std::to_string(p.ref_ctr_off) + ", ";
        } else if (p.type == 2) {
          int32_t id = p.tracepoint_id;
          std::string nr;
          if (id < 0) {
            id = bpftime_amd_tracepoint_id(p.sys_nr, 1);
            if (id < 0) nr = "\"sys_nr\": " + std::to_string(p.sys_nr) + ", ";
          }
          a = "\"data_type\": \"tracepoint_perf_event_data\", \"pid\": " + std::to_string(p.pid) + ", " + nr +
              "\"tracepoint_id\": " + std::to_string(id) + ", ";
        } else if (p.type == 1) {
          a = "\"config\": " + std::to_string(p.config) + ", \"cpu\": " + std::to_string(p.cpu) +
              ", \"data_type\": \"software_perf_event_shared_ptr\", \"pid\": " + std::to_string(p.pid) +
              ", \"sample_type\": " + std::to_string(p.sample_type) + ", ";
        }
        item = "{\"attr\": {" + a + "\"type\": " + std::to_string(p.type) + "}, \"enabled\": " +
               (p.enabled ? "true" : "false") + ", \"type\": \"bpf_perf_event_handler\"}";
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

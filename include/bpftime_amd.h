/*
 * bpftime_amd runtime C ABI (libbpftime_amd.so): device-resident maps, the
 * prog / bpf_link records of the XDP attach surface, and device utilities.
 *
 * The map / prog / link entry points keep the names, argument meaning and
 * error conventions of the reference's shared-memory runtime
 * (runtime/include/bpftime_shm.hpp:220-400, implemented in
 * runtime/src/bpftime_shm.cpp:69-140 / bpftime_shm_internal.cpp), with the
 * map storage living in GPU HBM instead of a boost.interprocess segment.
 */
#ifndef BPFTIME_AMD_H
#define BPFTIME_AMD_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>
#include "ebpf-vm.h"

#ifdef __cplusplus
extern "C" {
#endif

/* runtime/include/bpftime_shm.hpp:27-46 (same field order, C layout) */
struct bpf_map_attr {
	int type;
	uint32_t key_size;
	uint32_t value_size;
	uint32_t max_ents;
	uint64_t flags;
	uint32_t ifindex;
	uint32_t btf_vmlinux_value_type_id;
	uint32_t btf_id;
	uint32_t btf_key_type_id;
	uint32_t btf_value_type_id;
	uint64_t map_extra;
	uint32_t kernel_bpf_map_id;
	uint64_t gpu_thread_count;
};

/* runtime/include/bpftime_shm.hpp:250-301 (BPF_LINK_CREATE args; 48 B) */
struct bpf_link_create_args {
	uint32_t prog_fd;        /* union { prog_fd; map_fd; } */
	uint32_t target_fd;      /* union { target_fd; target_ifindex; } */
	uint32_t attach_type;    /* BPF_XDP = 37 (runtime/include/bpftime_epoll.h:1158) */
	uint32_t flags;
	uint64_t attach_union[4];
};

#define BPFTIME_AMD_BPF_XDP 37
#define BPFTIME_AMD_BPF_PERF_EVENT 41      /* BPFTIME_BPF_PERF_EVENT_ATTACH_TYPE, bpftime_shm.hpp:247 */
#define BPFTIME_AMD_PROG_TYPE_XDP 6        /* bpftime_shm.hpp:144-151 */
#define BPFTIME_AMD_PROG_TYPE_TRACEPOINT 5

/* ---- maps: bpftime_shm.hpp:316-345 ---- */
/* create a map at `fd` (-1: lowest unused fd).  Supported types: HASH (1,
 * fix-size hash, map_handler.cpp:54-58), ARRAY (2), PROG_ARRAY (3, prog
 * fds, prog_array.cpp; the targets of bpf_tail_call, linked into the caller's
 * image at launch), PERCPU_HASH (5), PERCPU_ARRAY (6), LPM_TRIE (11),
 * RINGBUF (27).  Returns fd or -1 (errno set). */
int bpftime_maps_create(int fd, const char *name, struct bpf_map_attr attr);
/* syscall-side ops (from_syscall = true), bpftime_shm.cpp:115-140 */
const void *bpftime_map_lookup_elem(int fd, const void *key);
long bpftime_map_update_elem(int fd, const void *key, const void *value, uint64_t flags);
long bpftime_map_delete_elem(int fd, const void *key);
int bpftime_map_get_next_key(int fd, const void *key, void *next_key);
uint32_t bpftime_map_value_size_from_syscall(int fd);
int bpftime_is_map_fd(int fd);
int bpftime_is_array_map(int fd);
int bpftime_is_prog_fd(int fd);
int bpftime_find_minimal_unused_fd(void);
void bpftime_close(int fd);
/* bpftime_shm.cpp:287-306: a map's creation attributes and name; -1 +
 * ENOENT for a non-map fd */
int bpftime_map_get_info(int fd, struct bpf_map_attr *out_attr, const char **out_name, int *type);
/* bpftime_shm.cpp:347-353 (what the syscall server's mmap64 of an array map
 * fd returns, syscall_context.cpp:915-920): a host view of an ARRAY map's
 * bytes, page aligned, stable until the map is closed.  The device holds the
 * map: host writes to the view reach it before the next launch; the view
 * receives the device bytes when a synchronous batch (EBPF_BATCH_SYNC,
 * ebpf_exec) returns and on bpftime_amd_map_msync.  NULL + EINVAL for other
 * maps. */
void *bpftime_get_array_map_raw_data(int fd);
int bpftime_amd_map_msync(int fd); /* push host writes, wait for the device, pull; 0 / -1 */

/* ---- progs / links (bpftime_shm.hpp:303-309) ---- */
int bpftime_progs_create(int fd, const void *insns, size_t insn_cnt, const char *prog_name, int prog_type);
int bpftime_link_create(int fd, struct bpf_link_create_args *args);
/* ---- perf events (bpftime_shm.hpp:351-380; bpf_perf_event_handler,
 * runtime/src/handler/perf_event_handler.hpp:161-215) ----
 * The targets a link or BPF_PROG_ATTACH names.  A syscall sys_enter or
 * sys_exit tracepoint drives the replay dispatch (bpftime_amd_syscall_dispatch);
 * the other kinds (uprobes, software events) are kept as records so the
 * reference's state imports, exports and links unchanged.
 *
 * A syscall sys_enter tracepoint perf event by syscall number (what
 * perf_event_open of syscalls:sys_enter_<nr>, or raw_syscalls:sys_enter for
 * sys_nr = -1, creates): a new fd, or `fd` when >= 0. */
int bpftime_amd_perf_event_syscall(int fd, int64_t sys_nr);
/* bpftime_shm.hpp:368 (add_tracepoint): by tracepoint id; the id resolves to
 * (syscall number, enter / exit) when a program attaches
 * (bpftime_amd_tracepoint_resolve). */
int bpftime_tracepoint_create(int fd, int pid, int32_t tp_id);
/* bpftime_shm.hpp:356-357: a uprobe / uretprobe record. */
int bpftime_uprobe_create(int fd, int pid, const char *name, uint64_t offset, bool retprobe, size_t ref_ctr_off);
/* bpftime_shm.hpp:371-374: the handler's enabled flag. */
int bpftime_perf_event_enable(int fd);
int bpftime_perf_event_disable(int fd);
int bpftime_is_perf_event_fd(int fd);
/* Any perf event record, with every field the reference's JSON carries
 * (bpftime_shm_json.cpp:66-95, :130-180); get: the record at fd (module_name
 * points into the record). */
struct bpftime_amd_perf_event {
  int type;               /* bpf_event_type: 1 software, 2 tracepoint, 6 uprobe, 7 uretprobe, 1008 override */
  int pid;
  int enabled;
  int32_t tracepoint_id;  /* tracepoint: kernel id, or -1 with sys_nr */
  int64_t sys_nr;         /* tracepoint without an id: the syscall (-1: every syscall) */
  uint64_t offset;        /* uprobe kinds */
  uint64_t ref_ctr_off;
  const char *module_name;
  int cpu;                /* software */
  int32_t sample_type;
  int64_t config;
};
int bpftime_amd_perf_event_record(int fd, const struct bpftime_amd_perf_event *e);
int bpftime_amd_perf_event_get(int fd, struct bpftime_amd_perf_event *e);
/* bpftime_shm.cpp:249-253 (BPF_PROG_ATTACH): link prog bpf_fd to the perf
 * event: a link fd whose close detaches it; a program linked to a sys_enter
 * tracepoint then runs in bpftime_amd_syscall_dispatch.  -1 + ENOENT when
 * perf_fd is not a perf event or bpf_fd not a program, -1 + EEXIST when a
 * tracepoint id does not resolve, -1 when the device cannot load the
 * program. */
int bpftime_attach_perf_to_bpf(int perf_fd, int bpf_fd);
/* The same link at `fd` (-1: a fresh one), leaving a link to an unresolvable
 * tracepoint id as a record (the JSON import's add_bpf_link: the reference
 * resolves the id only when its agent attaches). */
int bpftime_amd_link_perf(int fd, int prog_fd, int perf_fd);
/* 1: the link drives a syscall attachment, 0: a record only, -1: not a link. */
int bpftime_amd_link_attached(int fd);

/* Syscall tracepoint ids (attach/syscall_trace_attach_impl/src/
 * syscall_table.cpp:17-98, syscall_trace_attach_private_data.cpp:8-63):
 * the tracefs events directory the ids are read from (default
 * /sys/kernel/tracing/events, or $BPFTIME_AMD_TRACEFS_EVENTS); an id ->
 * (syscall number, enter) with the reference's rules (raw_syscalls sys_enter
 * / sys_exit -> -1; sys_enter_<name> / sys_exit_<name> -> <name>'s number),
 * 0 or -EEXIST; the reverse (-1 when the directory has no such tracepoint);
 * a syscall's number by name (-1 unknown). */
int bpftime_amd_set_tracefs_events(const char *dir);
int bpftime_amd_tracepoint_resolve(int32_t tp_id, int64_t *sys_nr, int *is_enter);
int32_t bpftime_amd_tracepoint_id(int64_t sys_nr, int is_enter);
int64_t bpftime_amd_syscall_nr(const char *name);

/* ---- bpf(2) commands from an interposed loader ----
 * syscall_context::handle_sysbpf's userspace branch
 * (runtime/syscall-server/syscall_context.cpp:429-668): `attr` is the
 * kernel's union bpf_attr.  BPF_MAP_CREATE / BPF_PROG_LOAD / BPF_LINK_CREATE
 * return a new fd; lookups copy the value out (ENOENT when absent); update,
 * delete and get-next-key return the map operation's status; BPF_MAP_FREEZE
 * returns 0; other commands -1 with errno ENOTSUP. */
long bpftime_amd_handle_sysbpf(int cmd, void *attr, uint32_t size);

/* ---- lddw helpers for the device VM (bpftime_shm.cpp:637-676) ---- */
uint64_t bpftime_amd_map_ptr_by_fd(uint32_t fd); /* the fd itself, ~0 if not a map */
uint64_t bpftime_amd_map_val(uint64_t map_ptr);  /* DEVICE address of the first value */

/* ---- bpftime_amd extensions ---- */
/* device address / byte size of a map's storage (layout: csrc/common.hpp DMap) */
uint64_t bpftime_amd_map_device_ptr(int fd, uint64_t *bytes);
/* raw device-layout copy of the map storage to / from the host */
int bpftime_amd_map_snapshot(int fd, void *out, uint64_t bytes);
int bpftime_amd_map_restore(int fd, const void *in, uint64_t bytes);
/* hash maps: bucket count and device slot geometry */
int bpftime_amd_map_geometry(int fd, uint64_t *nbuckets, uint32_t *slot_size, uint32_t *key_off,
                             uint32_t *val_off, uint32_t *ncpu);
uint64_t bpftime_amd_map_count(int fd);
/* An LPM trie whose device update (ORDERED batch) ran out of the node pool
 * keeps the state from before that batch and reports ENOMEM on every host op
 * and every launch of a program naming a trie until this acknowledges it:
 * 1 when a report was cleared, 0 when there was none, -1 not a map. */
int bpftime_amd_map_ack_error(int fd);
/* virtual CPU count for per-CPU maps and helper 8 (default 64) */
void bpftime_amd_set_ncpu(uint32_t ncpu);
uint32_t bpftime_amd_get_ncpu(void);
/* drop every map / prog / link record and free the device arena */
void bpftime_amd_reset(void);

/* XDP attach surface: enumerate BPF_XDP links -> (link fd, prog fd, ifindex) */
int bpftime_amd_xdp_links(int *link_fds, int *prog_fds, uint32_t *ifindexes, int max);
/* instantiate a prog record into a loaded "mi355x" VM with the default
 * helper groups registered (bpf_attach_ctx.cpp:40-57 equivalent). */
struct ebpf_vm *bpftime_amd_prog_instantiate(int prog_fd, char **errmsg);
/* registers the device helper set (ids 1,2,3,5,7,8,28,44,65,130-133) on a VM */
int bpftime_amd_register_default_helpers(struct ebpf_vm *vm);
/* loader facts: per-lane stack bytes, big (scratch) stack, fused RMW count */
int bpftime_amd_vm_info(const struct ebpf_vm *vm, uint32_t *stack_size, int *big_stack,
                        uint32_t *fused_rmw, uint32_t *n_insns);
void bpftime_amd_set_step_limit(struct ebpf_vm *vm, uint64_t limit);
/* Kernel time (ms) of the vm's last EBPF_BATCH_TIMED batch, waiting for it; -1 when none. */
float bpftime_amd_last_batch_ms(struct ebpf_vm *vm);
/* loads/stores (and array-lookup keys) the loader typed statically for the
 * fast path under the given ctx kind (packet, slot, ctx or stack bases) */
int bpftime_amd_vm_fast_info(const struct ebpf_vm *vm, uint32_t ctx_kind, uint32_t *specialized);
/* Counter adds of the loaded program for one entry form: `deferred` may be
 * summed per wave / block before they reach memory (nothing the unit runs
 * afterwards can observe them), `direct` reach memory at once. */
int bpftime_amd_vm_counter_info(const struct ebpf_vm *vm, uint32_t ctx_kind, uint32_t *deferred, uint32_t *direct);

/* ---- handler JSON (csrc/shm_json.cpp) ----
 * The reference's shm export / import format (runtime/include/bpftime_shm.hpp:
 * 237-241, runtime/src/bpftime_shm_json.cpp:103-327): {"<fd>": {"type":
 * "bpf_map_handler" | "bpf_prog_handler" | "bpf_link_handler", "name", "attr"}}.
 * Import recreates maps (in HBM), programs and links at the same fds; a link
 * to an XDP program becomes a BPF_XDP link (the format drops attach types).
 * 0 / -1 (errno, bpftime_amd_last_error). */
int bpftime_import_global_shm_from_json(const char *filename);
int bpftime_export_global_shm_to_json(const char *filename);
int bpftime_import_shm_handler_from_json(int fd, const char *json_string);

/* ---- eBPF ELF objects (csrc/object.cpp) ----
 * The reference opens objects with libbpf (runtime/object/bpftime_object.hpp:
 * bpftime_object_open / _close / _find_program_by_name / _by_secname,
 * bpf_object.cpp:149-260) and relies on libbpf's bpf_object__load for map
 * creation, map / global-data relocation and CO-RE before BPF_PROG_LOAD
 * reaches its syscall server.  These entry points do both: open parses the
 * object (programs, BTF / legacy maps, .bss/.data/.rodata, .rel sections,
 * .BTF.ext CO-RE field relocations against the target BTF); load creates the
 * maps and prog records (bpftime_maps_create / bpftime_progs_create) so the
 * programs run through bpftime_amd_prog_instantiate / bpftime_link_create.
 * Programs are addressed by prog fd (the reference returns bpftime_prog *). */
struct bpftime_object;
/* NULL only if the file cannot be read; parse errors: bpftime_object_error()
 * non-empty and every other call fails */
struct bpftime_object *bpftime_object_open(const char *obj_path);
struct bpftime_object *bpftime_object_open_mem(const void *buf, size_t len, const char *obj_name);
const char *bpftime_object_error(const struct bpftime_object *obj);
/* target BTF for CO-RE (libbpf's btf_custom_path, e.g. the xdp-counter
 * example's base.btf); default: the runtime's own xdp_md layout */
int bpftime_object_load_relocate_btf(struct bpftime_object *obj, const char *btf_path);
int bpftime_object_load_relocate_btf_mem(struct bpftime_object *obj, const void *btf, size_t len);
int bpftime_object_map_count(const struct bpftime_object *obj);
int bpftime_object_map_info(const struct bpftime_object *obj, int idx, const char **name,
                            struct bpf_map_attr *attr);
int bpftime_object_program_count(const struct bpftime_object *obj);
int bpftime_object_program_info(const struct bpftime_object *obj, int idx, const char **name,
                                const char **secname, int *prog_type, size_t *insn_cnt);
/* the relocated instructions of program idx for the given map fds (one per
 * object map, map_info order); returns the instruction count or -1 */
int bpftime_object_program_insns(const struct bpftime_object *obj, int idx, const int *map_fds, void *out,
                                 size_t insn_cap);
/* create the maps (initialised from .data/.rodata) and prog records; 0 / -1 */
int bpftime_object_load(struct bpftime_object *obj);
int bpftime_object_find_program_by_name(const struct bpftime_object *obj, const char *name);      /* prog fd */
int bpftime_object_find_program_by_secname(const struct bpftime_object *obj, const char *secname); /* prog fd */
int bpftime_object_find_map_fd_by_name(const struct bpftime_object *obj, const char *name);
const char *bpftime_object_license(const struct bpftime_object *obj);
void bpftime_object_close(struct bpftime_object *obj);

/* ring buffer consumer (ringbuf::fetch_data, ringbuf_map.cpp): committed
 * records from the consumer position on, each written to `out` as
 * [u32 len][len bytes]; advances the consumer position; returns the record
 * count (-1: not a ring buffer).  Waits for queued batches first. */
int64_t bpftime_amd_ringbuf_fetch(int fd, void *out, uint64_t cap, uint64_t *used);

/* ---- syscall tracepoint dispatch (csrc/syscall_dispatch.cpp) ----
 * syscall_trace_attach_impl.cpp:18-95 over recorded syscalls in device memory.
 *
 * attach (create_attach_with_ebpf_callback, :121-166): a program on the
 * sys_enter (is_enter = 1) or sys_exit (0) tracepoint of `sys_nr` in
 * [0, 512), or of every syscall (-1); an attach id, or -1 with errno EINVAL
 * (not a program, sys_nr out of range) or the load error.
 * bpftime_amd_syscall_attach(prog, nr) = bpftime_amd_syscall_attach_ex(prog, nr, 1).
 *
 * Replay records: BPFTIME_AMD_SYSCALL_RECORD (64 B) = trace_event_raw_sys_enter
 * {ent = 0, id, args[6]}; BPFTIME_AMD_SYSCALL_RECORD_FULL (96 B) = that, then
 * trace_event_raw_sys_exit {ent = 0, id, ret} (24 B) at +64, then the
 * calling thread's u64 pid_tgid (tgid << 32 | tid) at +88: the enter ctx and
 * the exit ctx as dispatch_syscall builds them (:57-66, :80-85), each the unit
 * its programs run on in place, and what bpf_get_current_pid_tgid returns to
 * them (bpf_helper.cpp:330-348; 64-B records: the dispatching thread's);
 * BPFTIME_AMD_SYSCALL_RECORD_TIMED (128 B) = the 96-B record, then the
 * recorded clock at sys_enter (u64 ns at +96) and after the call (+104), 16
 * zero bytes: what bpf_ktime_get_ns (bpf_helper.cpp:357-362) returns inside
 * the record's enter / exit callbacks (the replay definition of the clock;
 * other records: the device clock).  Per record
 * (dispatch_syscall :18-95): exit (60) / exit_group (231) run nothing and
 * return ret; the per-syscall enter programs, then the global ones; if one of
 * them called bpf_override_return / bpf_set_retval the record returns that
 * value and its exit programs do not run; else the per-syscall exit programs,
 * then the global ones, and the record returns ret, or the value an exit
 * program set.  Ids outside [0, 512) (the reference indexes its callback
 * arrays with them, undefined there) run only global programs.
 *
 * Order.  The reference runs a call's callbacks on the calling thread, one
 * call after another; threads run side by side.  Two plans give that result:
 *  - program-major (BPFTIME_AMD_DISPATCH_PROGRAMS): each program runs once
 *    over the batch, one lane per record, in the order above; a program that
 *    may store into its ctx runs on a copy of the records, as each reference
 *    callback runs on its own copy (:43-45).  Equal to the per-call order
 *    whenever the attached programs' map effects commute;
 *  - thread-ordered (BPFTIME_AMD_DISPATCH_THREADS): records are grouped by
 *    their recorded pid_tgid (64-B records: one thread, the dispatcher), one
 *    lane per thread walks its records in record order and runs each
 *    record's enter callbacks, the override check and its exit callbacks
 *    before the next record, every callback on a fresh ctx copy: the
 *    reference's own schedule for any programs, threads in parallel.
 * By default the dispatch picks thread-ordered when two attachments may not
 * commute (one writes a map the other reads or writes, or adds to a map the
 * other reads: the loader's map effects, loader.hpp FastForm::map_fx), else
 * program-major.  EBPF_BATCH_ORDERED runs thread-ordered on one lane over
 * every record in record order (the serial reference run).  Thread-ordered
 * dispatch does not run bpf_tail_call (the dispatch fails, named).
 * bpftime_amd_syscall_dispatch_plan(flags) says which plan a dispatch with
 * these flags would take for the current attachments: 1 thread-ordered, 0
 * program-major, -1 on errors.
 *
 * dispatch_records: `out_rets` (device i64 per record, nullable) receives the
 * value dispatch_syscall would return (64-B records have no ret: 0 unless
 * overridden).  64-B records with sys_exit programs attached are refused
 * (EINVAL).  Returns the failed-unit count summed over the programs (a
 * failed callback counts once) with EBPF_BATCH_SYNC, else 0; -1 on errors
 * (bpftime_amd_last_error).  Concurrent dispatches on one stream run one
 * after the other (the dispatch holds the stream's scratch until it has
 * queued its last launch).
 * bpftime_amd_syscall_dispatch(r, n, f, s) = dispatch_records(r, n, 64, NULL, f, s). */
#define BPFTIME_AMD_SYSCALL_RECORD 64
#define BPFTIME_AMD_SYSCALL_RECORD_FULL 96
#define BPFTIME_AMD_SYSCALL_RECORD_TIMED 128
#define BPFTIME_AMD_DISPATCH_THREADS 0x100  /* force the thread-ordered plan */
#define BPFTIME_AMD_DISPATCH_PROGRAMS 0x200 /* force the program-major plan */
int bpftime_amd_syscall_attach(int prog_fd, int64_t sys_nr);   /* attach id or -1 */
int bpftime_amd_syscall_attach_ex(int prog_fd, int64_t sys_nr, int is_enter);
int bpftime_amd_syscall_detach(int id);
int64_t bpftime_amd_syscall_dispatch(const void *records, uint64_t n, uint32_t flags, void *stream);
int64_t bpftime_amd_syscall_dispatch_records(const void *records, uint64_t n, uint32_t record_size,
                                             int64_t *out_rets, uint32_t flags, void *stream);
int bpftime_amd_syscall_dispatch_plan(uint32_t flags);
/* Struct-of-arrays replay records: the same calls as the AoS forms, each
 * field in its own device array, so a dispatch streams only what its
 * programs read (an exit-only dispatch: 32 B per call instead of a 96-B
 * record's three 128-B cache lines' worth).
 *   enter: count x 64 B trace_event_raw_sys_enter {ent = 0, id, args} (NULL
 *          when no sys_enter program is attached: the id comes from exit);
 *   exit:  count x 32 B {trace_event_raw_sys_exit {ent = 0, id, ret} (24 B),
 *          the caller's u64 pid_tgid};
 *   clock: count x 16 B {u64 ns at sys_enter, u64 ns after the call} (the
 *          replayed bpf_ktime_get_ns), or NULL (the device clock).
 * The dispatch runs as bpftime_amd_syscall_dispatch_records over the
 * equivalent 96- / 128-B records (same plans, results and errors). */
struct bpftime_amd_sys_records {
  const void *enter;
  const void *exit;
  const void *clock;
  uint64_t count;
};
int64_t bpftime_amd_syscall_dispatch_soa(const struct bpftime_amd_sys_records *records, int64_t *out_rets,
                                         uint32_t flags, void *stream);

/* ---- attach plugins (attach/base_attach_impl/base_attach_impl.hpp:24-71,
 * attach/simple_attach_impl/simple_attach_impl.cpp:7-55; csrc/attach.cpp) ----
 * An attach entry is a program loaded on the device.  bpftime_amd_attach_run
 * has the shape of ebpf_run_callback, int(void *memory, size_t memory_size,
 * uint64_t *return_value), with the entry as a leading context argument, so a
 * base_attach_impl can bind it as its callback: one unit,
 * bpftime_prog_exec's contract.  bpftime_amd_attach_run_batch runs the entry
 * over a device batch (ebpf_exec_batch's contract). */
struct bpftime_amd_attach;
struct bpftime_amd_attach *bpftime_amd_attach_create(int prog_fd, int ctx_kind); /* ctx_kind -1: from the prog type */
int bpftime_amd_attach_run(void *attach, void *memory, size_t memory_size, uint64_t *return_value);
int bpftime_amd_attach_run_batch(struct bpftime_amd_attach *attach, const struct ebpf_batch *batch);
void bpftime_amd_attach_destroy(struct bpftime_amd_attach *attach);
/* simple_attach_impl over device batches: create an impl for one attach
 * type with a callback; attach one program (a second attach, or a mismatched
 * type, fails: -1); trigger calls cb(attach-time argument, trigger argument,
 * the attach entry) and returns its result, or 1 when nothing is attached;
 * detach by the id attach returned. */
typedef int (*bpftime_amd_simple_callback)(const char *argument, void *trigger_argument,
                                           struct bpftime_amd_attach *attach);
int bpftime_amd_simple_attach_impl_create(int attach_type, bpftime_amd_simple_callback cb);
int bpftime_amd_simple_attach(int impl, int prog_fd, int ctx_kind, const char *argument, int attach_type);
int bpftime_amd_simple_detach(int impl, int id);
int bpftime_amd_simple_trigger(int impl, void *trigger_argument);
int bpftime_amd_simple_attach_impl_destroy(int impl);

/* ---- host merge of per-GPU map shards ---- */
/* acc += shard - init over u64 words (array counters, additive rule) */
int bpftime_amd_merge_delta_u64(void *acc, const void *init, const void *shard, uint64_t bytes);
/* The same rule counter by counter at `width` bytes (1, 2, 4, 8): a u32
 * counter's combined delta wraps at 2^32 instead of carrying into the next
 * field.  -1 when bytes is not a multiple of width. */
int bpftime_amd_merge_delta(void *acc, const void *init, const void *shard, uint64_t bytes, uint32_t width);

/* ---- device utilities (HIP runtime plumbing for callers without one) ---- */
int bpftime_amd_device_count(void);
int bpftime_amd_hip_runtime_version(void);  /* hipRuntimeGetVersion of the runtime this library runs on, -1 on error */
/* Experiment counters (BPFTIME_AMD_DBG=512: hash lookup-cache hit lanes, miss lanes): up to n
 * u64 into out after the device is idle, zeroed when reset; the count or -1. */
int bpftime_amd_dbg_counters(uint64_t *out, int n, int reset);
int bpftime_amd_set_device(int dev);
void *bpftime_amd_dev_alloc(uint64_t bytes);
void bpftime_amd_dev_free(void *p);
int bpftime_amd_memcpy_htod(void *dst, const void *src, uint64_t bytes);
int bpftime_amd_memcpy_dtoh(void *dst, const void *src, uint64_t bytes);
/* async copies on a stream (host side must be pinned for overlap) */
int bpftime_amd_memcpy_htod_async(void *dst, const void *src, uint64_t bytes, void *stream);
int bpftime_amd_memcpy_dtoh_async(void *dst, const void *src, uint64_t bytes, void *stream);
void *bpftime_amd_stream_create(void); /* non-blocking hipStream_t */
void bpftime_amd_stream_destroy(void *stream);
int bpftime_amd_stream_sync(void *stream);
int bpftime_amd_memset(void *dst, int v, uint64_t bytes);
int bpftime_amd_sync(void);
void *bpftime_amd_host_alloc(uint64_t bytes); /* pinned */
void bpftime_amd_host_free(void *p);
/* events on a stream: returns elapsed ms between start/stop records */
void *bpftime_amd_event_create(void);
void bpftime_amd_event_destroy(void *ev);
int bpftime_amd_event_record(void *ev, void *stream);
/* work queued on `stream` after this waits for the event's last record */
int bpftime_amd_stream_wait_event(void *stream, void *ev);
float bpftime_amd_event_elapsed_ms(void *start, void *stop);
const char *bpftime_amd_last_error(void);

/* ---- synthetic inputs (seeded splitmix64) ---- */
/* word k of the stream = splitmix64 output #k for `seed`:
 *   z = seed + (k+1)*0x9E3779B97F4A7C15; z = (z^(z>>30))*0xBF58476D1CE4E5B9;
 *   z = (z^(z>>27))*0x94D049BB133111EB; z ^= z>>31 */
/* n packets in `stride`-byte device slots (first `len` bytes random, bytes
 * 12..13 = 0x08 0x00); unit i uses words of stream index first+i. */
int bpftime_amd_gen_xdp(void *dev, uint64_t n, uint64_t stride, uint32_t len, uint64_t seed,
                        uint64_t first, void *stream);
/* config 3 frames (gen.py flow_packets): `cdf` = device copy of the Zipf
 * CDF (nflows doubles, computed on the host); per-unit lengths to `lens`. */
int bpftime_amd_gen_flow(void *dev, uint32_t *lens, uint64_t n, uint64_t stride, uint64_t seed,
                         uint64_t first, const double *cdf, uint32_t nflows, void *stream);
/* config 5 records (gen.py syscall_records), 64 B each. */
int bpftime_amd_gen_syscall(void *dev, uint64_t n, uint64_t seed, uint64_t first, const double *cdf,
                            uint32_t support, void *stream);
/* 96-B replay records (gen.py syscall_records_full): config 5's enter record
 * (id -1 for 0.5 %), then the exit ctx {0, id, ret}, then a pid_tgid. */
int bpftime_amd_gen_syscall_full(void *dev, uint64_t n, uint64_t seed, uint64_t first, const double *cdf,
                                 uint32_t support, void *stream);
/* The same calls as struct-of-arrays records (bpftime_amd_syscall_dispatch_soa):
 * enter (n x 64 B, may be NULL) and exit (n x 32 B {exit ctx, pid_tgid}). */
int bpftime_amd_gen_syscall_soa(void *enter, void *exit, uint64_t n, uint64_t seed, uint64_t first,
                                const double *cdf, uint32_t support, void *stream);
/* Static LDS bytes of the interpreter kernel for a launch shape (its
 * attribute; the restated sum without a device): with the dynamic part
 * (common.hpp dyn_lds_for) what a block needs of the CU's 160 KiB. */
size_t bpftime_amd_static_lds(uint32_t kind, bool big_stack, bool gregs, uint32_t block);
/* Dynamic + static LDS bytes of an interpreter block (ctx kind, 512-B scratch
 * stack, per-lane stack bytes, combining-table entries, lookup-cache sets,
 * ctx in LDS, register copy in global memory, lanes): a launch whose block
 * needs more than 160 KiB fails with a named error (vm_api.cpp). */
size_t bpftime_amd_lds_bytes(uint32_t kind, bool big_stack, uint32_t stack_size, uint32_t comb_entries,
                             uint32_t lcache_sets, bool ctx_lds, bool gregs, uint32_t block);

#ifdef __cplusplus
}
#endif
#endif

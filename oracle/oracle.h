/*
 * bpftime_amd CPU ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference's CPU path for the per-packet eBPF
 * hot path: the ubpf interpreter semantics bpftime calls
 * through vm/compat/ubpf-vm/compat_ubpf.cpp:207-210, the load-time patching of
 * compat_ubpf.cpp:50-200, bpftime's userspace map implementations and the
 * map/XDP helpers of runtime/src/bpf_helper.cpp.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / the timed CPU baseline.  The product
 * path (bpftime_amd/, libbpftime_amd.so) never links or calls it.
 *
 * Parity status: the interpreter arithmetic lives in iovisor/ubpf, an
 * un-vendored empty submodule (.gitmodules:16-18, pinned commit unknown), and
 * no executing reference test covers it -> the interpreter is "parity
 * unpinned" except for the analytic KATs (vm/example/bpf_progs.h,
 * .github/assets/sum.bpf.o semantics).  Map semantics are pinned by ports of
 * runtime/unit-test/maps/ (test_*.cpp) assertions (tests/test_oracle_maps.py).
 */
#ifndef BPFTIME_AMD_ORACLE_H
#define BPFTIME_AMD_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_MAX_INSTS 65536 /* vm/vm-core/include/ebpf-vm.h:33-35 */
#define ORC_STACK_SIZE 512  /* ebpf-vm.h:47-49 */
#define ORC_MAX_HELPERS 64  /* ubpf limit, vm/compat/ubpf-vm/README.md:4 */
#define ORC_MAX_FDS 1024

typedef uint64_t (*orc_helper_fn)(uint64_t, uint64_t, uint64_t, uint64_t, uint64_t);

struct orc_vm;

/* ---- VM (restates ebpf-vm.h C ABI over the ubpf backend) ---------------- */
struct orc_vm *orc_vm_create(void);
void orc_vm_destroy(struct orc_vm *vm);
int orc_vm_register(struct orc_vm *vm, unsigned index, const char *name, orc_helper_fn fn);
/* registers bpftime helper ids 1,2,3,5,7,8,28,44,65 (bpf_helper.cpp:1177-1401) */
int orc_vm_register_default_helpers(struct orc_vm *vm);
/* bpf_xdp_load_bytes (id 189): defined in bpf_helper.cpp:778-788 but not in
 * any default helper group; an embedder registers it explicitly. */
int orc_vm_register_xdp_load_bytes(struct orc_vm *vm);
/* helpers 6 (trace_printk, text to a log) and 14 (get_current_pid_tgid) */
int orc_vm_register_trace_helpers(struct orc_vm *vm);
size_t orc_trace_log(char *out, size_t cap);  /* bytes logged; copies up to cap */
void orc_trace_log_reset(void);
void orc_set_pid_tgid(uint64_t v);
void orc_vm_set_unwind_index(struct orc_vm *vm, int idx);
/* ebpf_load: 0 / <0, errbuf receives the message (compat_ubpf.cpp:61-200) */
int orc_vm_load(struct orc_vm *vm, const void *code, uint32_t code_len, char *errbuf, size_t errlen);
void orc_vm_unload(struct orc_vm *vm);
/* ebpf_exec: 0 / -1 (ubpf_exec) */
int orc_vm_exec(struct orc_vm *vm, void *mem, size_t mem_len, uint64_t *ret);
/* instructions executed by the last orc_vm_exec / accumulated by drivers */
uint64_t orc_vm_insn_count(struct orc_vm *vm);
void orc_vm_reset_insn_count(struct orc_vm *vm);

/* ---- maps (runtime/src/bpf_map/userspace, map_handler.cpp) ---------- */
void orc_maps_reset(void);
/* creates a map at `fd` (-1 = next free); returns fd or -1 */
/* ring buffer (ringbuf_map.cpp): reserve / submit as the helpers use them,
 * fetch = the consumer (ringbuf::fetch_data) */
void *orc_ringbuf_reserve(int fd, uint64_t size);
void orc_ringbuf_submit_fd(int fd, const void *sample, int discard);
int64_t orc_ringbuf_fetch(int fd, uint8_t *out, uint64_t cap, uint64_t *used);
int orc_map_create(int fd, uint32_t type, uint32_t key_size, uint32_t value_size,
                   uint32_t max_entries, uint32_t flags);
void orc_set_ncpu(int ncpu); /* per-CPU slot count (reference: sysconf(_SC_NPROCESSORS_ONLN)) */
void orc_set_cpu(int cpu);   /* current "sched_getcpu()" for per-CPU maps and helper 8 */
/* helper-side ops (from_syscall = false) */
void *orc_map_lookup(int fd, const void *key);
long orc_map_update(int fd, const void *key, const void *value, uint64_t flags);
long orc_map_delete(int fd, const void *key);
/* syscall-side ops (from_syscall = true): per-CPU maps use ncpu*value views */
void *orc_map_lookup_user(int fd, const void *key);
long orc_map_update_user(int fd, const void *key, const void *value, uint64_t flags);
long orc_map_delete_user(int fd, const void *key);
int orc_map_get_next_key(int fd, const void *key, void *next_key);
int orc_last_errno(void);
uint32_t orc_map_value_size_user(int fd);
/* raw storage views for bulk comparison */
void *orc_map_raw(int fd, size_t *bytes);
/* hash maps: bucket count (= next_prime(max_entries)), element count */
uint64_t orc_map_buckets(int fd);
uint64_t orc_map_count(int fd);
/* programs for bpf_tail_call (bpftime_progs_create records; bpf_helper.cpp:568-650):
 * the target runs as a nested exec over a 64-B copy of the ctx, depth <= 32 */
int orc_prog_create(int fd, const void *insns, uint32_t insn_cnt);
void orc_prog_close(int fd);
int orc_is_prog_fd(int fd);
int orc_map_is_prog_array(int fd);
/* lddw helpers (runtime/src/bpftime_shm.cpp:637-676) */
uint64_t orc_map_ptr_by_fd(uint32_t fd);
uint64_t orc_map_val(uint64_t map_ptr);
uint64_t orc_next_prime(uint64_t n);
uint64_t orc_hash_bytes(const void *key, uint64_t n);

/* ---- drivers ---------------------------------------------------------- */
/* XDP: per packet an xdp_md_userspace (runtime/extension/userspace_xdp.h:6-17)
 * with data = base + i*stride, data_end = data + len, buffer_[start,end) =
 * the slot; verdicts[i] = (u32) r0 (0 on exec error, bpftime_prog.cpp:237-257).
 * lens == NULL -> fixed_len for every packet. out_data_off / out_len (nullable)
 * receive data-slot and data_end-data after the program (adjust_head/tail).
 * head: data starts `head` bytes into the slot (headroom for adjust_head). */
int orc_run_xdp(struct orc_vm *vm, uint8_t *base, uint64_t n, uint64_t stride,
                const uint32_t *lens, uint32_t fixed_len, uint32_t *verdicts,
                int32_t *out_data_off, uint32_t *out_len, uint32_t ifindex, uint32_t rxq,
                uint32_t head);
/* raw: r1 = base + i*stride, r2 = len; rets[i] = r0 */
int orc_run_raw(struct orc_vm *vm, uint8_t *base, uint64_t n, uint64_t stride, uint32_t len,
                uint64_t *rets);
/* syscall-enter replay (syscall_trace_attach_impl.cpp:18-67): records are
 * 64-B trace_event_raw_sys_enter; exit(60)/exit_group(231) skipped (ran=0),
 * ctx is a zeroed copy with id/args filled. */
int orc_run_syscall(struct orc_vm *vm, const uint8_t *recs, uint64_t n, uint64_t *rets,
                    uint8_t *ran);
/* Syscall dispatch (syscall_trace_attach_impl.cpp:18-166).  attach: a VM on
 * the sys_enter (is_enter 1) or sys_exit (0) tracepoint of sys_nr in
 * [0, 512) or of every syscall (-1): an id > 0, or -EINVAL.  dispatch: per
 * record, in record order, dispatch_syscall with the recorded call: records
 * of rec_size 64 (trace_event_raw_sys_enter), 96 (that, then
 * trace_event_raw_sys_exit {0, id, ret} at +64, the caller's pid_tgid at +88)
 * or 128 (that, then the recorded enter and exit clocks at +96 / +104);
 * out[i] = what dispatch_syscall returns (ret, 0 for 64-B records, or an
 * override).  A callback's failed exec is ignored (:47-52).
 * bpf_get_current_pid_tgid returns a 96- / 128-B record's u64 at +88 (its
 * recorded caller); bpf_ktime_get_ns inside a 128-B record's enter callbacks
 * its u64 at +96, inside its exit callbacks the u64 at +104 (the replay
 * definition of the clock).  Ids outside [0, 512) have no per-syscall
 * callbacks here (the reference indexes its arrays with them). */
int orc_sys_attach(struct orc_vm *vm, int64_t sys_nr, int is_enter);
int orc_sys_detach(int id);
void orc_sys_reset(void);
int orc_sys_dispatch(const uint8_t *recs, uint64_t n, uint32_t rec_size, int64_t *out);
/* the thread's return callback (base_attach_impl.hpp:18-19), internal */
struct orc_retval_cb {
	int active, overridden;
	int64_t value;
};
extern struct orc_retval_cb orc_retval;
extern int orc_helper_abort;
/* bpf_get_current_pid_tgid of a replayed call (96-B records: the u64 at +88) */
void orc_pid_tgid_recorded(int on, uint64_t v);
/* bpf_ktime_get_ns of a replayed call (128-B records: the recorded clock) */
void orc_ktime_recorded(int on, uint64_t v);
/* timed XDP loop (steady clock around the packet loop only, like
 * tools/bpftimetool/main.cpp:42-58); returns seconds, pins to `cpu` if >=0 */
double orc_time_xdp(struct orc_vm *vm, uint8_t *base, uint64_t n, uint64_t stride,
                    uint32_t fixed_len, uint32_t *verdicts, int pin_cpu);

#ifdef __cplusplus
}
#endif
#endif

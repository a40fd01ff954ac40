/*
 * bpftime_amd drop-in VM C ABI (libbpftime_amd.so).
 *
 * Exports exactly the symbols of the reference's VM C ABI,
 * vm/vm-core/include/ebpf-vm.h:59-236 (implemented there by
 * vm/vm-core/src/ebpf-vm.cpp:6-98 over the bpftime_vm_impl plugin interface,
 * vm/compat/include/bpftime_vm_compat.hpp:27-263), backed by a gfx950 HIP
 * interpreter registered under the VM name "mi355x".  One additive entry
 * point, ebpf_exec_batch(), runs the loaded program over a device-resident
 * batch of packets / records.
 */
#ifndef BPFTIME_AMD_EBPF_VM_H
#define BPFTIME_AMD_EBPF_VM_H

#ifdef __cplusplus
extern "C" {
#endif

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

/* limits: vm/vm-core/include/ebpf-vm.h:33-49 */
#ifndef EBPF_MAX_INSTS
#define EBPF_MAX_INSTS 65536
#endif
#ifndef MAX_EXT_FUNCS
#define MAX_EXT_FUNCS 8192
#endif
#ifndef EBPF_STACK_SIZE
#define EBPF_STACK_SIZE 512
#endif

struct ebpf_vm;
typedef uint64_t (*ebpf_jit_fn)(void *mem, size_t mem_len);

/* ebpf-vm.h:67 / ebpf-vm.cpp:6-11.  Known names: "mi355x".  Unknown or empty
 * names return NULL (the reference throws a C++ exception,
 * bpftime_vm_compat.hpp:228-244). */
struct ebpf_vm *ebpf_create(const char *vm_name);
/* ebpf-vm.h:74 */
void ebpf_destroy(struct ebpf_vm *vm);
/* ebpf-vm.h:82; like the reference the name field is never set -> "" */
const char *ebpf_get_vm_name(struct ebpf_vm *vm);
/* ebpf-vm.h:92.  The device interpreter always confines global accesses to
 * the batch and the map arena; this flag toggles the stricter per-ubpf check
 * only in its reported value (returns previous value). */
bool ebpf_toggle_bounds_check(struct ebpf_vm *vm, bool enable);
/* ebpf-vm.h:100 */
void ebpf_set_error_print(struct ebpf_vm *vm, int (*error_printf)(FILE *stream, const char *format, ...));
/* ebpf-vm.h:117.  `index` is the bpftime helper id (BPF_FUNC_*); the host
 * function pointer is recorded for ABI compatibility, the device runs its own
 * implementation of ids 1,2,3 (map lookup / update / delete), 5 (ktime_get_ns),
 * 7 (get_prandom_u32), 8 (get_smp_processor_id), 12 (tail_call), 14
 * (get_current_pid_tgid), 28 (csum_diff), 44 (xdp_adjust_head), 58
 * (override_return), 65 (xdp_adjust_tail), 130-133 (ringbuf output / reserve /
 * submit / discard), 187 (set_retval) and 189 (xdp_load_bytes)
 * (loader.cpp device_helper_supported).  0 / -1. */
int ebpf_register(struct ebpf_vm *vm, unsigned int index, const char *name, void *fn);
/* ebpf-vm.h:137: copy, patch (compat_ubpf.cpp:61-200), validate, pre-decode
 * and upload.  0 / <0 with *errmsg strdup'd (caller frees). */
int ebpf_load(struct ebpf_vm *vm, const void *code, uint32_t code_len, char **errmsg);
/* ebpf-vm.h:148 */
void ebpf_unload_code(struct ebpf_vm *vm);
/* ebpf-vm.h:166: runs one unit on the GPU (mem copied in and back).  The
 * ctx kind (ebpf_set_ctx_kind) decides how `mem` is interpreted. 0 / -1. */
int ebpf_exec(const struct ebpf_vm *vm, void *mem, size_t mem_len, uint64_t *bpf_return_value);
/* ebpf-vm.h:180: the mi355x backend is an interpreter; returns NULL and sets
 * *errmsg (like an unsupported backend). */
ebpf_jit_fn ebpf_compile(struct ebpf_vm *vm, char **errmsg);
/* ebpf-vm.h:193 */
int ebpf_set_unwind_function_index(struct ebpf_vm *vm, unsigned int idx);
/* ebpf-vm.h:203 */
int ebpf_set_pointer_secret(struct ebpf_vm *vm, uint64_t secret);
/* ebpf-vm.h:222.  NULL helpers select the built-in device map registry
 * (bpftime_amd_map_ptr_by_fd / bpftime_amd_map_val). */
void ebpf_set_lddw_helpers(struct ebpf_vm *vm, uint64_t (*map_by_fd)(uint32_t),
                           uint64_t (*map_by_idx)(uint32_t), uint64_t (*map_val)(uint64_t),
                           uint64_t (*var_addr)(uint32_t), uint64_t (*code_addr)(uint32_t));
/* ebpf-vm.h:236: no AOT objects for the device interpreter -> NULL */
ebpf_jit_fn ebpf_load_aot_object(struct ebpf_vm *vm, const void *buf, size_t buf_len);

/* ---- additive batch API (SURVEY.md §8b "Additive batch entry point") ---- */
#define EBPF_CTX_RAW 0     /* r1 = unit memory, r2 = length */
#define EBPF_CTX_XDP 1     /* r1 = struct xdp_md_userspace (runtime/extension/userspace_xdp.h:6-17) */
#define EBPF_CTX_SYSCALL 2 /* r1 = 64-B trace_event_raw_sys_enter; nr 60/231 skipped */
/* r1 = 24-B trace_event_raw_sys_exit {ent = 0, id, ret} (syscall_trace_attach_impl.hpp:31-36,
 * built at syscall_trace_attach_impl.cpp:80-85), r2 = 24; nr 60/231 skipped.  The unit is the
 * exit half of a 96-B replay record (data = records + 64, stride 96), a 32-B
 * struct-of-arrays exit record {ctx, pid_tgid} (stride 32), or any record with that
 * layout at `stride`. */
#define EBPF_CTX_SYSCALL_EXIT 3

#define EBPF_BATCH_SYNC 0x1    /* wait for completion; return the failed-unit count */
#define EBPF_BATCH_ORDERED 0x2 /* one lane, units in index order (exact sequential semantics) */
#define EBPF_BATCH_UNCHECKED 0x4 /* skip the global-window confinement check */
#define EBPF_BATCH_SYS_NR 0x8    /* EBPF_CTX_SYSCALL: only records whose id == sys_nr run (per-syscall attach) */
#define EBPF_BATCH_TIMED 0x10    /* record events around the batch's kernels (bpftime_amd_last_batch_ms) */

struct ebpf_batch {
	uint32_t ctx_kind;       /* EBPF_CTX_* */
	uint32_t flags;          /* EBPF_BATCH_* */
	uint64_t count;          /* units */
	void *data;              /* device base of unit slots */
	uint64_t stride;         /* bytes between slots */
	const uint32_t *lens;    /* device per-unit lengths, or NULL -> fixed_len */
	uint32_t fixed_len;
	uint32_t ingress_ifindex;
	uint32_t rx_queue_index;
	uint32_t head;           /* XDP: initial data offset inside each slot */
	uint32_t *verdicts;      /* device u32 (r0) per unit, or NULL */
	uint64_t *rets;          /* device u64 r0 per unit, or NULL */
	int32_t *data_off_out;   /* XDP: data - slot after the program, or NULL */
	uint32_t *len_out;       /* XDP: data_end - data after the program, or NULL */
	uint64_t first_unit;     /* global index of unit 0 (shards) */
	void *stream;            /* hipStream_t, NULL = default stream */
	/* AF_XDP descriptor mode (descs != NULL): `data` is a umem of umem_bytes,
	 * unit i is the frame at data + descs[i].addr of descs[i].len bytes
	 * (struct xdp_desc, linux/if_xdp.h), `stride` the umem chunk size
	 * (ctx buffer_start / buffer_end = the frame's chunk); lens / fixed_len /
	 * head are not used.  A descriptor outside the umem fails its unit. */
	const struct ebpf_xdp_desc *descs;
	uint64_t umem_bytes;
	int64_t sys_nr;          /* with EBPF_BATCH_SYS_NR: the syscall nr a per-syscall program is attached to */
	/* Syscall dispatch state (bpftime_amd_syscall_dispatch_records sets these; NULL / 0
	 * otherwise).  Per unit a u32 of flags -- bit 0: an enter program overrode the
	 * syscall's return (bpf_override_return 58 / bpf_set_retval 187,
	 * base_attach_impl.hpp:76-105), bit 1: an exit program did -- and the i64 the
	 * dispatch returns for the record (the override value when one was set).
	 * sys_phase 1 (enter) / 2 (exit) is the bit those helpers set; an exit batch skips
	 * units whose bit 0 is set (syscall_trace_attach_impl.cpp:70-72).  Without
	 * sys_state helpers 58 / 187 fail the unit (the reference throws when no return
	 * callback is set). */
	uint32_t *sys_state;
	int64_t *sys_ret;
	uint32_t sys_phase;
	/* bpf_get_current_pid_tgid (14, bpf_helper.cpp:330-348) is the calling thread's
	 * tgid << 32 | tid: in a syscall replay the recorded caller's, a u64 at this
	 * offset from each unit (96-B records: +88 of the record); 0: the thread that
	 * launches the batch */
	int32_t pid_tgid_off;
	/* bpf_ktime_get_ns (5, bpf_helper.cpp:357-362) in a syscall replay: the
	 * recorded clock, a u64 at this offset from each unit (128-B records: +96 of
	 * the record at sys_enter, +104 at sys_exit); 0: the device clock.
	 * Both offsets are syscall-kind only, multiples of 8, and the u64 must lie
	 * inside the unit (EBPF_CTX_SYSCALL: off + 8 <= stride; EBPF_CTX_SYSCALL_EXIT
	 * units with stride >= 96 are the tail of a record whose first 64 bytes are
	 * the enter ctx: off + 8 <= stride - 64); else the batch fails (-1, named). */
	int32_t ktime_off;
	/* ... or, for struct-of-arrays replays, each in its own device array: unit
	 * i's pid_tgid / clock is the u64 at arr + i * stride (non-NULL arrays take
	 * the place of the offsets; syscall kinds only, stride a multiple of 8) */
	const void *pid_tgid_arr;
	uint64_t pid_tgid_stride;
	const void *ktime_arr;
	uint64_t ktime_stride;
};

/* linux/if_xdp.h struct xdp_desc */
struct ebpf_xdp_desc {
	uint64_t addr;
	uint32_t len;
	uint32_t options;
};

/* Launches the loaded program over `batch`.  Returns 0 when launched (async),
 * or with EBPF_BATCH_SYNC the number of units whose exec failed (>= 0);
 * -1 on API errors. */
int ebpf_exec_batch(const struct ebpf_vm *vm, const struct ebpf_batch *batch);
/* ctx kind used by ebpf_exec (default EBPF_CTX_RAW) */
int ebpf_set_ctx_kind(struct ebpf_vm *vm, uint32_t ctx_kind);

#ifdef __cplusplus
}
#endif
#endif

/*
 * ORACLE (test infrastructure only) -- see oracle.h.
 *
 * Batch drivers around orc_vm_exec, i.e. what a packet / record driver does
 * with the reference CPU path: the external DPDK/AF_XDP runner
 * (example/xdp-counter/README.md:26-28) calling bpftime_prog_exec per packet
 * (runtime/src/bpftime_prog.cpp:231-260: ret = 0 on exec error), and the
 * syscall dispatcher (attach/syscall_trace_attach_impl/src/
 * syscall_trace_attach_impl.cpp:18-67).  Timing follows
 * tools/bpftimetool/main.cpp:42-58 (steady clock around the loop only).
 */
#define _GNU_SOURCE
#include "oracle.h"
#include <sched.h>
#include <string.h>
#include <time.h>

struct xdp_md_userspace { /* runtime/extension/userspace_xdp.h:6-17 */
	uint64_t data, data_end;
	uint32_t data_meta, ingress_ifindex, rx_queue_index, egress_ifindex;
	uint64_t buffer_start, buffer_end;
};

static inline uint64_t exec_or_zero(struct orc_vm *vm, void *mem, size_t len)
{
	uint64_t v = 0;
	if (orc_vm_exec(vm, mem, len, &v) < 0)
		v = 0;
	return v;
}

int orc_run_xdp(struct orc_vm *vm, uint8_t *base, uint64_t n, uint64_t stride, const uint32_t *lens,
		uint32_t fixed_len, uint32_t *verdicts, int32_t *out_data_off, uint32_t *out_len,
		uint32_t ifindex, uint32_t rxq, uint32_t head)
{
	for (uint64_t i = 0; i < n; i++) {
		uint8_t *slot = base + i * stride;
		uint32_t len = lens ? lens[i] : fixed_len;
		/* bpf_tail_call copies 64 bytes from the 48-B ctx (bpf_helper.cpp:631-634):
		 * keep that read inside one zeroed object */
		union {
			struct xdp_md_userspace md;
			uint8_t bytes[64];
		} u;
		memset(&u, 0, sizeof(u));
		struct xdp_md_userspace ctx = {
			.data = (uintptr_t)slot + head,
			.data_end = (uintptr_t)slot + head + len,
			.data_meta = 0,
			.ingress_ifindex = ifindex,
			.rx_queue_index = rxq,
			.egress_ifindex = 0,
			.buffer_start = (uintptr_t)slot,
			.buffer_end = (uintptr_t)slot + stride,
		};
		u.md = ctx;
		uint64_t v = exec_or_zero(vm, &u.md, sizeof(u.md));
		if (verdicts)
			verdicts[i] = (uint32_t)v;
		if (out_data_off)
			out_data_off[i] = (int32_t)(u.md.data - (uintptr_t)slot);
		if (out_len)
			out_len[i] = (uint32_t)(u.md.data_end - u.md.data);
	}
	return 0;
}

int orc_run_raw(struct orc_vm *vm, uint8_t *base, uint64_t n, uint64_t stride, uint32_t len, uint64_t *rets)
{
	for (uint64_t i = 0; i < n; i++) {
		uint64_t v = exec_or_zero(vm, base + i * stride, len);
		if (rets)
			rets[i] = v;
	}
	return 0;
}

struct trace_event_raw_sys_enter { /* syscall_trace_attach_impl.hpp:17-29 */
	uint16_t type;
	uint8_t flags, preempt_count;
	int32_t pid;
	int64_t id;
	uint64_t args[6];
};

int orc_run_syscall(struct orc_vm *vm, const uint8_t *recs, uint64_t n, uint64_t *rets, uint8_t *ran)
{
	for (uint64_t i = 0; i < n; i++) {
		const struct trace_event_raw_sys_enter *r = (const void *)(recs + i * 64);
		int64_t nr = r->id;
		if (nr == 231 /*__NR_exit_group*/ || nr == 60 /*__NR_exit*/) { /* :25 */
			if (rets)
				rets[i] = 0;
			if (ran)
				ran[i] = 0;
			continue;
		}
		struct trace_event_raw_sys_enter ctx; /* :57-66 */
		memset(&ctx, 0, sizeof(ctx));
		ctx.id = nr;
		memcpy(ctx.args, r->args, sizeof(ctx.args));
		uint64_t v = exec_or_zero(vm, &ctx, sizeof(ctx));
		if (rets)
			rets[i] = v;
		if (ran)
			ran[i] = 1;
	}
	return 0;
}

struct trace_event_raw_sys_exit { /* syscall_trace_attach_impl.hpp:31-36 */
	uint16_t type;
	uint8_t flags, preempt_count;
	int32_t pid;
	int64_t id;
	int64_t ret;
};

/* syscall_trace_attach_impl.hpp:92-98: attach entries by id; the callback
 * sets are std::set of entry pointers, kept here in attach order */
#define ORC_SYS_MAX 256
static struct {
	int id;
	struct orc_vm *vm;
	int64_t sys_nr;
	int enter;
} g_sys[ORC_SYS_MAX];
static int g_sys_n, g_sys_next = 1;

int orc_sys_attach(struct orc_vm *vm, int64_t sys_nr, int is_enter)
{
	if (sys_nr >= 512 || sys_nr < -1 || g_sys_n == ORC_SYS_MAX) /* :134-139 */
		return -22;
	g_sys[g_sys_n].id = g_sys_next;
	g_sys[g_sys_n].vm = vm;
	g_sys[g_sys_n].sys_nr = sys_nr;
	g_sys[g_sys_n].enter = is_enter != 0;
	g_sys_n++;
	return g_sys_next++;
}

int orc_sys_detach(int id) /* :96-119 */
{
	for (int i = 0; i < g_sys_n; i++)
		if (g_sys[i].id == id) {
			memmove(&g_sys[i], &g_sys[i + 1], (size_t)(g_sys_n - i - 1) * sizeof(g_sys[0]));
			g_sys_n--;
			return 0;
		}
	return -2;
}

void orc_sys_reset(void)
{
	g_sys_n = 0;
	g_sys_next = 1;
}

/* run_callbacks (:41-53) over one callback set: each on its own ctx copy,
 * exec failures ignored */
static void run_set(int enter, int global, int64_t nr, const void *ctx, size_t len)
{
	for (int i = 0; i < g_sys_n; i++) {
		if (g_sys[i].enter != enter || (global ? g_sys[i].sys_nr != -1 : g_sys[i].sys_nr != nr))
			continue;
		uint8_t copy[64];
		memcpy(copy, ctx, len);
		uint64_t v;
		(void)orc_vm_exec(g_sys[i].vm, copy, len, &v);
	}
}

static int any_set(int enter, int64_t nr)
{
	for (int i = 0; i < g_sys_n; i++)
		if (g_sys[i].enter == enter && (g_sys[i].sys_nr == -1 || (nr >= 0 && g_sys[i].sys_nr == nr)))
			return 1;
	return 0;
}

int orc_sys_dispatch(const uint8_t *recs, uint64_t n, uint32_t rec_size, int64_t *out)
{
	if (rec_size != 64 && rec_size != 96 && rec_size != 128)
		return -22;
	for (uint64_t i = 0; i < n; i++) {
		const uint8_t *r = recs + i * rec_size;
		const struct trace_event_raw_sys_enter *er = (const void *)r;
		const int64_t nr = er->id;
		/* the "original syscall" is the recorded one: its ret */
		const int64_t ret = rec_size >= 96 ? ((const struct trace_event_raw_sys_exit *)(r + 64))->ret : 0;
		if (nr == 231 /*__NR_exit_group*/ || nr == 60 /*__NR_exit*/) { /* :25-26 */
			if (out)
				out[i] = ret;
			continue;
		}
		const int64_t pnr = nr >= 0 && nr < 512 ? nr : -2; /* no per-syscall set */
		if (rec_size >= 96) /* the recorded caller (bpf_helper.cpp:330-348) */
			orc_pid_tgid_recorded(1, *(const uint64_t *)(r + 88));
		if (rec_size == 128) /* the recorded clock at sys_enter (bpf_helper.cpp:357-362) */
			orc_ktime_recorded(1, *(const uint64_t *)(r + 96));
		orc_retval.active = 1; /* :35-40 */
		orc_retval.overridden = 0;
		if (any_set(1, pnr)) { /* :55-67 */
			struct trace_event_raw_sys_enter ctx;
			memset(&ctx, 0, sizeof(ctx));
			ctx.id = nr;
			memcpy(ctx.args, er->args, sizeof(ctx.args));
			run_set(1, 0, pnr, &ctx, sizeof(ctx));
			run_set(1, 1, pnr, &ctx, sizeof(ctx));
		}
		orc_retval.active = 0; /* :68-72 */
		if (orc_retval.overridden) {
			if (out)
				out[i] = orc_retval.value;
			continue;
		}
		orc_retval.active = 1; /* :73-78 */
		if (rec_size == 128) /* ... and after the call returned */
			orc_ktime_recorded(1, *(const uint64_t *)(r + 104));
		if (any_set(0, pnr)) { /* :80-89 */
			struct trace_event_raw_sys_exit ctx;
			memset(&ctx, 0, sizeof(ctx));
			ctx.id = nr;
			ctx.ret = ret;
			run_set(0, 0, pnr, &ctx, sizeof(ctx));
			run_set(0, 1, pnr, &ctx, sizeof(ctx));
		}
		orc_retval.active = 0; /* :90-94 */
		if (out)
			out[i] = orc_retval.overridden ? orc_retval.value : ret;
	}
	orc_pid_tgid_recorded(0, 0);
	orc_ktime_recorded(0, 0);
	return 0;
}

double orc_time_xdp(struct orc_vm *vm, uint8_t *base, uint64_t n, uint64_t stride, uint32_t fixed_len,
		    uint32_t *verdicts, int pin_cpu)
{
	cpu_set_t old;
	int pinned = 0;
	if (pin_cpu >= 0) {
		cpu_set_t set;
		CPU_ZERO(&set);
		CPU_SET(pin_cpu, &set);
		sched_getaffinity(0, sizeof(old), &old);
		pinned = sched_setaffinity(0, sizeof(set), &set) == 0;
	}
	struct timespec t0, t1;
	clock_gettime(CLOCK_MONOTONIC, &t0);
	orc_run_xdp(vm, base, n, stride, NULL, fixed_len, verdicts, NULL, NULL, 0, 0, 0);
	clock_gettime(CLOCK_MONOTONIC, &t1);
	if (pinned)
		sched_setaffinity(0, sizeof(old), &old);
	return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

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

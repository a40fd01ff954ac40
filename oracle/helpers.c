/*
 * ORACLE (test infrastructure only) -- see oracle.h.
 *
 * Helper functions the device path implements, restated from
 * runtime/src/bpf_helper.cpp:
 *   1/2/3 map lookup/update/delete   :387-408 (map arg = fd, cast to int)
 *   5 ktime_get_ns                    :357-362
 *   7 get_prandom_u32                 :301-304
 *   8 get_smp_processor_id            :702-710 (sched_getcpu -> orc_set_cpu)
 *   28 csum_diff                      :713-744
 *   44 xdp_adjust_head                :748-764
 *   65 xdp_adjust_tail                :766-776
 *   6 trace_printk                    :64-76   (orc_vm_register_trace_helpers;
 *   14 get_current_pid_tgid           :330-348  the host-process helpers of
 *                                               tools/aot/example/malloc.json)
 *   58 override_return, 187 set_retval attach/base_attach_impl/
 *                                     base_attach_impl.hpp:76-105 (the thread's
 *                                     return callback; orc_sys_dispatch sets it)
 * Registration order follows the kernel + shm-maps helper groups
 * (bpf_helper.cpp:1177-1401).
 */
#include "oracle.h"
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

struct xdp_md_userspace { /* runtime/extension/userspace_xdp.h:6-17 */
	uint64_t data, data_end;
	uint32_t data_meta, ingress_ifindex, rx_queue_index, egress_ifindex;
	uint64_t buffer_start, buffer_end;
};

static uint64_t h_lookup(uint64_t map, uint64_t key, uint64_t a, uint64_t b, uint64_t c)
{
	(void)a, (void)b, (void)c;
	return (uint64_t)(uintptr_t)orc_map_lookup((int)map, (const void *)(uintptr_t)key);
}

static uint64_t h_update(uint64_t map, uint64_t key, uint64_t value, uint64_t flags, uint64_t c)
{
	(void)c;
	return (uint64_t)orc_map_update((int)map, (const void *)(uintptr_t)key, (const void *)(uintptr_t)value,
					flags);
}

static uint64_t h_delete(uint64_t map, uint64_t key, uint64_t a, uint64_t b, uint64_t c)
{
	(void)a, (void)b, (void)c;
	return (uint64_t)orc_map_delete((int)map, (const void *)(uintptr_t)key);
}

/* a replayed call's recorded clock (orc_sys_dispatch, 128-B records) */
static int g_kt_rec_on;
static uint64_t g_kt_rec;

void orc_ktime_recorded(int on, uint64_t v)
{
	g_kt_rec_on = on;
	g_kt_rec = v;
}

static uint64_t h_ktime(uint64_t a, uint64_t b, uint64_t c, uint64_t d, uint64_t e)
{
	(void)a, (void)b, (void)c, (void)d, (void)e;
	if (g_kt_rec_on)
		return g_kt_rec;
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ULL + (uint64_t)ts.tv_nsec;
}

static uint64_t h_prandom(uint64_t a, uint64_t b, uint64_t c, uint64_t d, uint64_t e)
{
	(void)a, (void)b, (void)c, (void)d, (void)e;
	return (uint32_t)rand();
}

extern int orc_get_cpu(void);
static uint64_t h_cpu(uint64_t a, uint64_t b, uint64_t c, uint64_t d, uint64_t e)
{
	(void)a, (void)b, (void)c, (void)d, (void)e;
	return (uint64_t)orc_get_cpu();
}

/* bpf_helper.cpp:713-744 (from ebpf-for-windows) */
static uint64_t h_csum_diff(uint64_t from_, uint64_t from_size_, uint64_t to_, uint64_t to_size_,
			    uint64_t seed_)
{
	const void *from = (const void *)(uintptr_t)from_;
	const void *to = (const void *)(uintptr_t)to_;
	int from_size = (int)from_size_, to_size = (int)to_size_, seed = (int)seed_;
	int csum_diff = -EINVAL;
	if ((from_size % 4 != 0) || (to_size % 4 != 0))
		goto out;
	csum_diff = seed;
	if (to != NULL)
		for (int i = 0; i < to_size / 2; i++)
			csum_diff += (uint16_t)(*((const uint16_t *)to + i));
	if (from != NULL)
		for (int i = 0; i < from_size / 2; i++)
			csum_diff += (uint16_t)(~*((const uint16_t *)from + i));
	if (csum_diff < 0)
		csum_diff = -EINVAL;
out:
	return (uint64_t)(int64_t)csum_diff;
}

#define ETH_HLEN 14
/* bpf_helper.cpp:748-764 */
static uint64_t h_adjust_head(uint64_t ctx, uint64_t off_, uint64_t a, uint64_t b, uint64_t c)
{
	(void)a, (void)b, (void)c;
	struct xdp_md_userspace *xdp = (struct xdp_md_userspace *)(uintptr_t)ctx;
	int offset = (int)off_;
	uint64_t data = xdp->data + (int64_t)offset;
	if (data > xdp->data_end - ETH_HLEN || data > xdp->buffer_end)
		return (uint64_t)(int64_t)-EINVAL;
	if (data < xdp->buffer_start) {
		memmove((void *)(uintptr_t)(xdp->buffer_start + (xdp->buffer_start - data)),
			(void *)(uintptr_t)xdp->data, xdp->data_end - xdp->data);
		data = xdp->buffer_start;
	}
	xdp->data = data;
	return 0;
}

/* bpf_helper.cpp:766-776 */
static uint64_t h_adjust_tail(uint64_t ctx, uint64_t delta_, uint64_t a, uint64_t b, uint64_t c)
{
	(void)a, (void)b, (void)c;
	struct xdp_md_userspace *x = (struct xdp_md_userspace *)(uintptr_t)ctx;
	int delta = (int)delta_;
	uint64_t data = x->data_end + (int64_t)delta;
	if (data < x->data || data < x->buffer_start || data > x->buffer_end)
		return (uint64_t)(int64_t)-EINVAL;
	x->data_end = data;
	return 0;
}

/* bpf_helper.cpp:778-788 (no fragmented packets) */
static uint64_t h_xdp_load_bytes(uint64_t ctx, uint64_t off_, uint64_t buf, uint64_t len_, uint64_t c)
{
	(void)c;
	struct xdp_md_userspace *x = (struct xdp_md_userspace *)(uintptr_t)ctx;
	uint32_t offset = (uint32_t)off_, len = (uint32_t)len_;
	uint64_t data = x->data + offset;
	if (data + len > x->data_end)
		return (uint64_t)(int64_t)-EINVAL;
	memcpy((void *)(uintptr_t)buf, (const void *)(uintptr_t)data, len);
	return 0;
}

/* bpftime_trace_printk (:64-76): vprintf(fmt, r3..r5), returns 0.  Here the
 * formatted text is appended to a log the tests read (orc_trace_log) instead
 * of stdout; conversions d i u x X c s %% with l / ll length, as printf. */
static char g_trace[1 << 16];
static size_t g_trace_len;

size_t orc_trace_log(char *out, size_t cap)
{
	size_t n = g_trace_len < cap ? g_trace_len : cap;
	if (out)
		memcpy(out, g_trace, n);
	return g_trace_len;
}

void orc_trace_log_reset(void)
{
	g_trace_len = 0;
}

static void trace_put(const char *s, size_t n)
{
	if (n > sizeof(g_trace) - g_trace_len)
		n = sizeof(g_trace) - g_trace_len;
	memcpy(g_trace + g_trace_len, s, n);
	g_trace_len += n;
}

static uint64_t h_trace_printk(uint64_t fmt_, uint64_t fmt_size, uint64_t a3, uint64_t a4, uint64_t a5)
{
	const char *f = (const char *)(uintptr_t)fmt_;
	const uint64_t args[3] = { a3, a4, a5 };
	int ai = 0;
	char buf[64];
	(void)fmt_size; /* vprintf reads up to the NUL, whatever the size says */
	for (; *f; f++) {
		if (*f != '%') {
			trace_put(f, 1);
			continue;
		}
		f++;
		int l = 0;
		while (*f == 'l') {
			l++;
			f++;
		}
		if (!*f)
			break;
		const uint64_t v = ai < 3 ? args[ai] : 0;
		int n = 0;
		switch (*f) {
		case '%':
			trace_put("%", 1);
			continue;
		case 'd':
		case 'i':
			n = l ? snprintf(buf, sizeof(buf), "%lld", (long long)v) : snprintf(buf, sizeof(buf), "%d", (int)v);
			break;
		case 'u':
			n = l ? snprintf(buf, sizeof(buf), "%llu", (unsigned long long)v) :
				snprintf(buf, sizeof(buf), "%u", (unsigned)v);
			break;
		case 'x':
		case 'X':
			n = l ? snprintf(buf, sizeof(buf), *f == 'x' ? "%llx" : "%llX", (unsigned long long)v) :
				snprintf(buf, sizeof(buf), *f == 'x' ? "%x" : "%X", (unsigned)v);
			break;
		case 'c':
			buf[0] = (char)v;
			n = 1;
			break;
		case 's':
			if (v)
				trace_put((const char *)(uintptr_t)v, strlen((const char *)(uintptr_t)v));
			ai++;
			continue;
		default:
			continue;
		}
		ai++;
		trace_put(buf, (size_t)n);
	}
	return 0;
}

/* bpftime_get_current_pid_tgid (:330-348): getpid() << 32 | gettid(), or
 * the value a test fixes with orc_set_pid_tgid */
static int g_pid_set;
static uint64_t g_pid_tgid;

void orc_set_pid_tgid(uint64_t v)
{
	g_pid_tgid = v;
	g_pid_set = 1;
}

/* a replayed call's recorded caller (orc_sys_dispatch, 96-B records) */
static int g_pid_rec_on;
static uint64_t g_pid_rec;

void orc_pid_tgid_recorded(int on, uint64_t v)
{
	g_pid_rec_on = on;
	g_pid_rec = v;
}

static uint64_t h_pid_tgid(uint64_t a, uint64_t b, uint64_t c, uint64_t d, uint64_t e)
{
	if (g_pid_rec_on)
		return g_pid_rec;
	if (g_pid_set)
		return g_pid_tgid;
	return ((uint64_t)getpid() << 32) | (uint32_t)syscall(SYS_gettid);
}

int orc_vm_register_trace_helpers(struct orc_vm *vm)
{
	return orc_vm_register(vm, 6, "bpf_trace_printk", h_trace_printk) |
	       orc_vm_register(vm, 14, "bpf_get_current_pid_tgid", h_pid_tgid);
}

int orc_vm_register_xdp_load_bytes(struct orc_vm *vm)
{
	return orc_vm_register(vm, 189, "bpf_xdp_load_bytes", h_xdp_load_bytes);
}

/* bpf_helper.cpp:451-504 (map "pointer" = fd; flags other than 0 only warn).
 * bpf_ringbuf_output submits to the fd it reserved from (:460-465);
 * bpf_ringbuf_submit / _discard read the fd from the record header, ptr[-1]
 * (:478-479), which for a record whose data wrapped to the ring's first byte
 * is the zeroed word in front of the data (fd 0). */
static uint64_t h_rb_output(uint64_t rb, uint64_t data, uint64_t size, uint64_t flags, uint64_t c)
{
	(void)flags, (void)c;
	void *buf = orc_ringbuf_reserve((int)rb, size);
	if (!buf)
		return (uint64_t)-1;
	memcpy(buf, (const void *)(uintptr_t)data, size);
	orc_ringbuf_submit_fd((int)rb, buf, 0);
	return 0;
}

static uint64_t h_rb_reserve(uint64_t rb, uint64_t size, uint64_t flags, uint64_t b, uint64_t c)
{
	(void)flags, (void)b, (void)c;
	return (uint64_t)(uintptr_t)orc_ringbuf_reserve((int)rb, size);
}

static uint64_t h_rb_submit(uint64_t data, uint64_t flags, uint64_t a, uint64_t b, uint64_t c)
{
	(void)flags, (void)a, (void)b, (void)c;
	orc_ringbuf_submit_fd(((const int32_t *)(uintptr_t)data)[-1], (const void *)(uintptr_t)data, 0);
	return 0;
}

static uint64_t h_rb_discard(uint64_t data, uint64_t flags, uint64_t a, uint64_t b, uint64_t c)
{
	(void)flags, (void)a, (void)b, (void)c;
	orc_ringbuf_submit_fd(((const int32_t *)(uintptr_t)data)[-1], (const void *)(uintptr_t)data, 1);
	return 0;
}

/* ---- programs + bpf_tail_call (runtime/src/bpf_helper.cpp:568-650) ---- */
static struct {
	int used;
	uint8_t *insns;
	uint32_t n;
} g_progs[ORC_MAX_FDS];

int orc_prog_create(int fd, const void *insns, uint32_t n)
{
	if (fd < 0 || fd >= ORC_MAX_FDS)
		return -1;
	orc_prog_close(fd);
	g_progs[fd].insns = malloc((size_t)n * 8 + 1);
	memcpy(g_progs[fd].insns, insns, (size_t)n * 8);
	g_progs[fd].n = n;
	g_progs[fd].used = 1;
	return fd;
}

void orc_prog_close(int fd)
{
	if (fd < 0 || fd >= ORC_MAX_FDS || !g_progs[fd].used)
		return;
	free(g_progs[fd].insns);
	g_progs[fd].used = 0;
}

int orc_is_prog_fd(int fd)
{
	return fd >= 0 && fd < ORC_MAX_FDS && g_progs[fd].used;
}

static __thread uint32_t g_tail_depth;

static uint64_t h_tail_call(uint64_t ctx, uint64_t prog_array, uint64_t index, uint64_t a4, uint64_t a5)
{
	int fd = (int)prog_array;
	if (!orc_map_is_prog_array(fd))
		return (uint64_t)-1;
	int idx = (int)index;
	const int32_t *p = orc_map_lookup(fd, &idx);
	if (!p)
		return (uint64_t)-1;
	int to = *p;
	if (!orc_is_prog_fd(to))
		return (uint64_t)-1;
	if (g_tail_depth >= 32) /* MAX_TAIL_CALL_CNT */
		return (uint64_t)-1;
	g_tail_depth++;
	uint64_t rv = (uint64_t)-1;
	struct orc_vm *vm = orc_vm_create();
	char err[256];
	if (orc_vm_register_default_helpers(vm) == 0 &&
	    orc_vm_load(vm, g_progs[to].insns, g_progs[to].n * 8, err, sizeof(err)) == 0) {
		uint8_t context[64];
		if (ctx)
			memcpy(context, (const void *)(uintptr_t)ctx, sizeof(context));
		else
			memset(context, 0, sizeof(context));
		uint64_t ret = 0;
		if (orc_vm_exec(vm, context, sizeof(context), &ret) == 0)
			rv = ret;
	}
	orc_vm_destroy(vm);
	g_tail_depth--;
	return rv;
}

/* base_attach_impl.hpp:18-19 curr_thread_override_return_callback: set by
 * orc_sys_dispatch around each phase (syscall_trace_attach_impl.cpp:35-40,
 * :73-78); the callback records {overridden, value}.  Unset, the helpers
 * throw (:86-90, :99-103), which ends the program: orc_helper_abort makes
 * the interpreter fail the exec. */
struct orc_retval_cb orc_retval = {0, 0, 0};
int orc_helper_abort;

static uint64_t set_retval(uint64_t v)
{
	if (!orc_retval.active) {
		orc_helper_abort = 1;
		return 0;
	}
	orc_retval.overridden = 1;
	orc_retval.value = (int64_t)v;
	return 0;
}

static uint64_t h_override_return(uint64_t ctx, uint64_t v, uint64_t a, uint64_t b, uint64_t c)
{
	(void)ctx, (void)a, (void)b, (void)c;
	return set_retval(v);
}

static uint64_t h_set_retval(uint64_t v, uint64_t a, uint64_t b, uint64_t c, uint64_t d)
{
	(void)a, (void)b, (void)c, (void)d;
	return set_retval(v);
}

int orc_vm_register_default_helpers(struct orc_vm *vm)
{
	int err = 0;
	/* kernel helper group subset (bpf_helper.cpp:1177-1356) */
	err |= orc_vm_register(vm, 8, "bpf_get_smp_processor_id", h_cpu);
	err |= orc_vm_register(vm, 28, "bpf_csum_diff", h_csum_diff);
	err |= orc_vm_register(vm, 44, "bpf_xdp_adjust_head", h_adjust_head);
	err |= orc_vm_register(vm, 65, "bpf_xdp_adjust_tail", h_adjust_tail);
	err |= orc_vm_register(vm, 5, "bpf_ktime_get_ns", h_ktime);
	err |= orc_vm_register(vm, 7, "bpf_get_prandom_u32", h_prandom);
	err |= orc_vm_register(vm, 131, "bpf_ringbuf_reserve", h_rb_reserve);
	err |= orc_vm_register(vm, 132, "bpf_ringbuf_submit", h_rb_submit);
	err |= orc_vm_register(vm, 133, "bpf_ringbuf_discard", h_rb_discard);
	err |= orc_vm_register(vm, 130, "bpf_ringbuf_output", h_rb_output);
	err |= orc_vm_register(vm, 12, "bpf_tail_call", h_tail_call);
	/* shm maps helper group (bpf_helper.cpp:1359-1401) */
	err |= orc_vm_register(vm, 1, "bpf_map_lookup_elem", h_lookup);
	err |= orc_vm_register(vm, 2, "bpf_map_update_elem", h_update);
	err |= orc_vm_register(vm, 3, "bpf_map_delete_elem", h_delete);
	/* kernel helper group, bpf_helper.cpp:1264-1286 */
	err |= orc_vm_register(vm, 58, "bpf_override_return", h_override_return);
	err |= orc_vm_register(vm, 187, "bpf_set_retval", h_set_retval);
	err |= orc_vm_register(vm, 14, "bpf_get_current_pid_tgid", h_pid_tgid);
	return err ? -1 : 0;
}

/*
 * ORACLE (test infrastructure only) -- see oracle.h.
 *
 * Restatement of the CPU interpreter bpftime drives for this path:
 *   bpftime_prog::bpftime_prog_exec   runtime/src/bpftime_prog.cpp:231-260
 *   -> ebpf_exec                      vm/vm-core/src/ebpf-vm.cpp:56-60
 *   -> bpftime_ubpf_vm::exec          vm/compat/ubpf-vm/compat_ubpf.cpp:207-210
 *   -> ubpf_exec                      third_party/ubpf (ABSENT: empty submodule)
 * and of the load-time rewrite bpftime_ubpf_vm::load_code
 * (compat_ubpf.cpp:61-200) + register_external_function (:50-59).
 *
 * ubpf is not in /root/reference, so its interpreter is restated from the
 * eBPF ISA as bpftime's opcode table defines it (vm/compat/include/
 * ebpf_inst.h:22-200) with ubpf's conventions: r1 = mem, r2 = mem_len,
 * r10 = top of a 512-B stack (ebpf-vm.h:47-49), ALU32 results zero-extended,
 * shift counts masked to 31/63, div by zero -> 0, mod by zero -> dst
 * unchanged, helpers called as fn(r1..r5) leaving r1-r5 untouched, bounds
 * checking OFF (vm/example/main.c:32).  PARITY
 * UNPINNED for the arithmetic beyond the analytic KATs.
 */
#include "oracle.h"
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ebpf_inst.h:22-28 */
struct ebpf_inst {
	uint8_t code;
	uint8_t dst : 4;
	uint8_t src : 4;
	int16_t off;
	int32_t imm;
};

#define CLS(c) ((c)&0x07)
enum { C_LD = 0, C_LDX, C_ST, C_STX, C_ALU, C_JMP, C_JMP32, C_ALU64 };

struct orc_vm {
	struct ebpf_inst *insts;
	uint32_t n;
	/* compat_ubpf.hpp:42-44: bpftime helper id -> ubpf id, next id from 1 */
	int remap_from[ORC_MAX_HELPERS];
	int remap_count;
	orc_helper_fn ext[ORC_MAX_HELPERS];
	char ext_name[ORC_MAX_HELPERS][32];
	int unwind_idx;
	uint64_t insn_count;
};

struct orc_vm *orc_vm_create(void)
{
	struct orc_vm *vm = calloc(1, sizeof(*vm));
	vm->unwind_idx = -1;
	return vm;
}

void orc_vm_destroy(struct orc_vm *vm)
{
	if (!vm)
		return;
	free(vm->insts);
	free(vm);
}

/* compat_ubpf.cpp:50-59: each registration allocates the next ubpf id. */
int orc_vm_register(struct orc_vm *vm, unsigned index, const char *name, orc_helper_fn fn)
{
	int next = vm->remap_count + 1;
	if (next >= ORC_MAX_HELPERS)
		return -1; /* ubpf_register fails past 64 helpers */
	for (int i = 0; i < vm->remap_count; i++) {
		if (vm->remap_from[i] == (int)index) {
			/* helper_id_map[index] = next: the later mapping wins */
			vm->remap_from[i] = -1;
		}
	}
	vm->remap_from[vm->remap_count] = (int)index;
	vm->remap_count++;
	vm->ext[next] = fn;
	snprintf(vm->ext_name[next], sizeof(vm->ext_name[next]), "%s", name ? name : "");
	return 0;
}

void orc_vm_set_unwind_index(struct orc_vm *vm, int idx)
{
	vm->unwind_idx = idx;
}

static int remap_lookup(const struct orc_vm *vm, int32_t imm)
{
	for (int i = vm->remap_count - 1; i >= 0; i--)
		if (vm->remap_from[i] == imm)
			return i + 1;
	return -1;
}

static int fail(char *errbuf, size_t errlen, int code, const char *fmt, ...)
	__attribute__((format(printf, 4, 5)));
#include <stdarg.h>
static int fail(char *errbuf, size_t errlen, int code, const char *fmt, ...)
{
	if (errbuf && errlen) {
		va_list ap;
		va_start(ap, fmt);
		vsnprintf(errbuf, errlen, fmt, ap);
		va_end(ap);
	}
	return code;
}

static int opcode_known(uint8_t c)
{
	uint8_t cls = CLS(c);
	switch (cls) {
	case C_ALU:
	case C_ALU64: {
		uint8_t op = c & 0xf0;
		if (op > 0xd0)
			return 0;
		if (op == 0xd0) /* LE (0xd4) / BE (0xdc) are ALU32-only */
			return cls == C_ALU;
		if (op == 0x80) /* NEG takes no source */
			return (c & 0x08) == 0;
		return 1;
	}
	case C_JMP:
	case C_JMP32: {
		uint8_t op = c & 0xf0;
		if (op > 0xd0)
			return 0;
		if (cls == C_JMP32 && (op == 0x00 || op == 0x80 || op == 0x90))
			return 0;
		if (op == 0x00 || op == 0x80 || op == 0x90)
			return (c & 0x08) == 0;
		return 1;
	}
	case C_LDX:
		return (c & 0xe0) == 0x60;
	case C_ST:
		return (c & 0xe0) == 0x60;
	case C_STX:
		return (c & 0xe0) == 0x60 || (((c & 0xe0) == 0xc0) && ((c & 0x18) == 0x00 || (c & 0x18) == 0x18));
	case C_LD:
		return c == 0x18;
	}
	return 0;
}

static int writes_dst(uint8_t c)
{
	uint8_t cls = CLS(c);
	return cls == C_ALU || cls == C_ALU64 || cls == C_LDX || c == 0x18;
}

/* ubpf_load's validation (restated; ubpf absent -> messages unpinned). */
static int validate(const struct orc_vm *vm, const struct ebpf_inst *in, uint32_t n, char *errbuf,
		    size_t errlen)
{
	for (uint32_t i = 0; i < n; i++) {
		struct ebpf_inst d = in[i];
		if (!opcode_known(d.code))
			return fail(errbuf, errlen, -1, "unknown opcode 0x%02x at PC %u", d.code, i);
		if (d.src > 10)
			return fail(errbuf, errlen, -1, "invalid source register at PC %u", i);
		if (d.dst > 10 || (d.dst == 10 && writes_dst(d.code)))
			return fail(errbuf, errlen, -1, "invalid destination register at PC %u", i);
		uint8_t cls = CLS(d.code);
		if ((cls == C_JMP || cls == C_JMP32) && d.code != 0x85 && d.code != 0x95) {
			int64_t t = (int64_t)i + 1 + d.off;
			if (t < 0 || t >= (int64_t)n)
				return fail(errbuf, errlen, -1, "jump out of bounds at PC %u", i);
			if (t > 0 && in[t - 1].code == 0x18 && in[t].code == 0)
				return fail(errbuf, errlen, -1, "jump to middle of lddw at PC %u", i);
		}
		if (d.code == 0x85) {
			if (d.imm < 0 || d.imm >= ORC_MAX_HELPERS || !vm->ext[d.imm])
				return fail(errbuf, errlen, -1, "call to nonexistent function %d at PC %u",
					    d.imm, i);
		}
		if (d.code == 0x18) {
			if (i + 1 >= n || in[i + 1].code != 0)
				return fail(errbuf, errlen, -1, "incomplete lddw at PC %u", i);
			i++;
		}
	}
	return 0;
}

extern uint64_t orc_map_ptr_by_fd(uint32_t fd);
extern uint64_t orc_map_val(uint64_t map_ptr);

/* compat_ubpf.cpp:61-200 with bpftime_prog's lddw helpers (map_ptr_by_fd,
 * NULL, map_val, NULL, NULL: bpftime_prog.cpp:126-127). */
int orc_vm_load(struct orc_vm *vm, const void *code, uint32_t code_len, char *errbuf, size_t errlen)
{
	if (code_len % 8 != 0)
		return fail(errbuf, errlen, -1, "Length of code must be a multiple of 8");
	if (vm->insts)
		return fail(errbuf, errlen, -1,
			    "code has already been loaded into this VM. Use ebpf_unload_code() if you need to reuse this VM");
	uint32_t n = code_len / 8;
	if (n > ORC_MAX_INSTS)
		return fail(errbuf, errlen, -1, "too many instructions (max %u)", ORC_MAX_INSTS);
	struct ebpf_inst *in = malloc((n ? n : 1) * sizeof(*in));
	memcpy(in, code, code_len);
	for (uint32_t i = 0; i < n; i++) {
		struct ebpf_inst *cur = &in[i];
		if (cur->code == 0x85) {
			int id = remap_lookup(vm, cur->imm);
			if (id < 0) {
				int imm = cur->imm;
				free(in);
				if (imm >= 64)
					return fail(errbuf, errlen, -EINVAL, "invalid call immediate at PC %u", i);
				return fail(errbuf, errlen, -EINVAL, "call to nonexistent function %d at PC %u",
					    imm, i);
			}
			cur->imm = id;
		} else if (cur->code == 0x18) {
			if (i + 1 == n) {
				free(in);
				return fail(errbuf, errlen, -EINVAL,
					    "Unable to patch lddw instructions at %u, it's the last instruction", i);
			}
			struct ebpf_inst *nx = &in[i + 1];
			uint64_t imm;
			switch (cur->src) {
			case 0:
				imm = (uint64_t)(uint32_t)cur->imm | ((uint64_t)(uint32_t)nx->imm << 32);
				break;
			case 1:
				imm = orc_map_ptr_by_fd((uint32_t)cur->imm);
				break;
			case 2:
				imm = orc_map_val(orc_map_ptr_by_fd((uint32_t)cur->imm)) + (uint64_t)(int64_t)nx->imm;
				break;
			case 3:
				free(in);
				return fail(errbuf, errlen, -EINVAL,
					    "Unable to patch lddw instruction at %u, var_addr not defined", i);
			case 4:
				free(in);
				return fail(errbuf, errlen, -EINVAL,
					    "Unable to patch lddw instruction at %u, code_addr not defined", i);
			case 5:
				free(in);
				return fail(errbuf, errlen, -EINVAL,
					    "Unable to patch lddw instruction at %u, map_by_idx not defined", i);
			case 6:
				free(in);
				return fail(errbuf, errlen, -EINVAL,
					    "Unable to patch lddw instruction at %u, map_by_idx or map_val not defined", i);
			default:
				free(in);
				return fail(errbuf, errlen, -EINVAL,
					    "Unable to patch lddw instruction at %u, unsupported src_reg %u", i,
					    (unsigned)cur->src);
			}
			cur->imm = (int32_t)(uint32_t)(imm & 0xffffffffu);
			nx->imm = (int32_t)(uint32_t)(imm >> 32);
			cur->src = 0;
			i++;
		}
	}
	int err = validate(vm, in, n, errbuf, errlen);
	if (err < 0) {
		free(in);
		return err;
	}
	vm->insts = in;
	vm->n = n;
	return 0;
}

void orc_vm_unload(struct orc_vm *vm)
{
	free(vm->insts);
	vm->insts = NULL;
	vm->n = 0;
}

uint64_t orc_vm_insn_count(struct orc_vm *vm)
{
	return vm->insn_count;
}

void orc_vm_reset_insn_count(struct orc_vm *vm)
{
	vm->insn_count = 0;
}

static inline uint64_t bswap16(uint64_t v)
{
	return __builtin_bswap16((uint16_t)v);
}
static inline uint64_t bswap32(uint64_t v)
{
	return __builtin_bswap32((uint32_t)v);
}

#define U32(x) ((uint64_t)(uint32_t)(x))

int orc_vm_exec(struct orc_vm *vm, void *mem, size_t mem_len, uint64_t *ret)
{
	const struct ebpf_inst *in = vm->insts;
	if (!in)
		return -1;
	uint64_t reg[11] = {0};
	uint64_t stack[ORC_STACK_SIZE / 8];
	reg[1] = (uintptr_t)mem;
	reg[2] = (uint64_t)mem_len;
	reg[10] = (uintptr_t)stack + sizeof(stack);
	uint32_t pc = 0;
	uint64_t count = 0;
	for (;;) {
		if (pc >= vm->n)
			return -1;
		struct ebpf_inst d = in[pc++];
		count++;
		uint64_t *dst = &reg[d.dst];
		const uint64_t src = reg[d.src];
		const uint64_t simm = (uint64_t)(int64_t)d.imm; /* sign-extended */
		switch (d.code) {
		/* ---- ALU32 (results zero-extended) ---- */
		case 0x04: *dst = U32(*dst + simm); break;
		case 0x0c: *dst = U32(*dst + src); break;
		case 0x14: *dst = U32(*dst - simm); break;
		case 0x1c: *dst = U32(*dst - src); break;
		case 0x24: *dst = U32(*dst * simm); break;
		case 0x2c: *dst = U32(*dst * src); break;
		case 0x34: *dst = (uint32_t)d.imm ? U32((uint32_t)*dst / (uint32_t)d.imm) : 0; break;
		case 0x3c: *dst = (uint32_t)src ? U32((uint32_t)*dst / (uint32_t)src) : 0; break;
		case 0x44: *dst = U32(*dst | simm); break;
		case 0x4c: *dst = U32(*dst | src); break;
		case 0x54: *dst = U32(*dst & simm); break;
		case 0x5c: *dst = U32(*dst & src); break;
		case 0x64: *dst = U32((uint32_t)*dst << (d.imm & 31)); break;
		case 0x6c: *dst = U32((uint32_t)*dst << (src & 31)); break;
		case 0x74: *dst = U32((uint32_t)*dst >> (d.imm & 31)); break;
		case 0x7c: *dst = U32((uint32_t)*dst >> (src & 31)); break;
		case 0x84: *dst = U32(-(int64_t)*dst); break;
		case 0x94: *dst = (uint32_t)d.imm ? U32((uint32_t)*dst % (uint32_t)d.imm) : U32(*dst); break;
		case 0x9c: *dst = (uint32_t)src ? U32((uint32_t)*dst % (uint32_t)src) : U32(*dst); break;
		case 0xa4: *dst = U32(*dst ^ simm); break;
		case 0xac: *dst = U32(*dst ^ src); break;
		case 0xb4: *dst = U32(simm); break;
		case 0xbc: *dst = U32(src); break;
		case 0xc4: *dst = U32((int32_t)*dst >> (d.imm & 31)); break;
		case 0xcc: *dst = U32((int32_t)*dst >> (src & 31)); break;
		case 0xd4: /* LE: host is little-endian */
			if (d.imm == 16)
				*dst = (uint16_t)*dst;
			else if (d.imm == 32)
				*dst = (uint32_t)*dst;
			break;
		case 0xdc: /* BE */
			if (d.imm == 16)
				*dst = bswap16(*dst);
			else if (d.imm == 32)
				*dst = bswap32(*dst);
			else if (d.imm == 64)
				*dst = __builtin_bswap64(*dst);
			break;
		/* ---- ALU64 ---- */
		case 0x07: *dst += simm; break;
		case 0x0f: *dst += src; break;
		case 0x17: *dst -= simm; break;
		case 0x1f: *dst -= src; break;
		case 0x27: *dst *= simm; break;
		case 0x2f: *dst *= src; break;
		case 0x37: *dst = simm ? *dst / simm : 0; break;
		case 0x3f: *dst = src ? *dst / src : 0; break;
		case 0x47: *dst |= simm; break;
		case 0x4f: *dst |= src; break;
		case 0x57: *dst &= simm; break;
		case 0x5f: *dst &= src; break;
		case 0x67: *dst <<= (d.imm & 63); break;
		case 0x6f: *dst <<= (src & 63); break;
		case 0x77: *dst >>= (d.imm & 63); break;
		case 0x7f: *dst >>= (src & 63); break;
		case 0x87: *dst = (uint64_t)(-(int64_t)*dst); break;
		case 0x97: *dst = simm ? *dst % simm : *dst; break;
		case 0x9f: *dst = src ? *dst % src : *dst; break;
		case 0xa7: *dst ^= simm; break;
		case 0xaf: *dst ^= src; break;
		case 0xb7: *dst = simm; break;
		case 0xbf: *dst = src; break;
		case 0xc7: *dst = (uint64_t)((int64_t)*dst >> (d.imm & 63)); break;
		case 0xcf: *dst = (uint64_t)((int64_t)*dst >> (src & 63)); break;
		/* ---- memory (bounds check off) ---- */
		case 0x61: { uint32_t v; memcpy(&v, (void *)(uintptr_t)(src + d.off), 4); *dst = v; } break;
		case 0x69: { uint16_t v; memcpy(&v, (void *)(uintptr_t)(src + d.off), 2); *dst = v; } break;
		case 0x71: { uint8_t v; memcpy(&v, (void *)(uintptr_t)(src + d.off), 1); *dst = v; } break;
		case 0x79: { uint64_t v; memcpy(&v, (void *)(uintptr_t)(src + d.off), 8); *dst = v; } break;
		case 0x62: { uint32_t v = (uint32_t)d.imm; memcpy((void *)(uintptr_t)(*dst + d.off), &v, 4); } break;
		case 0x6a: { uint16_t v = (uint16_t)d.imm; memcpy((void *)(uintptr_t)(*dst + d.off), &v, 2); } break;
		case 0x72: { uint8_t v = (uint8_t)d.imm; memcpy((void *)(uintptr_t)(*dst + d.off), &v, 1); } break;
		case 0x7a: { uint64_t v = simm; memcpy((void *)(uintptr_t)(*dst + d.off), &v, 8); } break;
		case 0x63: { uint32_t v = (uint32_t)src; memcpy((void *)(uintptr_t)(*dst + d.off), &v, 4); } break;
		case 0x6b: { uint16_t v = (uint16_t)src; memcpy((void *)(uintptr_t)(*dst + d.off), &v, 2); } break;
		case 0x73: { uint8_t v = (uint8_t)src; memcpy((void *)(uintptr_t)(*dst + d.off), &v, 1); } break;
		case 0x7b: { uint64_t v = src; memcpy((void *)(uintptr_t)(*dst + d.off), &v, 8); } break;
		case 0xc3: /* atomic 32 (ebpf_inst.h:29-42); fetched values zero-extended */
		case 0xdb: { /* atomic 64 */
			int is64 = d.code == 0xdb;
			void *p = (void *)(uintptr_t)(*dst + d.off);
			int fetch = d.imm & 0x01;
			uint64_t old;
			if (d.imm == 0xf1) { /* CMPXCHG: r0 = old */
				if (is64) {
					uint64_t exp = reg[0];
					__atomic_compare_exchange_n((uint64_t *)p, &exp, reg[d.src], 0, __ATOMIC_SEQ_CST,
								    __ATOMIC_SEQ_CST);
					reg[0] = exp;
				} else {
					uint32_t exp = (uint32_t)reg[0];
					__atomic_compare_exchange_n((uint32_t *)p, &exp, (uint32_t)reg[d.src], 0,
								    __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST);
					reg[0] = exp;
				}
				break;
			}
			if (d.imm == 0xe1) { /* XCHG */
				if (is64)
					reg[d.src] = __atomic_exchange_n((uint64_t *)p, reg[d.src], __ATOMIC_SEQ_CST);
				else
					reg[d.src] = __atomic_exchange_n((uint32_t *)p, (uint32_t)reg[d.src],
									 __ATOMIC_SEQ_CST);
				break;
			}
			switch (d.imm & ~0x01) {
			case 0x00:
				old = is64 ? __atomic_fetch_add((uint64_t *)p, src, __ATOMIC_SEQ_CST)
					   : __atomic_fetch_add((uint32_t *)p, (uint32_t)src, __ATOMIC_SEQ_CST);
				break;
			case 0x40:
				old = is64 ? __atomic_fetch_or((uint64_t *)p, src, __ATOMIC_SEQ_CST)
					   : __atomic_fetch_or((uint32_t *)p, (uint32_t)src, __ATOMIC_SEQ_CST);
				break;
			case 0x50:
				old = is64 ? __atomic_fetch_and((uint64_t *)p, src, __ATOMIC_SEQ_CST)
					   : __atomic_fetch_and((uint32_t *)p, (uint32_t)src, __ATOMIC_SEQ_CST);
				break;
			case 0xa0:
				old = is64 ? __atomic_fetch_xor((uint64_t *)p, src, __ATOMIC_SEQ_CST)
					   : __atomic_fetch_xor((uint32_t *)p, (uint32_t)src, __ATOMIC_SEQ_CST);
				break;
			default:
				return -1;
			}
			if (fetch)
				reg[d.src] = old;
			break;
		}
		case 0x18: /* LDDW */
			*dst = U32(d.imm) | ((uint64_t)(uint32_t)in[pc].imm << 32);
			pc++;
			break;
		/* ---- JMP (64-bit compares; imm sign-extended) ---- */
#define J64(opc, cond_imm, cond_reg)                                                                     \
	case (opc):                                                                                          \
		if (cond_imm)                                                                                \
			pc += d.off;                                                                         \
		break;                                                                                       \
	case (opc) | 0x08:                                                                                   \
		if (cond_reg)                                                                                \
			pc += d.off;                                                                         \
		break;
		case 0x05: pc += d.off; break;
		J64(0x15, *dst == simm, *dst == src)
		J64(0x25, *dst > simm, *dst > src)
		J64(0x35, *dst >= simm, *dst >= src)
		J64(0x45, *dst & simm, *dst & src)
		J64(0x55, *dst != simm, *dst != src)
		J64(0x65, (int64_t)*dst > (int64_t)simm, (int64_t)*dst > (int64_t)src)
		J64(0x75, (int64_t)*dst >= (int64_t)simm, (int64_t)*dst >= (int64_t)src)
		J64(0xa5, *dst < simm, *dst < src)
		J64(0xb5, *dst <= simm, *dst <= src)
		J64(0xc5, (int64_t)*dst < (int64_t)simm, (int64_t)*dst < (int64_t)src)
		J64(0xd5, (int64_t)*dst <= (int64_t)simm, (int64_t)*dst <= (int64_t)src)
		/* ---- JMP32 ---- */
		J64(0x16, (uint32_t)*dst == (uint32_t)d.imm, (uint32_t)*dst == (uint32_t)src)
		J64(0x26, (uint32_t)*dst > (uint32_t)d.imm, (uint32_t)*dst > (uint32_t)src)
		J64(0x36, (uint32_t)*dst >= (uint32_t)d.imm, (uint32_t)*dst >= (uint32_t)src)
		J64(0x46, (uint32_t)*dst & (uint32_t)d.imm, (uint32_t)*dst & (uint32_t)src)
		J64(0x56, (uint32_t)*dst != (uint32_t)d.imm, (uint32_t)*dst != (uint32_t)src)
		J64(0x66, (int32_t)*dst > (int32_t)d.imm, (int32_t)*dst > (int32_t)src)
		J64(0x76, (int32_t)*dst >= (int32_t)d.imm, (int32_t)*dst >= (int32_t)src)
		J64(0xa6, (uint32_t)*dst < (uint32_t)d.imm, (uint32_t)*dst < (uint32_t)src)
		J64(0xb6, (uint32_t)*dst <= (uint32_t)d.imm, (uint32_t)*dst <= (uint32_t)src)
		J64(0xc6, (int32_t)*dst < (int32_t)d.imm, (int32_t)*dst < (int32_t)src)
		J64(0xd6, (int32_t)*dst <= (int32_t)d.imm, (int32_t)*dst <= (int32_t)src)
#undef J64
		case 0x85: {
			orc_helper_fn fn = vm->ext[d.imm];
			reg[0] = fn(reg[1], reg[2], reg[3], reg[4], reg[5]);
			if (orc_helper_abort) { /* the helper threw (helpers.c set_retval) */
				orc_helper_abort = 0;
				vm->insn_count += count;
				return -1;
			}
			if (d.imm == vm->unwind_idx && reg[0] == 0) {
				vm->insn_count += count;
				*ret = reg[0];
				return 0;
			}
			break;
		}
		case 0x95:
			vm->insn_count += count;
			*ret = reg[0];
			return 0;
		default:
			return -1;
		}
	}
}

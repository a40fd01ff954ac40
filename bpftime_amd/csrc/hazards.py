"""Wait-state check of the generated fast-path assembly (gen_fast.py).

The hardware does not interlock a few producer / consumer pairs; the
program must put independent instructions or s_nop between them.  Inside an
inline-asm block the compiler's hazard recognizer cannot help, so
gen_fast.py checks its own output with this module before it writes
fast_asm.inc, and `make` runs the check on every build.  Rules (CDNA3/4 ISA,
"Manually inserted wait states"), each `required` wait states between
producer and consumer:

  store-data  1  a VMEM store of more than 64 bits of data (global / flat /
                 buffer *_dwordx3, *_dwordx4), then a VALU write of any of its
                 data VGPRs (the store reads them after issue)
  sgpr-vmem   5  a VALU write of an SGPR (v_readfirstlane, v_readlane,
                 v_cmp sdst, carry-outs), then a VMEM instruction reading it
  sgpr-lane   4  a VALU write of an SGPR, then v_readlane / v_writelane using
                 it as the lane select
  trans       1  a transcendental VALU op (v_rcp / v_rsq / v_sqrt / v_exp /
                 v_log / v_sin / v_cos), then a VALU reading its result

Every instruction counts one wait state, `s_nop N` counts N + 1.  The check
walks the control-flow graph backwards from each consumer over every path
(fall-through, branches to labels, every handler entry and divergent stub
after any s_setpc_b64), so a producer before a branch is seen from the
branch target.
The block's entry is taken as a VALU write of every asm operand (%[name]:
the compiler may have produced an "s" operand with v_readfirstlane right
before the block) and its end as a VMEM read of them.  Index mode
(s_set_gpr_idx_on ... gpr_idx(DST)) writes v[k .. k + 21] for a written vk.
"""
from __future__ import annotations

import re
from typing import Dict, List, Optional, Set, Tuple

RULES = {"store-data": 1, "sgpr-vmem": 5, "sgpr-lane": 4, "trans": 1}
IDX_SPAN = 22  # index mode: r0..r10 pairs (v[R0 + 0 .. 21]) or staged dwords (<= 16)


def _regs(op: str) -> Set[str]:
    """Registers one operand names: v12, v[12:15], s40, s[40:47], vcc, exec,
    %[name] (an asm operand, by name)."""
    op = op.strip()
    m = re.fullmatch(r"([vs])\[(\d+):(\d+)\]", op)
    if m:
        return {f"{m.group(1)}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.fullmatch(r"([vs])(\d+)", op)
    if m:
        return {op}
    if op in ("vcc", "vcc_lo", "vcc_hi"):
        return {"vcc"}
    if op.startswith("%["):
        return {op.split("]")[0] + "]"}
    return set()


class Insn:
    __slots__ = ("i", "text", "mn", "ops", "waits", "vwrites", "swrites", "sreads_vmem", "lane_sel",
                 "store_data", "trans", "vreads", "valu", "uncond", "target", "setpc", "is_table")

    def __init__(self, i: int, text: str, idx_dst: bool, idx_src: bool):
        self.i, self.text = i, text
        parts = text.split(None, 1)
        self.mn = parts[0]
        rest = parts[1] if len(parts) > 1 else ""
        # operands: split at commas outside brackets; drop modifiers (offset:, glc, ...)
        ops, depth, cur = [], 0, ""
        for ch in rest:
            if ch in "[(":
                depth += 1
            elif ch in "])":
                depth -= 1
            if ch == "," and depth == 0:
                ops.append(cur.strip())
                cur = ""
            else:
                cur += ch
        if cur.strip():
            ops.append(cur.strip())
        if ops:
            ops[-1] = ops[-1].split()[0] if not ops[-1].startswith("%[") else ops[-1].split()[0]
        self.ops = ops
        mn = self.mn
        self.waits = 1
        m = re.fullmatch(r"s_nop", mn)
        if m and ops:
            self.waits = int(ops[0], 0) + 1
        self.valu = mn.startswith("v_")
        self.vwrites: Set[str] = set()
        self.swrites: Set[str] = set()
        self.vreads: Set[str] = set()
        self.sreads_vmem: Set[str] = set()
        self.lane_sel: Set[str] = set()
        self.store_data: Set[str] = set()
        self.trans = bool(re.match(r"v_(rcp|rsq|sqrt|exp|log|sin|cos)_", mn))
        vmem = mn.startswith(("global_", "flat_", "buffer_", "scratch_"))
        if self.valu and ops:
            if mn.startswith(("v_readlane", "v_readfirstlane")) or mn.startswith("v_cmp"):
                self.swrites |= _regs(ops[0])
                srcs = ops[1:]
            elif re.search(r"_co_|v_mad_u64_u32|v_mad_i64_i32", mn):
                self.vwrites |= _regs(ops[0])
                if len(ops) > 1:
                    self.swrites |= {r for r in _regs(ops[1]) if not r.startswith("v")}
                srcs = ops[2:]
            else:
                self.vwrites |= _regs(ops[0])
                srcs = ops[1:]
            if idx_dst:
                extra = set()
                for r in list(self.vwrites):
                    if r.startswith("v") and r[1:].isdigit():
                        extra |= {f"v{int(r[1:]) + k}" for k in range(IDX_SPAN)}
                self.vwrites |= extra
            for o in srcs:
                rr = _regs(o)
                if idx_src:
                    for r in list(rr):
                        if r.startswith("v") and r[1:].isdigit():
                            rr |= {f"v{int(r[1:]) + k}" for k in range(IDX_SPAN)}
                self.vreads |= rr
            if mn.startswith(("v_readlane", "v_writelane")) and len(ops) > 2:
                self.lane_sel = {r for r in _regs(ops[2]) if not r.startswith("v")}
        if vmem:
            for o in ops:
                self.sreads_vmem |= {r for r in _regs(o) if not r.startswith("v")}
            wide = re.search(r"store_dwordx[34]", mn)
            if wide and len(ops) > 1:
                self.store_data = _regs(ops[0] if mn.startswith("buffer_") else ops[1])
        self.uncond = mn in ("s_branch", "s_setpc_b64", "s_endpgm")
        self.target: Optional[str] = ops[0] if mn.startswith(("s_branch", "s_cbranch")) and ops else None
        self.setpc = mn == "s_setpc_b64"
        self.is_table = False


def parse(lines: List[str]) -> Tuple[List[Insn], Dict[str, int]]:
    insns: List[Insn] = []
    labels: Dict[str, int] = {}
    idx_dst = idx_src = False
    for raw in lines:
        t = raw.split(";")[0].strip()
        if not t:
            continue
        if t.endswith(":"):
            labels[t[:-1]] = len(insns)
            continue
        if t.startswith("."):  # a directive (.p2align: padding counts as no wait state)
            continue
        if t.startswith("s_set_gpr_idx_on"):
            modes = t[t.index("gpr_idx(") + 8:t.index(")", t.index("gpr_idx("))]
            idx_dst, idx_src = "DST" in modes, "SRC0" in modes or "SRC1" in modes
        ins = Insn(len(insns), t, idx_dst, idx_src)
        if t.startswith("s_set_gpr_idx_off"):
            idx_dst = idx_src = False
        insns.append(ins)
    # direct dispatch: every handler's divergent stub (`.._d_<name>`) and
    # the handler itself (`.._h_<name>`) are reached through any s_setpc_b64
    for name, k in labels.items():
        if re.search(r"_[dh]_[A-Z0-9_]+$", name) and k < len(insns):
            insns[k].is_table = True
    return insns, labels


def preds(insns: List[Insn], labels: Dict[str, int]) -> List[List[int]]:
    p: List[List[int]] = [[] for _ in insns]
    setpcs = [k for k, x in enumerate(insns) if x.setpc]
    for k, ins in enumerate(insns):
        if k + 1 < len(insns) and not ins.uncond:
            p[k + 1].append(k)
        if ins.target is not None and ins.target in labels and labels[ins.target] < len(insns):
            p[labels[ins.target]].append(k)
    for k, ins in enumerate(insns):
        if ins.is_table:
            p[k].extend(setpcs)
    return p


ENTRY = -1  # a virtual VALU writing every asm operand, before instruction 0


def check(lines: List[str]) -> List[str]:
    """Violations (text) of RULES in the block `lines`; [] when clean."""
    insns, labels = parse(lines)
    P = preds(insns, labels)
    operands: Set[str] = set()
    for ins in insns:
        for o in ins.ops:
            operands |= {r for r in _regs(o) if r.startswith("%[")}
    out: List[str] = []

    def walk(start: int, need: int, hit) -> Optional[str]:
        """Backwards from `start` over paths with fewer than `need` wait
        states in between: the first producer `hit` accepts."""
        seen: Dict[int, int] = {}
        stack = [(q, 0) for q in P[start]] + ([(ENTRY, 0)] if start == 0 or not P[start] else [])
        while stack:
            k, acc = stack.pop()
            if k == ENTRY:
                r = hit(None)
                if r:
                    return r
                continue
            if seen.get(k, 1 << 30) <= acc:
                continue
            seen[k] = acc
            r = hit(insns[k])
            if r:
                return f"{r} at #{k} `{insns[k].text}`"
            acc2 = acc + insns[k].waits
            if acc2 < need:
                stack.extend((q, acc2) for q in P[k])
                if k == 0 or not P[k]:
                    stack.append((ENTRY, acc2))
        return None

    for c, ins in enumerate(insns):
        if ins.valu and ins.vwrites:
            w = ins.vwrites
            r = walk(c, RULES["store-data"],
                     lambda x: x is not None and x.store_data & w and "store-data: wide store")
            if r:
                out.append(f"store-data: #{c} `{ins.text}` rewrites data of {r}")
        if ins.sreads_vmem:
            s = ins.sreads_vmem
            r = walk(c, RULES["sgpr-vmem"],
                     lambda x: ("sgpr-vmem: asm entry" if x is None and s & operands else
                                x is not None and x.valu and x.swrites & s and "sgpr-vmem: VALU SGPR write"))
            if r:
                out.append(f"sgpr-vmem: #{c} `{ins.text}` reads an SGPR of {r}")
        if ins.lane_sel:
            s = ins.lane_sel
            r = walk(c, RULES["sgpr-lane"],
                     lambda x: ("sgpr-lane: asm entry" if x is None and s & operands else
                                x is not None and x.valu and x.swrites & s and "sgpr-lane: VALU SGPR write"))
            if r:
                out.append(f"sgpr-lane: #{c} `{ins.text}` lane select from {r}")
        if ins.valu and ins.vreads:
            v = ins.vreads
            r = walk(c, RULES["trans"], lambda x: x is not None and x.trans and x.vwrites & v and "trans op")
            if r:
                out.append(f"trans: #{c} `{ins.text}` reads the result of {r}")
    # the block's end: the compiler's code after it may read any operand by VMEM
    ends = [k for k, x in enumerate(insns) if k == len(insns) - 1]
    for e in ends:
        need = RULES["sgpr-vmem"]
        acc, k = 0, e
        stack = [(e, 0)]
        seen: Dict[int, int] = {}
        while stack:
            k, acc = stack.pop()
            if seen.get(k, 1 << 30) <= acc:
                continue
            seen[k] = acc
            x = insns[k]
            if x.valu and x.swrites & operands:
                out.append(f"sgpr-vmem: block end within {acc} wait states of `{x.text}` (#{k})")
            if acc + x.waits < need:
                stack.extend((q, acc + x.waits) for q in P[k])
    return out

"""Programs for the bpf_tail_call / PROG_ARRAY parity tests (the builders
live in bpftime_amd/programs.py).  Semantics under test
(runtime/src/bpf_helper.cpp:568-650, the interpreter backend): the target
runs as a nested exec over a 64-B copy of the ctx (r2 = 64), its r0 comes
back to the caller as the helper's result, the caller's registers, stack and
ctx are unchanged, packet bytes written through ctx->data stay written, a
missing slot / non-prog-array map returns -1, and depth stops at 32."""
from bpftime_amd import isa
from bpftime_amd.programs import (tail_ref_kat_caller as ref_kat_caller,  # noqa: F401
                                  tail_ref_kat_target as ref_kat_target, tail_target_count as target_count,
                                  tail_target_recurse as target_recurse, tail_target_write as target_write,
                                  tail_xdp_caller as xdp_caller)

TAIL = isa.BPF_FUNC_tail_call

"""The wait-state check of the hand-written fast path (bpftime_amd/csrc/
hazards.py, run by gen_fast.py and `make`): the committed fast_asm.inc is
clean, and each rule fires on a seeded violation -- including the round-3
miss-log bug (a global_store_dwordx4 whose data VGPR the next instruction
rewrote, fixed with s_nop 1)."""
import os
import subprocess
import sys

import pytest

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bpftime_amd", "csrc")
sys.path.insert(0, CSRC)

import gen_fast  # noqa: E402
import hazards  # noqa: E402


def test_committed_fast_path_is_clean():
    r = subprocess.run([sys.executable, os.path.join(CSRC, "gen_fast.py"), "--check"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    blocks = gen_fast.inc_blocks(os.path.join(CSRC, "fast_asm.inc"))
    assert sorted(blocks) == ["BPFTIME_AMD_FAST_ASM", "BPFTIME_AMD_FAST_ASM_G"]
    for lines in blocks.values():
        assert len(lines) > 10000 and hazards.check(lines) == []


def test_generator_output_matches_the_committed_file():
    for greg, name in ((False, "BPFTIME_AMD_FAST_ASM"), (True, "BPFTIME_AMD_FAST_ASM_G")):
        g = gen_fast.Gen(greg)
        g.build()
        assert [gen_fast.relocate(x) for x in g.out] == gen_fast.inc_blocks(os.path.join(CSRC, "fast_asm.inc"))[name]


def test_miss_log_store_without_its_nop_is_flagged():
    g = gen_fast.Gen(False)
    g.build()
    seeded = [l for i, l in enumerate(g.out)
              if not (l.strip().startswith("s_nop") and i and "store_dwordx4" in g.out[i - 1])]
    assert len(seeded) < len(g.out)
    bad = hazards.check(seeded)
    assert bad and all(b.startswith("store-data:") for b in bad)
    assert any("global_store_dwordx4 v42, v[56:59]" in b for b in bad)
    with pytest.raises(SystemExit, match="wait-state hazards"):
        gen_fast.check_hazards({"seeded": seeded})


@pytest.mark.parametrize("lines,rule", [
    (["global_store_dwordx4 v42, v[56:59], s[52:53]", "v_mov_b32 v57, 0"], "store-data"),
    (["flat_store_dwordx4 v[48:49], v[84:87]", "s_cbranch_scc1 .Lx", ".Lx:", "v_mov_b32 v85, 0"], None),
    (["global_store_dwordx4 v42, v[56:59], off", "s_cbranch_scc1 .Lx", "s_nop 0", ".Lx:",
      "v_add_u32 v59, 1, v59"], None),
    (["global_store_dwordx2 v42, v[56:57], off", "v_mov_b32 v56, 0"], None),          # 64 bits: no hazard
    (["s_set_gpr_idx_on s44, gpr_idx(DST)", "global_store_dwordx4 v42, v[62:65], off",
      "v_mov_b32 v60, v44", "s_set_gpr_idx_off"], "store-data"),                      # index mode reaches v63
    (["v_readfirstlane_b32 s52, v41", "s_nop 2", "global_load_dword v42, v41, s[52:53]"], "sgpr-vmem"),
    (["v_readfirstlane_b32 s52, v41", "s_nop 4", "global_load_dword v42, v41, s[52:53]"], None),
    (["v_cmp_eq_u32_e64 s[54:55], v41, 0", "global_atomic_add v41, v42, s[54:55]"], "sgpr-vmem"),
    (["v_readfirstlane_b32 s69, v41", "v_readlane_b32 s70, v42, s69"], "sgpr-lane"),
    # alignment padding may be empty: a directive counts as no wait state
    (["global_store_dwordx4 v42, v[56:59], off", ".p2align 6", ".Lh:", "v_mov_b32 v57, 0"], "store-data"),
    (["v_readfirstlane_b32 s52, v41", "s_nop 3", ".p2align 6", "global_load_dword v42, v41, s[52:53]"],
     "sgpr-vmem"),
    (["v_readfirstlane_b32 s69, v41", "s_nop 3", "v_readlane_b32 s70, v42, s69"], None),
    (["v_rcp_f64 v[44:45], v[46:47]", "v_mul_f64 v[48:49], v[44:45], v[50:51]"], "trans"),
    (["v_rcp_f64 v[44:45], v[46:47]", "s_nop 0", "v_mul_f64 v[48:49], v[44:45], v[50:51]"], None),
    (["global_load_dword v42, v41, %[maps]"], "sgpr-vmem"),                            # an operand at block entry
    (["s_nop 4", "global_load_dword v42, v41, %[maps]"], None),
    (["s_mov_b32 s52, 0", "v_readfirstlane_b32 %[why], v41"], "sgpr-vmem"),             # an operand at block end
])
def test_each_rule(lines, rule):
    bad = hazards.check(lines)
    if rule is None:
        assert bad == [], bad
    else:
        assert bad and all(b.startswith(rule + ":") for b in bad), bad

"""The device LPM flat table (maps.cpp LpmTrie::flat, the DIR-24-8 form of
an IPv4 trie that device lookups of full-length keys take) against the trie
walk it replaces (LpmTrie::lookup, lpm_trie_map.cpp:192-264), host-only:
random route sets with stray bits beyond the prefix, logical deletions
(including /32s, which the walk then reports as absent rather than falling
back to a covering prefix), every route's ends and neighbours, random
addresses and every address of sampled /24s (tests/cpp/lpm_flat_test.cpp)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bpftime_amd", "lib", "lpm_flat_test")


def test_flat_table_matches_the_trie_walk():
    out = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.strip().endswith("OK")

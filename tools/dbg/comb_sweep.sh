set -e
for e in auto 2048 4096; do echo "comb $e"; if [ $e = auto ]; then timeout -k 10 120 python tools/dbg/micro_hash.py 2>&1 | grep full; else BPFTIME_AMD_COMB_ENTRIES=$e timeout -k 10 120 python tools/dbg/micro_hash.py 2>&1 | grep full; fi; done

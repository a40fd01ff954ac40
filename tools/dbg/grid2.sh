set -e
for m in 1 2 4; do echo "mult $m"; BPFTIME_AMD_GRID_MULT=$m timeout -k 10 120 python tools/dbg/micro_hash.py 2>&1 | grep full; done

set -e
for m in 1 2 4 8; do echo "mult $m"; BPFTIME_AMD_GRID_MULT=$m timeout -k 10 100 python tools/dbg/micro.py 2>&1 | grep -E "exit only|ld\+st|xdp-counter"; done

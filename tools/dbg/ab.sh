set -e
for m in 1 4; do echo "mult $m"; BPFTIME_AMD_GRID_MULT=$m timeout -k 10 100 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_avg_ms'])"; BPFTIME_AMD_GRID_MULT=$m timeout -k 10 100 python tools/dbg/micro.py 2>&1 | grep xdp-counter; done

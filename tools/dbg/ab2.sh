set -e
for w in 3 50 500; do echo "warmup $w"; timeout -k 10 100 python bench.py --steps 20 --warmup $w --no-cpu-baseline --no-e2e 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_avg_ms'])"; done

set -e
for st in 2 3 4; do for c in 18 20; do echo "streams $st chunk 2^$c"; timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --e2e-streams $st --e2e-chunk-log2 $c 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['e2e']; print(e['verdicts_out'], e['frames_and_verdicts_out'], e['ok'])"; done; done

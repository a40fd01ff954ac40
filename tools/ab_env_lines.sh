# A/B of an environment switch over bench lines on one box, alternating:
#   VAR=BPFTIME_AMD_LANE_PAD VALS="1 0" WL="tail-call flow-hash" REPS=2 bash tools/ab_env_lines.sh
set -o pipefail
mkdir -p gpurun_out
for r in $(seq 1 ${REPS:-2}); do
  for w in $WL; do
    for v in $VALS; do
      if [ "$w" = xdp-counter ]; then A="--no-cpu-baseline --no-e2e"; else A="--workload $w --no-cpu-baseline"; fi
      env $VAR=$v timeout -k 10 200 python bench.py $A > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
      python -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('$w $VAR=$v', d['value'], d['roofline']['kernel_avg_ms'], d['parity'].get('ok'), flush=True)"
    done
  done
done

#!/bin/bash
# A/B timing of library builds under ab/: bash tools/experiments/ab.sh variant... (workloads via WL)
set -u
mkdir -p gpurun_out
WL=${WL:-"main flow-hash tail-call"}
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in "$@"; do
    for w in $WL; do
      if [ "$w" = main ]; then args="--steps ${MAIN_STEPS:-20} --warmup 5"; else args="--workload $w --steps 10 --warmup 3"; fi
      BPFTIME_AMD_LIB=$PWD/ab/$v.so timeout -k 10 300 python bench.py $args --no-cpu-baseline > gpurun_out/ab_${v}_$w.json 2> gpurun_out/ab_${v}_$w.err || { echo "FAIL $v $w"; tail -3 gpurun_out/ab_${v}_$w.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/ab_${v}_$w.json'));print('$round $v $w',d['value'],d['ms_per_step'],(d.get('parity') or {}).get('ok', d.get('parity')))"
    done
  done
done

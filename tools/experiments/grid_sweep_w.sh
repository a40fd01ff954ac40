#!/bin/bash
# One bench workload per grid multiplier (BPFTIME_AMD_GRID_MULT):
#   bash tools/experiments/grid_sweep_w.sh <workload> "<mults...>"
set -u
mkdir -p gpurun_out
w=$1
for m in $2; do
  BPFTIME_AMD_GRID_MULT=$m timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/gsw_${w}_$m.json 2> gpurun_out/gsw_${w}_$m.err || { tail -3 gpurun_out/gsw_${w}_$m.err; exit 1; }
  python3 -c "import json;a=json.load(open('gpurun_out/gsw_${w}_$m.json'));print('$w mult $m', a['ms_per_step'], a['value'], a['parity'].get('ok'))"
done

#!/bin/bash
# Headline kernel time per grid multiplier (BPFTIME_AMD_GRID_MULT; resident blocks x mult):
#   bash tools/experiments/grid_sweep.sh "<mults...>"
set -u
mkdir -p gpurun_out
for m in $1; do
  BPFTIME_AMD_GRID_MULT=$m timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-e2e > gpurun_out/gs_$m.json 2> gpurun_out/gs_$m.err || { tail -3 gpurun_out/gs_$m.err; exit 1; }
  python3 -c "import json;a=json.load(open('gpurun_out/gs_$m.json'));print('mult $m', a['ms_per_step'], a['value'], a['roofline']['achieved'])"
done

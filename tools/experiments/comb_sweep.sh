#!/bin/bash
# Kernel time of one workload per combining-table size (BPFTIME_AMD_COMB_ENTRIES; "auto": the library's choice):
#   bash tools/experiments/comb_sweep.sh <workload> "<entries...>" [extra env]
set -u
mkdir -p gpurun_out
w=$1
for e in $2; do
  ce="BPFTIME_AMD_COMB_ENTRIES=$e"; [ "$e" = auto ] && ce="X=1"
  env ${3:-} $ce BPFTIME_AMD_VERBOSE=1 timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 20 > gpurun_out/cs_${w}_$e.json 2> gpurun_out/cs_${w}_$e.err || { tail -3 gpurun_out/cs_${w}_$e.err; exit 1; }
  python3 -c "import json;a=json.load(open('gpurun_out/cs_${w}_$e.json'));print('$w comb $e', a['ms_per_step'], a['parity']['ok'])"
  tail -1 gpurun_out/cs_${w}_$e.err
done

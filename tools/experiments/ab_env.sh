#!/bin/bash
# one build, several environments: bash tools/experiments/ab_env.sh build workload "ENV1" "ENV2" ...
set -u
v=$1; w=$2; shift 2
for round in 1 2; do
  for e in "$@"; do
    env $e BPFTIME_AMD_LIB=$PWD/ab/$v.so timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abe.json 2> gpurun_out/abe.err || { tail -3 gpurun_out/abe.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abe.json'));print('$round', '$e', '$w', d['value'], d['ms_per_step'])"
  done
done

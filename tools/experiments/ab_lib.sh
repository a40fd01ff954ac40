#!/bin/bash
# Same-box A/B of two builds of libbpftime_amd.so, alternating, every bench
# line without CPU legs:  tools/experiments/ab_lib.sh <tag> <lib A> <lib B>
# (a path "default" = the in-tree library)
set -o pipefail
TAG=${1:?tag}; A=${2:?lib A}; B=${3:?lib B}
mkdir -p gpurun_out
OUT=gpurun_out/ab_$TAG.txt
: > $OUT
for rep in 1 2; do
  for lib in "$A" "$B"; do
    for w in xdp-counter flow-hash syscall-agg syscount tail-call syscount-latency; do
      if [ "$lib" = default ]; then unset BPFTIME_AMD_LIB; else export BPFTIME_AMD_LIB=$PWD/$lib; fi
      timeout -k 10 120 python bench.py --workload $w --no-cpu-baseline --no-e2e > gpurun_out/ab_line.json 2> gpurun_out/ab_line.err || { echo "FAIL $lib $w" >> $OUT; tail -5 gpurun_out/ab_line.err >> $OUT; exit 1; }
      python3 -c "import json;d=json.loads(open('gpurun_out/ab_line.json').read().strip().splitlines()[-1]);print('$rep $lib $w', d['value'], d['ms_per_step'], d['roofline'].get('kernel_avg_ms'), d.get('parity',{}).get('ok'))" >> $OUT
    done
  done
done
unset BPFTIME_AMD_LIB
cat $OUT

#!/bin/bash
# A/B of the dispatch table's branch hop (gen_fast.py BPFTIME_AMD_EXTRA_HOP, at commit aabfa90:
# the knob went with the table when dispatch became direct, 54c3d9e):
# the default library against one built with a second branch per dispatch
# (bpftime_amd/lib_hop), alternating, every line without CPU legs.
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/ab_hop.txt
: > $OUT
for rep in 1 2; do
  for lib in default hop; do
    for w in xdp-counter flow-hash syscall-agg syscount tail-call syscount-latency; do
      if [ $lib = hop ]; then export BPFTIME_AMD_LIB=$PWD/bpftime_amd/lib_hop/libbpftime_amd.so; else unset BPFTIME_AMD_LIB; fi
      timeout -k 10 120 python bench.py --workload $w --no-cpu-baseline --no-e2e > gpurun_out/ab_line.json 2> gpurun_out/ab_line.err || { echo "FAIL $lib $w" >> $OUT; tail -5 gpurun_out/ab_line.err >> $OUT; exit 1; }
      python3 -c "import json;d=json.loads(open('gpurun_out/ab_line.json').read().strip().splitlines()[-1]);print('$rep $lib $w', d['value'], d['ms_per_step'], d['roofline'].get('kernel_avg_ms'), d.get('parity',{}).get('ok'))" >> $OUT
    done
  done
done
unset BPFTIME_AMD_LIB
cat $OUT

#!/bin/bash
# PMC + kernel-trace passes of every bench line (tools/prof_workload.sh), their
# JSON summaries copied to gpurun_out/pmc_<workload>.json for profiles/.
set -u
TAG=${1:-r02}
for w in ${WS:-xdp-counter flow-hash syscall-agg syscount tail-call lpm-route ringbuf-sample}; do
  u=16777216
  case $w in syscall-agg|syscount) u=33554432;; esac
  UNITS=$u bash tools/prof_workload.sh $w $TAG > gpurun_out/prof_${TAG}_$w.out 2>&1 || { echo "FAIL $w"; tail -5 gpurun_out/prof_${TAG}_$w.out; exit 1; }
  cp gpurun_out/prof_${TAG}_$w.pmc.json gpurun_out/pmc_$w.json
  grep -E "kernel avg ms|HBM" gpurun_out/prof_${TAG}_$w.out | sed "s/^/$w: /"
done

#!/bin/bash
# round 3 (second part): kernel-trace + PMC passes of bench lines
# (tools/prof_workload.sh), summaries to gpurun_out/ for profiles/r03b_pmc/
#   bash tools/r03b_prof.sh workload...
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in "$@"; do
  u=16777216
  [ "$w" = syscall-agg ] && u=33554432
  UNITS=$u bash tools/prof_workload.sh $w r03b > gpurun_out/prof_r03b_$w.out 2>&1 || { echo "FAIL $w"; tail -5 gpurun_out/prof_r03b_$w.out; exit 1; }
  cp gpurun_out/prof_r03b_$w.pmc.json gpurun_out/pmc_$w.json
  grep -E "kernel avg ms|HBM" gpurun_out/prof_r03b_$w.out | sed "s/^/$w: /"
done

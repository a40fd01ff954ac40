#!/bin/bash
# round 3 (second part): kernel-trace + PMC passes of every bench line
# (tools/prof_all.sh), summaries to gpurun_out/ for profiles/r03b_pmc/
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/prof_all.sh r03b || exit 1

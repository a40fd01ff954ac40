#!/bin/bash
# round 3 end: PMC passes of the lines the last changes moved, then every
# bench line with its CPU baseline (bench traffic from the refreshed passes)
set -o pipefail
export TMPDIR=/tmp
bash tools/r03b_prof.sh syscall-agg tail-call flow-hash || exit 1
for w in syscall-agg tail-call flow-hash; do cp gpurun_out/pmc_$w.json profiles/pmc_$w.json; done
bash tools/bench_all.sh || exit 1

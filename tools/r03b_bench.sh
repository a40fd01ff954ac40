#!/bin/bash
# round 3 (second part): every bench line with its CPU baseline
set -o pipefail
export TMPDIR=/tmp
bash tools/bench_all.sh || exit 1

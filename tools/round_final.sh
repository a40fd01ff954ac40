#!/bin/bash
# A round's final measurement: PMC + kernel-trace passes of every bench line
# (tools/prof_all.sh -> gpurun_out/<tag>_pmc/, gpurun_out/pmc_<w>.json), then
# every bench line with its CPU baseline, reading the refreshed traffic
# (gpurun_out/<tag>_bench_lines.jsonl).  Copy what is judged into profiles/.
#   tools/round_final.sh <tag>
set -o pipefail
TAG=${1:?tag}
export TMPDIR=/tmp
WS=${WS:-"xdp-counter flow-hash syscall-agg syscount tail-call lpm-route ringbuf-sample"}
mkdir -p gpurun_out/${TAG}_pmc
WS="$WS" bash tools/prof_all.sh $TAG || exit 1
for w in $WS; do
  cp gpurun_out/pmc_$w.json profiles/pmc_$w.json
  cp gpurun_out/prof_${TAG}_$w.summary.txt gpurun_out/${TAG}_pmc/$w.txt
  cp gpurun_out/prof_${TAG}_$w/kt_kernel_stats.csv gpurun_out/${TAG}_pmc/${w}_kernel_stats.csv 2>/dev/null || true
done
[ -n "${NO_BENCH:-}" ] && exit 0
bash tools/bench_all.sh || exit 1
for w in $WS syscount-latency; do cat gpurun_out/bench_$w.json; done > gpurun_out/${TAG}_bench_lines.jsonl

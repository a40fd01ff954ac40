#!/bin/bash
# round 4 (final) measurement: PMC + kernel-trace passes of every bench line
# (profiles/r04f_pmc, profiles/pmc_<w>.json), then every bench line with its
# CPU baseline, reading the refreshed traffic (profiles/r04f_bench_lines.jsonl)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04f_pmc
bash tools/prof_all.sh r04f || exit 1
for w in xdp-counter flow-hash syscall-agg tail-call lpm-route ringbuf-sample; do
  cp gpurun_out/pmc_$w.json profiles/pmc_$w.json
  cp gpurun_out/prof_r04f_$w.summary.txt gpurun_out/r04f_pmc/$w.txt
  cp gpurun_out/prof_r04f_$w/kt_kernel_stats.csv gpurun_out/r04f_pmc/${w}_kernel_stats.csv 2>/dev/null || true
done
bash tools/bench_all.sh || exit 1
cat gpurun_out/bench_xdp-counter.json gpurun_out/bench_flow-hash.json gpurun_out/bench_syscall-agg.json gpurun_out/bench_tail-call.json gpurun_out/bench_lpm-route.json gpurun_out/bench_ringbuf-sample.json > gpurun_out/r04f_bench_lines.jsonl

#!/bin/bash
# Every bench line once (the headline with its CPU baseline and e2e leg), JSON
# lines to gpurun_out/bench_<workload>.json
set -u
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_xdp-counter.json 2> gpurun_out/bench_xdp-counter.err || { tail gpurun_out/bench_xdp-counter.err; exit 1; }
for w in flow-hash syscall-agg syscount syscount-latency tail-call lpm-route ringbuf-sample; do
  timeout -k 10 400 python bench.py --workload $w > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { tail gpurun_out/bench_$w.err; exit 1; }
done
for w in xdp-counter flow-hash syscall-agg syscount syscount-latency tail-call lpm-route ringbuf-sample; do
  python3 -c "import json;d=json.load(open('gpurun_out/bench_$w.json'));r=d['roofline'];c=d.get('cpu_baseline') or {};print('$w', d['value'], d['unit'], d['ms_per_step'], 'frac', r['frac'], 'traffic', r['traffic'], 'cpu', c.get('value'), c.get('cores'), 'parity', d.get('parity', d.get('checks')))"
done

#!/bin/bash
# GPU suite, then same-box A/B of 1024-lane blocks (default for G launches)
# against 256-lane blocks (BPFTIME_AMD_BLOCK=256) on the table workloads
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/blk_pytest.log 2>&1 || { tail -30 gpurun_out/blk_pytest.log; exit 1; }
tail -2 gpurun_out/blk_pytest.log
for round in 1 2; do
  for bs in 1024 256; do
    for w in ${WL:-flow-hash syscall-agg}; do
      BPFTIME_AMD_BLOCK=$bs timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/blk_${bs}_$w.json 2> gpurun_out/blk_${bs}_$w.err || { tail gpurun_out/blk_${bs}_$w.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/blk_${bs}_$w.json'));print('$round $bs $w',d['value'],d['ms_per_step'],d['roofline']['achieved'] if d.get('roofline') else '', (d.get('parity') or {}).get('ok', d.get('parity')))"
    done
  done
done

#!/bin/bash
# round-4 experiment batch: 8-KiB ring staging at grid x1 (in-tree), GPU
# suite, ring line A/B
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_suite.txt 2>&1 &&
WL="ringbuf-sample main" ROUNDS=2 timeout -k 10 300 bash tools/ab.sh pop1 rb8k1 > gpurun_out/ab_rb.txt 2>&1

#!/bin/bash
# round-4 experiment batch: lane groups through the asm tier for XDP G launches
set -u
mkdir -p gpurun_out
WL="main flow-hash syscall-agg tail-call" ROUNDS=2 timeout -k 10 600 bash tools/ab.sh base grpX > gpurun_out/ab_grp.txt 2>&1 &&
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_suite.txt 2>&1

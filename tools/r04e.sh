#!/bin/bash
# round-4 experiment batch: the kernel prologue's divisions computed on the
# host (in-tree), GPU suite, A/B
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_suite.txt 2>&1 &&
WL="main flow-hash syscall-agg tail-call" MAIN_STEPS=200 ROUNDS=2 timeout -k 10 400 bash tools/ab.sh cur hdiv > gpurun_out/ab_hdiv.txt 2>&1

#!/bin/bash
# round-4 experiment batch: tail-call pops restore their first ctx and stack
# words with the registers (one round trip); tail-call tests, A/B
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_tailcall.py tests/test_oracle_tailcall.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tail_tests.txt 2>&1 &&
WL="tail-call main" ROUNDS=3 timeout -k 10 400 bash tools/ab.sh grpX pop1 > gpurun_out/ab_pop.txt 2>&1

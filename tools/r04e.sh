#!/bin/bash
# round-4 experiment batch: bpf_ringbuf_output in the asm tier (staged
# path), ring tests, A/B, then the GPU suite
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ringbuf.py -x -v --timeout 120 --timeout-method thread > gpurun_out/rb_tests.txt 2>&1 &&
WL="ringbuf-sample main" ROUNDS=2 timeout -k 10 300 bash tools/ab.sh cur rbasm > gpurun_out/ab_rbasm.txt 2>&1 &&
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_suite.txt 2>&1

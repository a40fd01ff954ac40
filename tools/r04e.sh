#!/bin/bash
# round-4 experiment batch: tail-call images at 5 waves per SIMD (asm block
# at v34-v95), with the combining table at 512 / 256 entries
set -u
mkdir -p gpurun_out
timeout -k 10 300 bash tools/ab_env_k.sh w5 tail-call "X=1" "BPFTIME_AMD_COMB_ENTRIES=256" > gpurun_out/ab_w5_tail.txt 2>&1
WL="main flow-hash syscall-agg" ROUNDS=1 timeout -k 10 300 bash tools/ab.sh cur w5 > gpurun_out/ab_w5.txt 2>&1
BPFTIME_AMD_LIB=$PWD/ab/w5.so timeout -k 10 300 python -u -m pytest tests/test_gpu_tailcall.py -x -q --timeout 120 --timeout-method thread > gpurun_out/w5_tail_tests.txt 2>&1

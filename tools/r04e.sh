#!/bin/bash
# round-4 experiment batch: insert-path counters of the cold flow table
# (reserved entries passed; + empty entries confirmed coherently in asm), A/B
set -u
mkdir -p gpurun_out
BPFTIME_AMD_LIB=$PWD/ab/istats_ixres.so timeout -k 10 200 python tools/insert_stats.py > gpurun_out/istats_ixres.txt 2>&1 &&
BPFTIME_AMD_LIB=$PWD/ab/istats_ixc.so timeout -k 10 200 python tools/insert_stats.py > gpurun_out/istats_ixc.txt 2>&1 &&
WL="flow-hash syscall-agg" ROUNDS=2 timeout -k 10 400 bash tools/ab.sh base ixres ixc > gpurun_out/ab_ixc.txt 2>&1

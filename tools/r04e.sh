#!/bin/bash
# round-4 experiment batch: insert-path counters of the cold flow table
# (one-word and eight-word bitmap scans), next-unit prefetch / scan A/B,
# dispatch-count sensitivity (pair fusion off)
set -u
mkdir -p gpurun_out
BPFTIME_AMD_LIB=$PWD/ab/istats.so timeout -k 10 200 python tools/insert_stats.py > gpurun_out/istats.txt 2>&1 &&
BPFTIME_AMD_LIB=$PWD/ab/istats8.so timeout -k 10 200 python tools/insert_stats.py > gpurun_out/istats8.txt 2>&1 &&
WL="main flow-hash syscall-agg tail-call lpm-route" MAIN_STEPS=200 ROUNDS=2 timeout -k 10 600 bash tools/ab.sh base pf scan8 > gpurun_out/ab_pf.txt 2>&1 &&
timeout -k 10 300 bash tools/ab_env.sh pf flow-hash "X=1" "BPFTIME_AMD_NO_FUSE=1" > gpurun_out/ab_fuse.txt 2>&1

#!/bin/bash
# rocprofv3 passes for the headline bench (kernel-trace stats, then separate
# PMC passes as MI355X_MICROARCH.md §rocprofv3 prescribes).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o kt -- python3 bench.py $ARGS > gpurun_out/prof_${TAG}_kt.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/prof_$TAG -o sq -- python3 bench.py $ARGS > gpurun_out/prof_${TAG}_sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_$TAG -o fetch -- python3 bench.py $ARGS > gpurun_out/prof_${TAG}_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_$TAG -o write -- python3 bench.py $ARGS > gpurun_out/prof_${TAG}_write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_FLAT SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof_$TAG -o sq2 -- python3 bench.py $ARGS > gpurun_out/prof_${TAG}_sq2.log 2>&1 || exit $?
find gpurun_out/prof_$TAG -type f | head -40

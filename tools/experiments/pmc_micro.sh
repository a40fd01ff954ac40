#!/bin/bash
# PMC passes of one tools/experiments/micro.py flow variant per library build:
#   tools/experiments/pmc_micro.sh "<lib1> <lib2>" <variant>      (ab/<lib>.so)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in $1; do
  D=gpurun_out/pmcm_$v
  mkdir -p $D
  i=0
  for c in "SQ_INSTS_LDS SQ_INSTS_LDS_ATOMIC SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU" \
           "TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_BUSY_CYCLES"; do
    i=$((i+1))
    BPFTIME_AMD_LIB=$PWD/ab/$v.so MICRO_FLOW=1 MICRO_ONLY=$2 timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $D -o p$i -- python3 tools/experiments/micro.py > $D.p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -3 $D.p$i.log; exit 1; }
  done
  python3 tools/pmc_table.py $D 16777216 | tail -25
done

#!/bin/bash
# rocprofv3 passes for one bench workload: kernel-trace stats, then separate
# PMC passes (MI355X_MICROARCH.md §rocprofv3: one block budget per pass).
#   tools/prof_workload.sh <workload> <tag> [extra bench args]
set -u
W=${1:-flow-hash}
TAG=${2:-r02}
shift 2 || true
EXTRA="$*"
mkdir -p gpurun_out
export TMPDIR=/tmp
D=gpurun_out/prof_${TAG}_${W}
if [ "$W" = xdp-counter ]; then  # the headline bench line
  ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-e2e $EXTRA"
else
  ARGS="--workload $W --steps 3 --warmup 1 --no-cpu-baseline $EXTRA"
fi
run() {  # name, counters...
  local name=$1; shift
  if [ "$name" = kt ]; then
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o kt -- python3 bench.py $ARGS > $D.kt.log 2>&1
  else
    timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $D -o $name -- python3 bench.py $ARGS > $D.$name.log 2>&1
  fi
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
mkdir -p $D
# PASSES (default all): a subset, e.g. PASSES="kt sq1 sq2"
P=" ${PASSES:-kt sq1 sq2 fetch write l2 tcp} "
on() { [[ "$P" == *" $1 "* ]]; }
if on kt; then run kt || exit $?; fi
if on sq1; then run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || exit $?; fi
if on sq2; then run sq2 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAVES || exit $?; fi
if on fetch; then run fetch FETCH_SIZE || exit $?; fi
if on write; then run write WRITE_SIZE || exit $?; fi
if on l2; then run l2 TCC_HIT_sum TCC_MISS_sum || exit $?; fi
if on tcp; then run tcp TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum || true; fi
U=${UNITS:-16777216}
python3 tools/pmc_table.py $D $U $D.pmc.json > $D.summary.txt 2>&1 || true
cat $D.summary.txt

#!/bin/bash
# GPU-box check: parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash / fault / timeout ends the
# script (exit codes other than 0 and pytest's 1 = "tests failed").
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  return $rc
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  step pytest_gpu 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider
  rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 600 python bench.py --steps 10 --warmup 2 --cpu-seconds 8 || exit $?
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- \
      python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline || exit $?
  find gpurun_out/prof -name "*stats*" | head -20
fi
exit 0

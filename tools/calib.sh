#!/bin/bash
# PMC calibration passes over tools/sol/calib (known byte counts per access
# shape): timings, a kernel trace, then FETCH_SIZE, WRITE_SIZE and TCC
# hit/miss in passes of their own (MI355X_MICROARCH.md rocprofv3 budgets).
#   tools/calib.sh <tag>      -> gpurun_out/calib_<tag>/, summary via tools/calib_table.py
set -u
TAG=${1:-r03}
export TMPDIR=/tmp
D=gpurun_out/calib_$TAG
mkdir -p $D
B=tools/sol/calib
[ -x $B ] || { echo "build $B first (hipcc -O3 --offload-arch=gfx950 -o $B tools/sol/calib.hip)"; exit 1; }
timeout -k 10 120 $B > $D/plain.jsonl || exit $?
echo "plain rc=0"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o kt -- $B > $D/kt.log 2>&1 || exit $?
echo "kt rc=0"
for pass in "fetch FETCH_SIZE" "write WRITE_SIZE" "tcc TCC_HIT_sum TCC_MISS_sum"; do
  set -- $pass
  name=$1; shift
  timeout -s KILL 180 rocprofv3 --pmc "$@" --output-format csv -d $D -o $name -- $B > $D/$name.log 2>&1 || exit $?
  echo "$name rc=0"
done
python3 tools/calib_table.py $D

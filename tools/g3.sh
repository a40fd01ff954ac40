set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/g3_pytest.log 2>&1 || { tail -40 gpurun_out/g3_pytest.log; exit 1; }
tail -2 gpurun_out/g3_pytest.log
cp bpftime_amd/lib/libbpftime_amd.so ab/new.so
WL="flow-hash syscall-agg" bash tools/ab.sh cur new || exit 1
LOG2N=24 timeout -k 10 200 python tools/micro_dbg/micro_hash.py flow || exit 1

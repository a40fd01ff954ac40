set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/g11_pytest.log 2>&1 || { tail -30 gpurun_out/g11_pytest.log; exit 1; }
tail -1 gpurun_out/g11_pytest.log
WL="main flow-hash syscall-agg" bash tools/ab.sh head || exit 1

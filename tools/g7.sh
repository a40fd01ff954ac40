set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_ringbuf.py > gpurun_out/g7_pytest.log 2>&1 || { tail -40 gpurun_out/g7_pytest.log; exit 1; }
tail -1 gpurun_out/g7_pytest.log
WL="ringbuf-sample" bash tools/ab.sh base head v1 || exit 1

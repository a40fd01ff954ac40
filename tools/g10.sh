set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_tailcall.py tests/test_gpu_chain.py tests/test_unwind.py > gpurun_out/g10_pytest.log 2>&1 || { tail -30 gpurun_out/g10_pytest.log; exit 1; }
tail -1 gpurun_out/g10_pytest.log
WL="tail-call" bash tools/ab.sh base head || exit 1

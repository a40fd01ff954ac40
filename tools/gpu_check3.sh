set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tailcall.py > gpurun_out/gpu_tail.log 2>&1 || { tail -30 gpurun_out/gpu_tail.log; exit 1; }
tail -2 gpurun_out/gpu_tail.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/gpu_all.log 2>&1 || { tail -30 gpurun_out/gpu_all.log; exit 1; }
tail -2 gpurun_out/gpu_all.log
WL="main tail-call" bash tools/ab.sh head v6 v9

# GPU suite, then the micro model, then A/B of builds: bash tools/gpu_ab.sh "v1 v2" "wl1 wl2"
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/gpu_all.log 2>&1 || { tail -30 gpurun_out/gpu_all.log; exit 1; }
tail -2 gpurun_out/gpu_all.log
timeout -k 10 200 python tools/micro.py || exit 1
bash tools/ab_cmp.sh "$1" "$2"

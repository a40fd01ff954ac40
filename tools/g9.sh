set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/kt9
timeout -k 10 120 python -u -m pytest -x -q --timeout 60 --timeout-method thread -m gpu tests/test_gpu_maps.py -k "miss_log or flow_hash_parity" > gpurun_out/g9_pytest.log 2>&1 || { tail -30 gpurun_out/g9_pytest.log; exit 1; }
tail -1 gpurun_out/g9_pytest.log
bash tools/ab_env.sh head flow-hash X=0 BPFTIME_AMD_NO_MISS_LOG=1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt9 -o kt -- python3 bench.py --workload flow-hash --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/kt9.log 2>&1 || exit 1
cat gpurun_out/kt9/kt_kernel_stats.csv | cut -d, -f1-6 | head

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_shm_json_perf.py tests/test_shm_json.py tests/test_gpu_sysbpf.py tests/test_gpu_syscall_dispatch.py "tests/test_gpu_maps.py::test_ctx_stack_lookup_fits_cu" > gpurun_out/gj.log 2>&1; rc=$?; tail -30 gpurun_out/gj.log; exit $rc

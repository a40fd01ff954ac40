# round-3 GPU check: the new / changed tests first (verbose), then the whole GPU suite
set -o pipefail
mkdir -p gpurun_out
NEW="${NEW:-tests/test_ringbuf.py tests/test_gpu_lpm.py tests/test_unwind.py tests/test_gpu_maps.py tests/test_gpu_sysbpf.py tests/test_gpu_sharded.py}"
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu $NEW > gpurun_out/g1_new.log 2>&1 || { tail -60 gpurun_out/g1_new.log; exit 1; }
tail -15 gpurun_out/g1_new.log
[ -n "$SKIP_ALL" ] && exit 0
timeout -k 10 900 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests > gpurun_out/g1_all.log 2>&1 || { tail -40 gpurun_out/g1_all.log; exit 1; }
tail -3 gpurun_out/g1_all.log

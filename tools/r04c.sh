# hash-map GPU tests, then flow-hash (cold + steady)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_maps.py tests/test_gpu_sharded.py tests/test_gpu_lru.py tests/test_gpu_counters.py tests/test_shm_json_perf.py tests/test_gpu_sysbpf.py > gpurun_out/r04c_gpu.log 2>&1 || { tail -30 gpurun_out/r04c_gpu.log; exit 1; }
tail -2 gpurun_out/r04c_gpu.log
timeout -k 10 300 python bench.py --workload flow-hash --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04c_fh.json 2> gpurun_out/r04c_fh.err || { tail gpurun_out/r04c_fh.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r04c_fh.json'));print('flow-hash',d['value'],d['roofline']['kernel_avg_ms'],d['parity']['ok'],d['cold'])"

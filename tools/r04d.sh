# ring-buffer GPU tests and the sampler line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_ringbuf.py tests/test_gpu_lpm.py > gpurun_out/r04d_gpu.log 2>&1 || { tail -40 gpurun_out/r04d_gpu.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/r04d_gpu.log | tail -20
timeout -k 10 300 python bench.py --workload ringbuf-sample --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04d_rb.json 2> gpurun_out/r04d_rb.err || { tail gpurun_out/r04d_rb.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r04d_rb.json'));print('ringbuf',d['value'],d['roofline']['kernel_avg_ms'],d['parity'])"

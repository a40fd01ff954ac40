# GPU suite, then flow-hash / syscall-agg / headline lines and lookup-cache hit rates
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r04b_gpu.log 2>&1 || { tail -30 gpurun_out/r04b_gpu.log; exit 1; }
tail -2 gpurun_out/r04b_gpu.log
for w in flow-hash syscall-agg; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04b_$w.json 2> gpurun_out/r04b_$w.err || { tail gpurun_out/r04b_$w.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r04b_$w.json'));print('$w',d['value'],d['ms_per_step'],d['roofline']['kernel_avg_ms'],d['parity']['ok'],d.get('cold'))"
  BPFTIME_AMD_DBG=512 timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04b_${w}_dbg.json 2> gpurun_out/r04b_${w}_dbg.err || { tail gpurun_out/r04b_${w}_dbg.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r04b_${w}_dbg.json'));print('$w dbg',d['parity']['ok'],d.get('dbg_lcache'))"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > gpurun_out/r04b_main.json 2> gpurun_out/r04b_main.err || { tail gpurun_out/r04b_main.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r04b_main.json'));print('main',d['value'],d['ms_per_step'],d['roofline']['kernel_avg_ms'],d['parity']['ok'])"

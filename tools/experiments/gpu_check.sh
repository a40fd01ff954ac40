set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/gpu_all.log 2>&1 || { tail -30 gpurun_out/gpu_all.log; exit 1; }
tail -3 gpurun_out/gpu_all.log
for w in tail-call flow-hash syscall-agg; do timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b_$w.json 2> gpurun_out/b_$w.err || { tail gpurun_out/b_$w.err; exit 1; }; python -c "import json;d=json.load(open('gpurun_out/b_$w.json'));print('$w',d['value'],d['ms_per_step'],d.get('parity'))"; done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_main.json 2> gpurun_out/b_main.err && python -c "import json;d=json.load(open('gpurun_out/b_main.json'));print('main',d['value'],d['ms_per_step'])"

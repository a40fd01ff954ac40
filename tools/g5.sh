set -o pipefail
export TMPDIR=/tmp
for e in X=0 BPFTIME_AMD_DBG=1 BPFTIME_AMD_DBG=128 BPFTIME_AMD_DBG=129; do env $e timeout -k 10 200 python bench.py --workload flow-hash --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/e.json 2>gpurun_out/e.err || { tail gpurun_out/e.err; exit 1; }; python -c "import json;d=json.load(open('gpurun_out/e.json'));print('$e',d['value'],d['ms_per_step'],d['parity']['ok'])"; done
BPFTIME_AMD_VERBOSE=1 timeout -k 10 200 python bench.py --workload flow-hash --steps 1 --warmup 0 --no-cpu-baseline --no-e2e 2>&1 | grep 'launch units' | tail -1

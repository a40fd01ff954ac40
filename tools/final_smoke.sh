set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/fs_smoke.log 2>&1 || { tail -20 gpurun_out/fs_smoke.log; exit 1; }
tail -1 gpurun_out/fs_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/fs_bench.json 2> gpurun_out/fs_bench.err || { tail gpurun_out/fs_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/fs_bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'], d['parity'])"

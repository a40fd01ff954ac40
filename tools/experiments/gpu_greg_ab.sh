mkdir -p gpurun_out
timeout -k 10 120 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 60 --timeout-method thread -p no:cacheprovider > gpurun_out/g1_chain.log 2>&1 || { tail -5 gpurun_out/g1_chain.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/g1_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/g1_pytest.log; [ $rc -le 1 ] || exit $rc
for w in flow-hash syscall-agg tail-call; do
  BPFTIME_AMD_VERBOSE=1 timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 20 > gpurun_out/g1_$w.json 2> gpurun_out/g1_$w.err || exit 1
  BPFTIME_AMD_LDS_REGS=1 timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 20 > gpurun_out/g1_${w}_lds.json 2>/dev/null || exit 1
  python3 -c "import json;a=json.load(open('gpurun_out/g1_$w.json'));b=json.load(open('gpurun_out/g1_${w}_lds.json'));print('$w greg',a['ms_per_step'],a['parity']['ok'],'lds',b['ms_per_step'],b['parity']['ok'])"
  tail -1 gpurun_out/g1_$w.err
done

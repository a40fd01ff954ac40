# thread-ordered kernel, asm tier: tier / ORDERED diffs vs the oracle, the GPU
# suite, the per-region profile (ab/seqprof.so) and the dispatch timings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/experiments/dbg/seq_ordered_diff.py || exit 1
timeout -k 10 400 python tools/experiments/dbg/seq_asm_diff.py 4096 > gpurun_out/seqdiff.txt 2>&1 && cat gpurun_out/seqdiff.txt || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/seqasm_pytest.log 2>&1 || { tail -30 gpurun_out/seqasm_pytest.log; exit 1; }
tail -2 gpurun_out/seqasm_pytest.log
for t in 64 4096; do
BPFTIME_AMD_LIB=$PWD/ab/seqprof.so timeout -k 10 120 python tools/experiments/seq_prof.py --threads $t --n 18 > gpurun_out/sp.txt 2>&1 || { cat gpurun_out/sp.txt; exit 1; }
echo "asm $(cat gpurun_out/sp.txt)"
done
timeout -k 10 300 python tools/sys_threads_time.py --n 20 --threads 64,4096,65536 --reps 2 || exit 1
for w in xdp-counter flow-hash tail-call syscount-latency; do
timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/q_$w.json 2> gpurun_out/q_$w.err || { tail gpurun_out/q_$w.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/q_$w.json').read().strip().splitlines()[-1]); print('$w', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d.get('parity'))"
done

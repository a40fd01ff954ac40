# the asm HASH-update handler: GPU suite, the thread-ordered timings and
# profile, and every bench line's parity / time (no CPU legs)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/upd_pytest.log 2>&1 || { tail -30 gpurun_out/upd_pytest.log; exit 1; }
tail -2 gpurun_out/upd_pytest.log
BPFTIME_AMD_LIB=$PWD/ab/seqprof.so timeout -k 10 120 python tools/experiments/seq_prof.py --threads 64 --n 18 || exit 1
timeout -k 10 300 python tools/sys_threads_time.py --n 22 --threads 64,4096,16384 --reps 2 || exit 1
for w in xdp-counter flow-hash syscall-agg syscount tail-call syscount-latency; do
timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/q_$w.json 2> gpurun_out/q_$w.err || { tail gpurun_out/q_$w.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/q_$w.json').read().strip().splitlines()[-1]); print('$w', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d.get('parity', {}).get('ok'))"
done

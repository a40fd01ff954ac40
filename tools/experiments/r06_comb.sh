# round 6 layout checks: GPU suite, then bench lines and their LDS counters
# (kt + SQ passes: SQ_LDS_BANK_CONFLICT, SQ_INSTS_LDS).  TAG names the run.
set -o pipefail
TAG=${TAG:-r06c}
WL=${WL:-flow-hash syscall-agg syscount}
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
fi
for w in $WL; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > gpurun_out/${TAG}_$w.json 2> gpurun_out/${TAG}_$w.err || { tail gpurun_out/${TAG}_$w.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/${TAG}_$w.json').read().strip().splitlines()[-1]); print('$w', d['value'], d['roofline']['kernel_avg_ms'], d['parity'].get('ok'))"
done
if [ -z "$NOPMC" ]; then
for w in $WL; do
  U=16777216; case $w in syscall-agg|syscount) U=33554432;; esac
  PASSES="kt sq1 sq2" UNITS=$U bash tools/prof_workload.sh $w $TAG || exit 1
done
fi

set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/g6_pytest.log 2>&1 || { tail -40 gpurun_out/g6_pytest.log; exit 1; }
tail -2 gpurun_out/g6_pytest.log
for w in flow-hash syscall-agg tail-call; do
  bash tools/ab_env.sh head $w X=0 BPFTIME_AMD_NO_MISS_LOG=1 || exit 1
done
WL="ringbuf-sample" bash tools/ab.sh base head v1 || exit 1

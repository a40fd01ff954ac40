set -o pipefail
export TMPDIR=/tmp
BPFTIME_AMD_SYNC_EACH=1 BPFTIME_AMD_VERBOSE=1 timeout -k 10 120 python -u -m pytest -x -q --timeout 60 --timeout-method thread -m gpu "tests/test_gpu_chain.py::test_syscall_records" "tests/test_gpu_maps.py::test_miss_log_parity" > gpurun_out/g8.log 2>&1; rc=$?
grep -v '^bpftime_amd: launch' gpurun_out/g8.log | tail -30; grep '^bpftime_amd: launch' gpurun_out/g8.log | sort | uniq -c | tail -5
exit $rc

# round 6 final checks: smoke + default bench line, the GPU suite, and the
# thread-ordered dispatch's two tiers at 4096 / 65536 threads (2^22 calls)
set -o pipefail
mkdir -p gpurun_out
bash tools/final_smoke.sh || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_pytest_gpu_final.log 2>&1 || { tail -30 gpurun_out/r06_pytest_gpu_final.log; exit 1; }
tail -2 gpurun_out/r06_pytest_gpu_final.log
for a in 1 0; do BPFTIME_AMD_SEQ_ASM=$a timeout -k 10 300 python tools/sys_threads_time.py --n 22 --threads 4096,65536 --reps 2 | sed "s/^/asm=$a /" || exit 1; done

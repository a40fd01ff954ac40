set -u
for w in main flow-hash syscall-agg tail-call lpm-route ringbuf-sample; do
  if [ $w = main ]; then a=""; else a="--workload $w"; fi
  BPFTIME_AMD_VERBOSE=1 timeout -k 10 120 python bench.py $a --steps 2 --warmup 1 --no-cpu-baseline --no-e2e 2> gpurun_out/verbose_$w.err > /dev/null || exit 1
  echo "$w: $(grep -m1 'bpftime_amd: launch' gpurun_out/verbose_$w.err) ($(grep -c 'bpftime_amd: launch' gpurun_out/verbose_$w.err) launches)"
done
timeout -k 10 300 bash tools/experiments/ab_env.sh base flow-hash "X=1" "BPFTIME_AMD_NO_LCACHE=1" "BPFTIME_AMD_LCACHE_SETS=512" "BPFTIME_AMD_LCACHE_SETS=4096" > gpurun_out/ab_lcache.txt 2>&1

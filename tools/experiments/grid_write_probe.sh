#!/bin/bash
# Headline per grid multiplier: bench time and the median launch's
# WRITE_SIZE / FETCH_SIZE per packet (raw KiB counters, 2^24 packets)
#   bash tools/experiments/grid_write_probe.sh "<mults...>"
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in $1; do
  BPFTIME_AMD_GRID_MULT=$m timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-e2e > gpurun_out/gw_$m.json 2> gpurun_out/gw_$m.err || { tail -3 gpurun_out/gw_$m.err; exit 1; }
  D=gpurun_out/gw_$m.pmc; rm -rf $D
  BPFTIME_AMD_GRID_MULT=$m timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D -o w -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $D.log 2>&1 || { echo "pmc fail $m"; tail -5 $D.log; exit 1; }
  BPFTIME_AMD_GRID_MULT=$m timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D -o f -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $D.log2 2>&1 || { echo "pmc fail $m"; tail -5 $D.log2; exit 1; }
  python3 - $D $m <<'PY'
import csv, glob, json, statistics, sys, collections
D, m = sys.argv[1], sys.argv[2]
per = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(D + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_interp" in r["Kernel_Name"]:
            per[r["Counter_Name"]][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
a = json.load(open(f"gpurun_out/gw_{m}.json"))
out = {k: statistics.median(v.values()) * 1024 / (1 << 24) for k, v in per.items()}
print("mult", m, "ms", a["ms_per_step"], "kernel", a["roofline"]["kernel_avg_ms"], "B/pkt raw", {k: round(v, 2) for k, v in out.items()})
PY
done

#!/bin/bash
# One bench line's raw WRITE_SIZE / FETCH_SIZE per unit of the median
# interpreter launch under several environments (write attribution):
#   bash tools/experiments/wprobe.sh <workload> <units> "ENV1" "ENV2" ...   ("X=1": none)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
W=$1; U=$2; shift 2
if [ "$W" = xdp-counter ]; then A="--steps 3 --warmup 1 --no-cpu-baseline --no-e2e"; else A="--workload $W --steps 3 --warmup 1 --no-cpu-baseline"; fi
i=0
for e in "$@"; do
  i=$((i + 1)); D=gpurun_out/wp_${W}_$i.pmc; rm -rf $D
  env $e timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D -o w -- python3 bench.py $A > $D.log 2>&1 || { echo "pmc fail $e"; tail -5 $D.log; exit 1; }
  env $e timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D -o f -- python3 bench.py $A > $D.log2 2>&1 || { echo "pmc fail $e"; tail -5 $D.log2; exit 1; }
  python3 - $D "$e" $U <<'PY'
import csv, glob, statistics, sys, collections
D, e, U = sys.argv[1], sys.argv[2], int(sys.argv[3])
per = collections.defaultdict(lambda: collections.defaultdict(float))
other = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(D + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        tgt = per if "k_interp" in r["Kernel_Name"] else other
        tgt[r["Counter_Name"]][(f, r["Kernel_Name"][:40], r["Dispatch_Id"])] += float(r["Counter_Value"])
out = {k: round(statistics.median(v.values()) * 1024 / U, 2) for k, v in per.items()}
oth = {k: round(sum(v.values()) * 1024 / U / 4, 2) for k, v in other.items()}   # (4 runs: warmup + 3)
print(e, "interp B/unit raw", out, "other kernels B/unit per run", oth)
PY
done

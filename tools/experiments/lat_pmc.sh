#!/bin/bash
# latency / occupancy PMC passes (rocprofv3 derived metrics, one per pass)
# of one bench workload: bash tools/experiments/lat_pmc.sh <workload> [tag]
set -u
export TMPDIR=/tmp
W=${1:-flow-hash}; T=${2:-lat}
D=gpurun_out/${T}_$W; rm -rf $D; mkdir -p $D
if [ "$W" = xdp-counter ]; then A="--steps 3 --warmup 1 --no-cpu-baseline --no-e2e"; else A="--workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-e2e"; fi
for m in InstrFetchLatency LdsLatency SmemLatency VmemLatency MeanOccupancyPerCU "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_WAVES SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_IFETCH"; do
  n=$(echo $m | cut -d' ' -f1)_$(echo $m | wc -w)
  timeout -s KILL 120 rocprofv3 --pmc $m --output-format csv -d $D -o $n -- python3 bench.py $A > $D/$n.log 2>&1 || { echo "FAIL $m"; tail -5 $D/$n.log; exit 1; }
done
python3 - $D <<'PY'
import csv, collections, glob, sys, statistics
D = sys.argv[1]
per = collections.defaultdict(dict)
for f in glob.glob(D + "/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "k_interp" in r["Kernel_Name"]:
            k = (r["Dispatch_Id"], f)
            per[r["Counter_Name"]][k] = per[r["Counter_Name"]].get(k, 0) + float(r["Counter_Value"])
agg = {k: statistics.median(v.values()) for k, v in per.items()}
w = agg.get("SQ_WAVES", 1)
for k, v in sorted(agg.items()):
    print(f"{k:26s} {v:16.1f}" + (f"  per-wave {v / w:12.1f}" if k.startswith("SQ_") and k != "SQ_WAVES" else ""))
PY

#!/bin/bash
# SQ counters of one workload under several environments: bash tools/experiments/ab_pmc_env.sh build workload "ENV1" "ENV2"
set -u
export TMPDIR=/tmp
v=$1; w=$2; shift 2
i=0
for e in "$@"; do
  i=$((i+1)); D=gpurun_out/abpe_$i; rm -rf $D
  env $e BPFTIME_AMD_LIB=$PWD/ab/$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT --output-format csv -d $D -o sq -- python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $D.log 2>&1 || { echo "FAIL $e"; tail -5 $D.log; exit 1; }
  env $e BPFTIME_AMD_LIB=$PWD/ab/$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $D -o sq2 -- python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $D.log2 2>&1 || { echo "FAIL2 $e"; tail -5 $D.log2; exit 1; }
  python3 - "$D" "$e" <<'PY'
import csv, collections, glob, sys, statistics
D, e = sys.argv[1], sys.argv[2]
per = collections.defaultdict(dict)
for f in glob.glob(D + "/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "k_interp" in r["Kernel_Name"]:
            per[r["Counter_Name"]][(r["Dispatch_Id"], f)] = per[r["Counter_Name"]].get((r["Dispatch_Id"], f), 0) + float(r["Counter_Value"])
agg = {k: statistics.median(v.values()) for k, v in per.items()}
w = agg["SQ_WAVES"]
print(e, " ".join(f"{k[3:]}={v / w:.0f}" for k, v in sorted(agg.items()) if k != "SQ_WAVES"))
PY
done

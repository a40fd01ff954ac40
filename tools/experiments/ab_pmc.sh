#!/bin/bash
# SQ counters of the headline kernel for library builds under ab/: bash tools/experiments/ab_pmc.sh variant...
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  D=gpurun_out/abpmc_$v
  rm -rf $D
  BPFTIME_AMD_LIB=$PWD/ab/$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $D -o sq -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $D.log 2>&1 || { echo "FAIL $v"; tail -5 $D.log; exit 1; }
  BPFTIME_AMD_LIB=$PWD/ab/$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_WAIT_ANY SQ_IFETCH SQ_INSTS_SENDMSG SQ_WAVES --output-format csv -d $D -o sq2 -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $D.log2 2>&1 || { echo "FAIL2 $v"; tail -5 $D.log2; exit 1; }
  python3 - "$D" "$v" <<'PY'
import csv, collections, glob, sys
D, v = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for f in glob.glob(D + "/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "k_interp" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
waves = sum(agg["SQ_WAVES"]) / len(agg["SQ_WAVES"])
print(v, " ".join(f"{k[3:]}={sum(x)/len(x)/waves:.0f}" for k, x in sorted(agg.items()) if k != "SQ_WAVES"))
PY
done

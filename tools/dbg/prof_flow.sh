set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pf
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/pf -o a -- python3 tools/dbg/micro_hash.py flow > gpurun_out/pf/a.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pf -o b -- python3 tools/dbg/micro_hash.py flow > gpurun_out/pf/b.log 2>&1 || exit $?
python3 - <<'PY'
import csv, collections, glob
for f in sorted(glob.glob("gpurun_out/pf/*counter_collection.csv")):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "k_interp" in r["Kernel_Name"]:
            agg[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    ids = sorted(agg)
    print(f, len(ids), "dispatches")
    for i in ids:
        print(i, {k: int(v) for k, v in sorted(agg[i].items())})
PY

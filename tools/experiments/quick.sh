#!/bin/bash
# quick GPU iteration: parity tests, bench, one SQ counter pass
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/q_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/q_pytest.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/q_bench.log 2>&1 || exit $?
cat gpurun_out/q_bench.log
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/q_prof -o sq -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/q_prof.log 2>&1 || exit $?
python3 - <<'PY'
import csv, collections, glob
f = glob.glob("gpurun_out/q_prof/sq_counter_collection.csv")[0]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if "k_interp" in r["Kernel_Name"]:
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
waves = sum(agg["SQ_WAVES"]) / len(agg["SQ_WAVES"])
for k, v in sorted(agg.items()):
    m = sum(v) / len(v)
    print(f"{k:22s} {m:16.0f}  per-wave {m / waves:12.1f}")
PY

# PMC passes over the thread-ordered dispatch kernel (k_sys_seq) for one
# program pair at 64 threads: instruction mix and waits per call
set -u
export TMPDIR=/tmp
P=${P:-pid}
D=gpurun_out/seq_pmc_$P
mkdir -p $D
A="tools/sys_threads_time.py --n 18 --threads 64 --reps 1 --progs $P"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o kt -- python3 $A > $D.kt.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $D -o sq1 -- python3 $A > $D.sq1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU SQ_WAVES --output-format csv -d $D -o sq2 -- python3 $A > $D.sq2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_DCACHE_REQ SQC_DCACHE_MISSES --output-format csv -d $D -o sqc -- python3 $A > $D.sqc.log 2>&1 || exit 1
python3 - <<PY
import csv, glob, collections
for tag in ("sq1", "sq2", "sqc"):
    for f in glob.glob("$D/**/%s_counter_collection.csv" % tag, recursive=True):
        acc = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if "k_sys_seq" in r.get("Kernel_Name", ""):
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
        for k, v in sorted(acc.items()):
            print(k, v)
PY
grep -h "k_sys_seq" $D/*/kt_kernel_stats.csv $D/kt_kernel_stats.csv 2>/dev/null | head -3

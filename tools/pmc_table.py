"""Per-launch PMC medians of the interpreter kernel for one tools/prof_workload.sh
run, as a table and as JSON (the `traffic` figure bench_workloads.py reads).

    python tools/pmc_table.py gpurun_out/prof_<tag>_<workload> <units per launch> [out.json]

FETCH_SIZE / WRITE_SIZE are kilobytes, turned into bytes with the factors
measured on known byte counts by tools/sol/calib.hip (profiles/r03_calib.json,
tools/calib.sh): reads x2 for every read shape the lines use (whole 64-B
slots, 16 B of a 64-B slot -- the memory side moves the whole 64 B --, a
128-B line per 2048-B slot: all 2.00); writes x2 for lines whose writes are
16-B-per-lane stores at a 64-B stride, i.e. in-place packet rewrites (the
c_rw16of64 / c_rwfull64 shapes: 2.00, and a 16-B rewrite costs the same
time as rewriting the whole 64-B line), x1 for coalesced stores (verdicts,
r0: c_wr4 1.00) and memory-side atomics (c_atom8: 32 B reported per 8-B
add, taken as moved).
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

HOT = "k_interp"
FETCH_FACTOR = 2.0
# bench lines whose dominant writes are strided in-place packet rewrites
WRITE_FACTOR = {"xdp-counter": 2.0, "tail-call": 2.0}


def means(d):
    per = defaultdict(lambda: defaultdict(float))
    big = 0
    rows = []
    for f in glob.glob(os.path.join(d, "*_counter_collection.csv")):
        with open(f) as fh:
            rows += [(r, os.path.basename(f)) for r in csv.DictReader(fh) if HOT in r["Kernel_Name"]]
    for r, _ in rows:
        big = max(big, int(r["Grid_Size"]))
    for r, f in rows:
        if int(r["Grid_Size"]) == big:
            per[r["Counter_Name"]][(r["Dispatch_Id"], f)] += float(r["Counter_Value"])
    # the median launch: a bench's first launch can differ (e.g. flow-hash
    # inserts its 65536 flows there), the timed ones are alike
    return {c: statistics.median(v.values()) for c, v in per.items()}


def kernel_ms(d):
    """(median launch ms, launches) of the hot kernel from the kernel trace."""
    f = os.path.join(d, "kt_kernel_trace.csv")
    if not os.path.exists(f):
        return None
    with open(f) as fh:
        ds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in csv.DictReader(fh)
              if HOT in r["Kernel_Name"]]
    return (statistics.median(ds), len(ds)) if ds else None


def main():
    d, units = sys.argv[1], int(sys.argv[2])
    cs = means(d)
    km = kernel_ms(d)
    out = {"dir": d, "units": units, "kernel_avg_ms": km[0] if km else None, "calls": km[1] if km else None,
           "counters": cs}
    w = cs.get("SQ_WAVES")
    print(f"kernel avg ms: {km}")
    for c in sorted(cs):
        extra = f"  per-wave {cs[c] / w:10.1f}" if w and c.startswith("SQ_") and c != "SQ_WAVES" else ""
        print(f"{c:36s} {cs[c]:16.1f}{extra}")
    if "TCC_HIT_sum" in cs and "TCC_MISS_sum" in cs and cs["TCC_HIT_sum"] + cs["TCC_MISS_sum"]:
        out["l2_hit"] = cs["TCC_HIT_sum"] / (cs["TCC_HIT_sum"] + cs["TCC_MISS_sum"])
        print(f"L2 hit rate {out['l2_hit']:.3f}")
    if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
        wl = os.path.basename(os.path.normpath(d)).split("_", 2)[-1]
        wf = WRITE_FACTOR.get(wl, 1.0)
        fb, wb = cs["FETCH_SIZE"] * 1024 * FETCH_FACTOR, cs["WRITE_SIZE"] * 1024 * wf
        out["hbm_bytes_per_launch"] = fb + wb
        out["bytes_per_unit"] = (fb + wb) / units
        out["factors"] = {"fetch": FETCH_FACTOR, "write": wf, "calibration": "profiles/r03_calib.json"}
        print(f"HBM bytes/launch {fb + wb:.4g} (fetch x{FETCH_FACTOR:g} {fb:.4g}, write x{wf:g} {wb:.4g}), "
              f"per unit {(fb + wb) / units:.1f}")
        if km:
            print(f"HBM GB/s {(fb + wb) / km[0] / 1e6:.1f}")
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

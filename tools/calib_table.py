"""Calibration factors from tools/calib.sh: for each access shape of
tools/sol/calib.hip, the known bytes per dispatch against the median
FETCH_SIZE / WRITE_SIZE rocprofv3 reported for it.

    python tools/calib_table.py gpurun_out/calib_<tag> [out.json]

factor_fetch = known read bytes / (FETCH_SIZE KB * 1024); a shape whose
reads cover whole lines gives the counter's bytes-per-unit rule; a partial
shape (16 B of a 64-B slot) gives how many bytes the memory side really
moved per byte the kernel asked for.  Same for writes.  tools/pmc_table.py
applies the factors of the shapes a bench line is made of."""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict


def counters(d):
    per = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "*_counter_collection.csv")):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"].split("(")[0].split("<")[0].strip()
                if "c_gather8" in r["Kernel_Name"]:
                    for t, nm in (("4194304", "c_gather8_4M"), ("67108864", "c_gather8_64M"),
                                  ("1073741824", "c_gather8_1G")):
                        if t in r["Kernel_Name"]:
                            k = nm
                per[k][r["Counter_Name"]].append((r["Dispatch_Id"], float(r["Counter_Value"])))
    out = {}
    for k, cs in per.items():
        out[k] = {}
        for c, vals in cs.items():
            byd = defaultdict(float)
            for did, v in vals:
                byd[did] += v
            out[k][c] = statistics.median(byd.values())
    return out


def main():
    d = sys.argv[1]
    known = {}
    for line in open(os.path.join(d, "plain.jsonl")):
        line = line.strip()
        if line:
            r = json.loads(line)
            known[r["kernel"]] = r
    cs = counters(d)
    rows = {}
    print(f"{'shape':16s} {'known rd':>12s} {'FETCH B':>12s} {'rd factor':>9s} {'known wr':>12s} {'WRITE B':>12s} "
          f"{'wr factor':>9s} {'L2 hit':>7s} {'GB/s':>8s}")
    for k, r in known.items():
        c = cs.get(k, {})
        fb = c.get("FETCH_SIZE", 0) * 1024
        wb = c.get("WRITE_SIZE", 0) * 1024
        hit, miss = c.get("TCC_HIT_sum"), c.get("TCC_MISS_sum")
        rf = r["read_bytes"] / fb if fb and r["read_bytes"] else None
        wf = r["write_bytes"] / wb if wb and r["write_bytes"] else None
        hr = hit / (hit + miss) if hit is not None and miss is not None and hit + miss else None
        rows[k] = {"units": r["units"], "known_read": r["read_bytes"], "fetch_bytes": fb, "read_factor": rf,
                   "known_write": r["write_bytes"], "write_bytes": wb, "write_factor": wf, "l2_hit": hr,
                   "ms": r["ms"], "GBps": r["GBps"]}
        f = lambda x: f"{x:9.3f}" if x is not None else f"{'-':>9s}"
        print(f"{k:16s} {r['read_bytes']:12.0f} {fb:12.0f} {f(rf)} {r['write_bytes']:12.0f} {wb:12.0f} {f(wf)} "
              f"{f(hr)[2:] if hr is not None else '      -'} {r['GBps']:8.1f}")
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as fh:
            json.dump({"dir": d, "shapes": rows}, fh, indent=1)


if __name__ == "__main__":
    main()

"""Per-dispatch PMC values of k_interp launches from rocprofv3 csv files
(one row per dispatch, counters summed over dimensions), grouped in runs of
`--group` consecutive dispatches (e.g. one micro-benchmark variant)."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
group = int(sys.argv[2]) if len(sys.argv) > 2 else 1
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
vals = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{d}/*_counter_collection.csv"):
    tag = f.split("/")[-1].split("_")[0]
    for r in csv.DictReader(open(f)):
        if "k_interp" in r["Kernel_Name"]:
            vals[(tag, int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
bytag = collections.defaultdict(list)
for (tag, i), cs in sorted(vals.items()):
    bytag[tag].append(cs)
for tag, rows in bytag.items():
    rows = rows[skip:]
    print("==", tag, len(rows), "dispatches")
    for g in range(0, len(rows), group):
        chunk = rows[g:g + group][-1:]  # last dispatch of each group (warm)
        cs = chunk[0]
        print(g // group, " ".join(f"{k}={v:.0f}" for k, v in sorted(cs.items())))

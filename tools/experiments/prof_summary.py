"""Summarise a tools/experiments/prof.sh run into profiles/ (tracked).

    python tools/experiments/prof_summary.py gpurun_out/prof_r01 r01 [packets_per_launch]

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_summary.md         per-kernel durations + per-launch PMC means
  profiles/pmc_traffic.json         HBM bytes per k_interp launch (read by bench.py)

FETCH_SIZE / WRITE_SIZE are kilobytes.  FETCH_SIZE is doubled: on gfx950 it
reports half the bytes of a coalesced streaming read (MI355X_MICROARCH.md,
HBM section); WRITE_SIZE is taken as is.
"""
import csv
import json
import os
import shutil
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
HOT = "k_interp"


def pmc_means(path):
    """{kernel: {counter: mean per dispatch}} over the dispatches of each
    kernel with its largest grid (the timed batch, not warm-up or e2e chunks)."""
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        rows = list(csv.DictReader(f))
    big = defaultdict(int)
    for row in rows:
        big[row["Kernel_Name"]] = max(big[row["Kernel_Name"]], int(row["Grid_Size"]))
    for row in rows:
        if int(row["Grid_Size"]) == big[row["Kernel_Name"]]:
            per[row["Kernel_Name"]][row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    return {k: {c: statistics.mean(d.values()) for c, d in cs.items()} for k, cs in per.items()}


def main():
    src, tag = sys.argv[1], sys.argv[2]
    packets = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 24
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    stats = os.path.join(src, "kt_kernel_stats.csv")
    shutil.copy(stats, os.path.join(out, f"{tag}_kernel_stats.csv"))
    with open(stats) as f:
        rows = list(csv.DictReader(f))
    pmc = {}
    for name in ("sq", "sq2", "fetch", "write"):
        for k, cs in pmc_means(os.path.join(src, f"{name}_counter_collection.csv")).items():
            pmc.setdefault(k, {}).update(cs)
    lines = [f"# rocprofv3 summary ({tag})", "",
             "Command: `tools/experiments/prof.sh` (bench.py --steps 10 --warmup 2 --no-cpu-baseline), "
             "one pass per counter group.", "",
             "| kernel | calls | avg ns | min ns | max ns | % |", "|---|---|---|---|---|---|"]
    for r in rows:
        lines.append(f"| `{r['Name']}` | {r['Calls']} | {float(r['AverageNs']):.0f} | {r['MinNs']} | "
                     f"{r['MaxNs']} | {float(r['Percentage']):.2f} |")
    hot = next((k for k in pmc if HOT in k), None)
    traffic = None
    if hot:
        cs = pmc[hot]
        lines += ["", f"Per-launch counter means for `{hot}`:", "", "| counter | value |", "|---|---|"]
        lines += [f"| {c} | {v:.1f} |" for c, v in sorted(cs.items())]
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            fetch_b = cs["FETCH_SIZE"] * 1024 * 2
            write_b = cs["WRITE_SIZE"] * 1024
            traffic = {"kernel": hot, "tag": tag, "program": "xdp-counter", "packets": packets,
                       "bytes_per_packet": (fetch_b + write_b) / packets, "fetch_size_kb_raw": cs["FETCH_SIZE"],
                       "write_size_kb": cs["WRITE_SIZE"], "fetch_bytes_corrected": fetch_b,
                       "write_bytes": write_b, "hbm_bytes_per_launch": fetch_b + write_b,
                       "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), KB -> bytes"}
            lines += ["", f"HBM bytes per launch: {fetch_b + write_b:.4g} "
                          f"(FETCH {fetch_b:.4g} after x2, WRITE {write_b:.4g})"]
        if "SQ_WAVES" in cs:
            w = cs["SQ_WAVES"]
            lines += ["", "Per-wave instruction mix: " + ", ".join(
                f"{c[8:]}={cs[c] / w:.0f}" for c in sorted(cs) if c.startswith("SQ_INSTS_"))]
    with open(os.path.join(out, f"{tag}_summary.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    if traffic:
        with open(os.path.join(out, "pmc_traffic.json"), "w") as f:
            json.dump(traffic, f, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()

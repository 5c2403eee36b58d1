#!/usr/bin/env python3
"""Summarise rocprofv3 CSV outputs (kernel stats and optional PMC counter
collections) into a compact text table for profiles/."""
import csv
import glob
import sys
from collections import defaultdict


def short(name, n=70):
    name = name.split("(")[0]
    return name if len(name) <= n else name[:n] + "..."


def stats(path):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# kernel stats: {path}\n# total kernel time {tot/1e6:.3f} ms")
    print(f"{'kernel':72s} {'calls':>6s} {'total_ms':>10s} {'avg_us':>9s} {'pct':>6s}")
    for r in rows:
        print(f"{short(r['Name']):72s} {int(r['Calls']):6d} {float(r['TotalDurationNs'])/1e6:10.3f} "
              f"{float(r['AverageNs'])/1e3:9.2f} {float(r['Percentage']):6.2f}")


def pmc(path):
    rows = list(csv.DictReader(open(path)))
    agg = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(int))
    for r in rows:
        k = short(r["Kernel_Name"])
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k][r["Counter_Name"]] += 1
    print(f"# PMC counters (per-dispatch averages): {path}")
    for k, d in sorted(agg.items()):
        parts = [f"{c}={v / cnt[k][c]:.4g}" for c, v in sorted(d.items())]
        print(f"{k:72s} " + " ".join(parts))


if __name__ == "__main__":
    for p in sys.argv[1:]:
        for f in sorted(glob.glob(p)):
            if f.endswith("kernel_stats.csv"):
                stats(f)
            elif f.endswith("counter_collection.csv"):
                pmc(f)

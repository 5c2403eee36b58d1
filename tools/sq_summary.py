#!/usr/bin/env python3
"""Per-kernel sums of rocprofv3 PMC counters (counter_collection.csv) for the kernels matching
a regex: dispatches and each counter's total, plus per-wave figures.

usage: sq_summary.py COUNTER_CSV [KERNEL_REGEX]"""
import collections
import csv
import re
import sys

rx = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"]
    if rx and not rx.search(k):
        continue
    k = k.split("(")[0][:60]
    tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
for k, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    w = c.get("SQ_WAVES", 0) or 1
    extra = ""
    if "SQ_WAVE_CYCLES" in c:
        wc = c["SQ_WAVE_CYCLES"]
        extra = " | per wave: " + " ".join(f"{n}={v / w:.0f}" for n, v in sorted(c.items()) if n != "SQ_WAVES")
        if "SQ_WAIT_ANY" in c:
            extra += f" | parked {c['SQ_WAIT_ANY'] / wc:.2f} issue-stalled {c.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} active {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f}"
    print(f"{k:60s} dispatches={len(disp[k]):4d} " + " ".join(f"{n}={v:.3e}" for n, v in sorted(c.items())) + extra)

#!/usr/bin/env python3
"""HBM traffic per launch of one kernel from two rocprofv3 PMC passes
(FETCH_SIZE and WRITE_SIZE in separate runs, as MI355X_MICROARCH.md prescribes:
FETCH_SIZE needs 3 TCC slots, WRITE_SIZE 2).  Units: both counters are KiB;
on gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane, incl. LDS-DMA)
streaming reads, so it is doubled here.  Writes the per-launch figure as JSON
(consumed by bench.py's roofline "traffic").

With ALG_JSON (tools/profile_forward.py --alg-json over the same command) and the engine profiler
TAG(s) the regex's symbols launch under ("a+b" for a union), the file also carries the algorithmic
bytes per launch of that same launch set and their ratio, so bench.py need not compare the PMC mean
with a different launch mix.

usage: pmc_traffic.py FETCH_CSV WRITE_CSV KERNEL_REGEX OUT_JSON [ALG_JSON TAG[+TAG]]"""
import csv
import json
import re
import sys


def per_launch(path, counter, rx):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and rx.search(r["Kernel_Name"])]
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


fetch_csv, write_csv, pattern, out = sys.argv[1:5]
rx = re.compile(pattern)
f, nf = per_launch(fetch_csv, "FETCH_SIZE", rx)
w, nw = per_launch(write_csv, "WRITE_SIZE", rx)
res = {"kernel_regex": pattern, "launches": [nf, nw],
       "fetch_bytes_per_launch": None if f is None else 2.0 * f * 1024,
       "write_bytes_per_launch": None if w is None else w * 1024,
       "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, KiB->B, mean per dispatch"}
if f is not None and w is not None:
    res["traffic_bytes_per_launch"] = res["fetch_bytes_per_launch"] + res["write_bytes_per_launch"]
if len(sys.argv) > 6 and "traffic_bytes_per_launch" in res:
    alg = json.load(open(sys.argv[5]))
    tags = sys.argv[6].split("+")
    n = sum(alg[t]["launches"] for t in tags if t in alg)
    b = sum(alg[t]["bytes"] for t in tags if t in alg)
    res["algorithmic_tags"] = tags
    res["algorithmic_launches"] = n
    if n:
        res["algorithmic_bytes_per_launch"] = b / n
        res["traffic_over_algorithmic"] = round(res["traffic_bytes_per_launch"] * n / b, 3) if b else None
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))

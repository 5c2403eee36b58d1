#!/usr/bin/env python3
"""Kernel concurrency in a rocprofv3 kernel trace (``--kernel-trace -f csv``).

With the decoder split over several streams, per-kernel durations no longer add up to
the wall time: kernels of different row blocks co-run.  This tool takes the kernel
trace of a run, keeps the dispatches inside the busiest window of ``--window-ms``
(default: all), and reports per kernel class: dispatches, summed duration, and the
time during which at least one kernel of the class was running (its union), plus the
whole trace's union ("GPU busy") and mean concurrency (sum of durations / union).

usage: trace_overlap.py KERNEL_TRACE_CSV [--top 20]
"""
import argparse
import csv
import re
from collections import defaultdict

CLASSES = [
    ("gemm_resid", re.compile(r"zv_gemm_kernel<.*, 1>$")),
    ("gemm", re.compile(r"zv_gemm_kernel")),
    ("gemm_ws", re.compile(r"zv_gemm_resid_ws")),
    ("attn_sa", re.compile(r"zv_attn_sa")),
    ("attn_na", re.compile(r"zv_attn_na")),
    ("attn_stats", re.compile(r"zv_attn_stats")),
    ("dwconv", re.compile(r"dwconv")),
    ("biasnorm", re.compile(r"biasnorm")),
    ("vocoder", re.compile(r"zv_voc|vocos")),
]


def klass(name):
    for c, rx in CLASSES:
        if rx.search(name):
            return c
    return "other"


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if ce is not None:
        tot += ce - cs
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    iv.sort()
    t0, t1 = iv[0][0], max(e for _, e, _ in iv)
    by = defaultdict(list)
    for s, e, n in iv:
        by[klass(n)].append((s, e))
    busy = union([(s, e) for s, e, _ in iv])
    total = sum(e - s for s, e, _ in iv)
    print(f"trace span {(t1 - t0) / 1e6:.2f} ms, GPU busy (union) {busy / 1e6:.2f} ms, "
          f"sum of kernel durations {total / 1e6:.2f} ms, mean concurrency {total / busy:.2f}")
    print(f"{'class':12s} {'n':>7s} {'sum ms':>9s} {'union ms':>9s} {'sum/union':>9s}")
    for c, v in sorted(by.items(), key=lambda kv: -sum(e - s for s, e in kv[1])):
        sm = sum(e - s for s, e in v)
        un = union(v)
        print(f"{c:12s} {len(v):7d} {sm / 1e6:9.2f} {un / 1e6:9.2f} {sm / max(un, 1):9.2f}")


if __name__ == "__main__":
    main()

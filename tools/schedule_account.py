#!/usr/bin/env python3
"""Where the timed step's wall time goes, from a rocprofv3 kernel trace of
tools/trace_step.py (the bench's C2 step on its default decoder streams).

The timed steps are the last busy cluster of the trace (idle gaps >= --gap-ms fence it).
Reports, per step: wall (first dispatch start -> last end), kernel-busy union (>= 1
kernel running), idle time inside the window and its largest gaps, the sum of kernel
durations and mean concurrency (sum / union), then per kernel class: dispatches, summed
duration, union, and the time the class ran ALONE (no other kernel concurrently).

usage: schedule_account.py KERNEL_TRACE_CSV --steps 2 [--gap-ms 100] [--json OUT]
"""
import argparse
import csv
import json
import re
from collections import defaultdict

CLASSES = [
    ("ffn_fused", re.compile(r"zv_ffn_kernel")),
    ("gemm256_plain/glu", re.compile(r"zv_gemm256_kernel")),
    ("gemm_resid", re.compile(r"zv_gemm_kernel<.*, [1245], \d+, \d+>\(")),
    ("gemm_na", re.compile(r"zv_gemm_kernel<128, 96, 2, 2, 1, 2,")),
    ("gemm_glu", re.compile(r"zv_gemm_kernel<128, 128, 2, 2, 1, 3,")),
    ("gemm_vt", re.compile(r"zv_gemm_kernel<64, 64,")),
    ("gemm_other", re.compile(r"zv_gemm_kernel")),
    ("attn_sa", re.compile(r"zv_attn_sa")),
    ("attn_na", re.compile(r"zv_attn_na")),
    ("attn_stats", re.compile(r"zv_attn_stats")),
    ("dwconv", re.compile(r"dwconv")),
    ("biasnorm", re.compile(r"biasnorm")),
    ("vocoder", re.compile(r"zv_voc|vocos")),
    ("copy/fill", re.compile(r"rocclr|copy|fill")),
]


def klass(name):
    for c, rx in CLASSES:
        if rx.search(name):
            return c
    return "other_elementwise"


def merge(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def length(iv):
    return sum(e - s for s, e in iv)


def subtract(a, b):
    """a minus b (both merged, sorted)."""
    out, j = [], 0
    for s, e in a:
        cur = s
        while j < len(b) and b[j][1] <= cur:
            j += 1
        k = j
        while k < len(b) and b[k][0] < e:
            if b[k][0] > cur:
                out.append([cur, b[k][0]])
            cur = max(cur, b[k][1])
            k += 1
        if cur < e:
            out.append([cur, e])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--gap-ms", type=float, default=100.0)
    ap.add_argument("--json")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    gap = a.gap_ms * 1e6
    # clusters separated by idle gaps; the timed steps are the last cluster
    clusters, cur, end = [], [], None
    for s, e, n in iv:
        if cur and s - end > gap:
            clusters.append(cur)
            cur = []
        cur.append((s, e, n))
        end = e if end is None else max(end, e)
    clusters.append(cur)
    win = clusters[-1]
    t0, t1 = win[0][0], max(e for _, e, _ in win)
    wall = (t1 - t0) / a.steps
    allv = merge([(s, e) for s, e, _ in win])
    busy = length(allv) / a.steps
    tot = sum(e - s for s, e, _ in win) / a.steps
    gaps = sorted(((allv[i + 1][0] - allv[i][1]) for i in range(len(allv) - 1)), reverse=True)
    byc = defaultdict(list)
    for s, e, n in win:
        byc[klass(n)].append((s, e))
    res = {"steps": a.steps, "wall_ms": wall / 1e6, "busy_union_ms": busy / 1e6,
           "idle_ms": (wall - busy) / 1e6, "sum_kernel_ms": tot / 1e6,
           "mean_concurrency": tot / busy, "dispatches_per_step": len(win) / a.steps,
           "largest_gaps_us": [g / 1e3 for g in gaps[:8]],
           "gaps_over_10us_per_step": sum(1 for g in gaps if g > 1e4) / a.steps, "classes": {}}
    print(f"window: {len(win)} dispatches, {a.steps} steps")
    print(f"per step: wall {wall/1e6:.2f} ms | busy union {busy/1e6:.2f} | idle {(wall-busy)/1e6:.2f} | "
          f"sum of kernel durations {tot/1e6:.2f} | mean concurrency {tot/busy:.3f}")
    print(f"largest idle gaps (us): {', '.join(f'{g/1e3:.1f}' for g in gaps[:8])}; "
          f"gaps > 10 us per step: {res['gaps_over_10us_per_step']:.1f}")
    # what borders the largest gaps: the last kernel to end before, the first to start after
    ends = sorted((e, n) for _, e, n in win)
    starts = sorted((s, n) for s, _, n in win)
    for i in sorted(range(len(allv) - 1), key=lambda i: allv[i][1] - allv[i + 1][0])[:4]:
        g0, g1 = allv[i][1], allv[i + 1][0]
        before = max((e, n) for e, n in ends if e <= g0)[1]
        after = min((s, n) for s, n in starts if s >= g1)[1]
        print(f"  gap {(g1 - g0) / 1e3:9.1f} us at {(g0 - t0) / 1e6:8.2f} ms: after {before[:60]} | "
              f"before {after[:60]}")
    print(f"{'class':22s} {'disp':>6s} {'sum ms':>8s} {'union ms':>9s} {'alone ms':>9s}")
    for c, v in sorted(byc.items(), key=lambda kv: -sum(e - s for s, e in kv[1])):
        mv = merge(v)
        others = merge([(s, e) for cc, vv in byc.items() if cc != c for s, e in vv])
        alone = length(subtract(mv, others))
        d = {"dispatches": len(v) / a.steps, "sum_ms": sum(e - s for s, e in v) / a.steps / 1e6,
             "union_ms": length(mv) / a.steps / 1e6, "alone_ms": alone / a.steps / 1e6}
        res["classes"][c] = d
        print(f"{c:22s} {d['dispatches']:6.0f} {d['sum_ms']:8.2f} {d['union_ms']:9.2f} {d['alone_ms']:9.2f}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()

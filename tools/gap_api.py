#!/usr/bin/env python3
"""Which host calls fill the largest idle gaps of a traced step (the GPU waits on the host).

  rocprofv3 --kernel-trace --hip-runtime-trace -f csv -d OUT -o run -- python3 tools/trace_step.py
  python3 tools/gap_api.py OUT/*kernel_trace.csv OUT/*hip_api_trace.csv [--top 4]

For each of the top gaps between kernels of the last busy cluster (the timed steps): the
HIP API calls that overlap it, longest first, with their overlap in us.
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernels")
    ap.add_argument("api")
    ap.add_argument("--top", type=int, default=4)
    ap.add_argument("--gap-ms", type=float, default=100.0)
    a = ap.parse_args()
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                for r in csv.DictReader(open(a.kernels)))
    clusters, cur, end = [], [], None
    for s, e, n in iv:
        if cur and s - end > a.gap_ms * 1e6:
            clusters.append(cur)
            cur = []
        cur.append((s, e, n))
        end = e if end is None else max(end, e)
    clusters.append(cur)
    win = clusters[-1]
    t0 = win[0][0]
    merged = []
    for s, e, _ in win:
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])
    gaps = sorted(((merged[i][1], merged[i + 1][0]) for i in range(len(merged) - 1)),
                  key=lambda g: g[0] - g[1])[:a.top]
    api = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"])
           for r in csv.DictReader(open(a.api))]
    for g0, g1 in gaps:
        over = defaultdict(lambda: [0, 0])
        for s, e, f in api:
            o = min(e, g1) - max(s, g0)
            if o > 0:
                over[f][0] += o
                over[f][1] += 1
        print(f"gap {(g1 - g0) / 1e3:.1f} us at {(g0 - t0) / 1e6:.2f} ms: host calls in it "
              f"(overlap us, count): " + ", ".join(f"{f} {v[0] / 1e3:.1f} x{v[1]}" for f, v in
                                                   sorted(over.items(), key=lambda kv: -kv[1][0])[:6]))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-stage kernel time of one BigVGAN decode from a rocprofv3 kernel-trace CSV
(tools/bigvgan_bench.py run): the last decode in the trace is split at its
ConvTranspose gathers and each stage's time is reported by kernel family."""
import csv
import sys
from collections import defaultdict


def family(name):
    if "zv_gemm_kernel" in name:
        return "gemm_conv" if name.rstrip().endswith("1>") else "gemm_plain"
    for k in ("act_kernel", "convt_gather", "avg_kernel", "post_kernel", "im2col"):
        if k in name:
            return k
    return None


rows = [r for r in csv.DictReader(open(sys.argv[1]))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ks = [(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows
      if family(r["Kernel_Name"])]
starts = [i for i, (n, _) in enumerate(ks) if "im2col" in n]
last = ks[starts[-1]:]
stage, agg = -1, defaultdict(lambda: defaultdict(float))
for n, us in last:
    if "convt_gather" in n:
        stage += 1
    agg[stage][family(n)] += us
tot = 0.0
for st in sorted(agg):
    s = sum(agg[st].values())
    tot += s
    print(f"stage {st:2d}: {s:8.1f} us  " + "  ".join(f"{k}={v:.1f}" for k, v in sorted(agg[st].items())))
print(f"total {tot:.1f} us")

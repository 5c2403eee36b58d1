#!/usr/bin/env python3
"""Run exactly the bench's timed C2 step under a kernel tracer, fenced by idle gaps, so a
trace of the 3-stream schedule can be cut to the timed steps (tools/schedule_account.py).

  rocprofv3 --kernel-trace -f csv -d OUT -o run -- python tools/trace_step.py [--steps 2]

Two warm-up steps (graph capture), 300 ms idle, --steps timed steps, 300 ms idle.
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--precision", default="bf16")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    conf = bench.CONFIGS["C2"]
    m = bench.build(conf["variant"], args.precision, dev)
    job = bench.Job(conf, m, bench.build_vocoder(dev), conf["per_gpu"], dev)
    for _ in range(2):
        job.step()
    torch.cuda.synchronize()
    time.sleep(0.3)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        job.step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    time.sleep(0.3)
    print(f"timed {args.steps} steps: {dt * 1e3:.2f} ms per step (host clock)", flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Host side of one C2 benchmark step on one GPU (the per-rank host budget of the 8-GPU runs):
how long ZipVoice.sample() + the vocoder take to RETURN (the host issuing every launch of the
step: text encoder, conditions, the 16-step guided Euler loop on the decoder's streams, the
prompt split, the vocoder) against the step's wall time once the GPU has drained.  With
the launch count of the same step (rocprofv3 --kernel-trace --stats of this command, calls /
steps) this gives the host time per launch.  If issue time < wall time the host runs ahead of
the GPU and a rank's host thread is not the bottleneck.

usage: python tools/host_rate.py [--steps 3]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=3)
a = ap.parse_args()
dev = torch.device("cuda", 0)
conf = bench.CONFIGS["C2"]
model = bench.build(conf["variant"], "bf16", dev)
voc = bench.build_vocoder(dev)
job = bench.Job(conf, model, voc, conf["per_gpu"], dev)
for _ in range(2):
    job.compute(list(range(job.n_local)))
torch.cuda.synchronize()
issue, wall = [], []
for _ in range(a.steps):
    t0 = time.perf_counter()
    job.compute(list(range(job.n_local)))
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    issue.append(t1 - t0)
    wall.append(t2 - t0)
print(f"C2 step (sample + vocoder, 32 utterances, one GPU): host issue {1e3 * min(issue):.1f} ms "
      f"(median {1e3 * sorted(issue)[len(issue) // 2]:.1f}), wall {1e3 * min(wall):.1f} ms "
      f"(median {1e3 * sorted(wall)[len(wall) // 2]:.1f}); issue / wall {min(issue) / min(wall):.2f}")

#!/usr/bin/env python3
"""Throughput of the BigVGAN-v2 vocoder (bigvgan_v2_24khz_100band_256x shapes, synthetic
weights) on one GPU: audio seconds generated per wall second for B utterances of T
frames (24 kHz, hop 256), both precisions.  Prints one JSON line per precision.

    python tools/bigvgan_bench.py [--frames 938] [--batch 1] [--iters 5]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from zipvoice_amd.bigvgan import BigVGAN, BigVGANConfig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=938)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--precision", default="fp32,bf16")
    a = ap.parse_args()
    cfg = BigVGANConfig()
    g = torch.Generator().manual_seed(0)
    mel = (1.5 * torch.randn(a.batch, 100, a.frames, generator=g) - 4.0).cuda()
    for prec in a.precision.split(","):
        v = BigVGAN(cfg, precision=prec).load_synthetic(0).to("cuda:0")
        v.decode(mel)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.iters):
            wav = v.decode(mel)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / a.iters
        audio_s = a.batch * a.frames * cfg.hop_length / cfg.sampling_rate
        print(json.dumps({"vocoder": "bigvgan_v2_24khz_100band_256x", "precision": prec,
                          "batch": a.batch, "frames": a.frames, "ms": round(dt * 1e3, 3),
                          "audio_s_per_s": round(audio_s / dt, 1),
                          "finite": bool(torch.isfinite(wav).all()),
                          "device_MB": round(v.device_bytes() / 2**20, 1)}), flush=True)
        del v
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-GPU throughput of the other BASELINE.json configurations (single GPU, the
per-GPU share of the multi-GPU ones), ``ZipVoice*.sample()`` only (text encoder,
conditions, the guided / distilled Euler loop; no vocoder):

  C3  ZipVoice-Distill, N_steps=8, 16 utterances per GPU (128 over 8 GPUs),
      3 s prompt + 10 s generated (T = 1219), guidance 3.0 as an embedding
  C4  ZipVoice-Dialog, N_steps=16, 16 x (6 s prompt + 30 s generated, T = 3376),
      CFG 1.5 (32 rows)
  C5  ZipVoice-Dialog-Stereo, N_steps=16, 4 per GPU (32 over 8 GPUs), T = 3376,
      200-dim two-channel features, CFG 1.5; run it with precision fp8 for the BASELINE
      "fp8 MFMA weights" mode (ZV_FP8: MX-fp8 feed-forward / conv / NA-out linears)

usage: config_bench.py [C3,C4,C5] [steps] [precision (bf16)]
Two untimed warm-up steps (the first sizes the workspace, the second captures the graph)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from zipvoice_amd.config import default_config  # noqa: E402
from zipvoice_amd.models import build_model  # noqa: E402
from zipvoice_amd.weights import synthetic_state_dict  # noqa: E402

CONFIGS = {
    "C3": dict(variant="zipvoice_distill", B=16, Tp=281, Tg=938, Sp=40, St=134, N=8, g=3.0, F=100),
    "C4": dict(variant="zipvoice_dialog", B=16, Tp=563, Tg=2813, Sp=80, St=400, N=16, g=1.5, F=100),
    "C5": dict(variant="zipvoice_dialog_stereo", B=4, Tp=563, Tg=2813, Sp=80, St=400, N=16, g=1.5,
               F=200),
}


def run(name, steps, precision="bf16"):
    c = CONFIGS[name]
    dev = torch.device("cuda:0")
    cfg = default_config(c["variant"])
    m = build_model(cfg, precision=precision)
    m.load_state_dict(synthetic_state_dict(cfg, 0))
    m = m.to(dev)
    rng = np.random.default_rng(7)
    dialog = c["variant"].startswith("zipvoice_dialog")

    def toks(n):
        t = [int(v) for v in rng.integers(1, 360, n)]
        if dialog:                      # [S1] ... [S2] ... turns
            t[0], t[n // 2] = 360, 361
        return t

    B = c["B"]
    tokens = [toks(c["St"]) for _ in range(B)]
    ptokens = [toks(c["Sp"]) for _ in range(B)]
    pf = torch.from_numpy((0.3 * rng.standard_normal((B, c["Tp"], c["F"])) - 0.5).astype(np.float32)).to(dev)
    plens = torch.full((B,), c["Tp"], dtype=torch.int64, device=dev)
    flens = torch.full((B,), c["Tg"], dtype=torch.int64, device=dev)

    def step():
        return m.sample(tokens=tokens, prompt_tokens=ptokens, prompt_features=pf,
                        prompt_features_lens=plens, features_lens=flens, t_shift=0.5,
                        duration="real", num_step=c["N"], guidance_scale=c["g"])

    step()
    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    frames = B * c["Tg"]
    audio_s = frames * 256 / 24000
    return {"config": name, "variant": c["variant"], "precision": precision, "utterances_per_gpu": B, "T": c["Tp"] + c["Tg"],
            "num_step": c["N"], "ms_per_step": round(dt * 1e3, 2),
            "mel_frames_per_s_per_gpu": round(frames / dt, 1), "x_realtime_per_gpu": round(audio_s / dt, 1)}


if __name__ == "__main__":
    names = sys.argv[1].split(",") if len(sys.argv) > 1 else list(CONFIGS)
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    prec = sys.argv[3] if len(sys.argv) > 3 else "bf16"
    for n in names:
        print(json.dumps(run(n, steps, prec)), flush=True)

"""Measure the second-generation attention consumers (csrc/zv_flash2.inc) through the engine:
fast path vs forced exact path (ZV_ATTN2_EXACT=1), ATTN2=1 vs ATTN2=0 (first generation), the
materialising fallback (ZV_ATTN_MATERIALIZE=1), and how often the exact path fires when the
attention-score projection's q / p rows are scaled by S (scores x S).  Prints one line per case;
the bounds of tests/test_gpu_attn2.py come from these numbers.

    python tools/attn2_probe.py [--T 1219 3376] [--scales 1 4 8 16 32]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from zipvoice_amd.config import default_config  # noqa: E402
from zipvoice_amd.models import build_model  # noqa: E402
from zipvoice_amd.weights import synthetic_state_dict  # noqa: E402


def scaled_scores_sd(cfg, sd, S):
    """q and p rows (and biases) of every decoder attention-score projection times S."""
    out = dict(sd)
    H, qd, pd = cfg.fm_decoder_num_heads, cfg.query_head_dim, cfg.pos_head_dim
    for k in sd:
        if k.startswith("fm_decoder.") and "self_attn_weights.in_proj" in k:
            a = np.array(sd[k], dtype=np.float32, copy=True)
            a[:H * qd] *= S
            a[2 * H * qd:2 * H * qd + H * pd] *= S
            out[k] = a
    return out


def engine(cfg, sd, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        m = build_model(cfg, precision="bf16")
        m.load_state_dict(sd)
        return m.to("cuda:0")
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def inputs(B, T, lens, seed):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((B, T, 100), dtype=np.float32)
    tc = rng.standard_normal((B, T, 100), dtype=np.float32)
    sc = (0.3 * rng.standard_normal((B, T, 100)) - 0.5).astype(np.float32)
    pm = np.arange(T)[None] >= np.array(lens)[:, None]
    return [torch.from_numpy(a).to("cuda:0") for a in (x, tc, sc, pm)]


def vel(m, ins):
    x, tc, sc, pm = ins
    v = m.engine.velocity(0.3, 1.0, x, tc, sc, pm)
    torch.cuda.synchronize()
    return v.float().cpu()


def stats(a, b, valid):
    d = (a - b).abs()[valid]
    return f"mean {d.mean().item():.3e} max {d.max().item():.3e}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, nargs="+", default=[1219, 3376])
    ap.add_argument("--scales", type=float, nargs="+", default=[1, 4, 8, 16, 32])
    a = ap.parse_args()
    cfg = default_config("zipvoice")
    sd0 = synthetic_state_dict(cfg, 0)
    for T in a.T:
        lens = [T, int(T * 0.82)]
        ins = inputs(2, T, lens, seed=T)
        valid = ~ins[3].cpu()
        for S in a.scales:
            sd = scaled_scores_sd(cfg, sd0, S) if S != 1 else sd0
            e2 = engine(cfg, sd, {})
            e2.engine.attn_fallbacks(reset=True)
            v2 = vel(e2, ins)
            c2 = e2.engine.attn_fallbacks(reset=True)
            del e2
            ex = engine(cfg, sd, {"ZV_ATTN2_EXACT": "1"})
            vx = vel(ex, ins)
            cx = ex.engine.attn_fallbacks(reset=True)
            del ex
            e1 = engine(cfg, sd, {"ZV_ATTN2": "0"})
            v1 = vel(e1, ins)
            del e1
            line = (f"T={T} S={S:g}: fallbacks fast {c2} forced {cx}; fast==exact {torch.equal(v2, vx)} "
                    f"(|d| {stats(v2, vx, valid)}); attn2 vs attn1 {stats(v2, v1, valid)}; "
                    f"finite {bool(torch.isfinite(v2).all())}")
            if S == 1:
                em = engine(cfg, sd, {"ZV_ATTN_MATERIALIZE": "1"})
                vm = vel(em, ins)
                del em
                line += f"; fused vs materialised {stats(v2, vm, valid)}; attn1 vs mat {stats(v1, vm, valid)}"
            print(line, flush=True)
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

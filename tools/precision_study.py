#!/usr/bin/env python3
"""Where does the bf16 mode's error come from?  A CPU emulation study on the oracle.

The engine's bf16 mode rounds every MFMA operand to bf16 (activations written by the
producing kernels, weights once at load) and keeps everything else fp32: accumulation,
residual stream, softmax statistics, BiasNorm, activations' arithmetic.  This tool
re-runs the fp32 oracle (oracle/zipvoice_np.py) with exactly those rounding points
emulated in numpy, per GEMM family, and measures the mean |error| of ZipVoice.sample()
against the reference's own output (tests/golden/sample_c1.npz: C1 shapes, T = 422,
4 guided steps).  Formats: bf16 (8-bit significand), fp16 (11-bit significand, same
MFMA rate on gfx950).  Families:

  attn   self_attn_weights.in_proj (q, k, positional p) and the score operands q, k
  ff     feed_forward{1,2,3} in/out projections and the SwooshL hidden activation
  na     nonlin_attention projections, the x*tanh(s) values, y and the head-0 P.V
  sa     self_attn{1,2} projections, V and the P.V operands
  conv   conv_module{1,2} projections, GLU output and the depthwise-conv output
  io     decoder in_proj / out_proj, text encoder projections

usage: python tools/precision_study.py [--out profiles/r02_precision_study.txt]
Analysis tool only (imports the oracle, runs on the CPU); nothing here is on the product path.
"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import oracle.zipvoice_np as Z  # noqa: E402
from golden_io import load, tokens_list  # noqa: E402

F32 = np.float32
ORIG = {k: getattr(Z, k) for k in ("linear", "attn_weights", "feed_forward", "nonlin_attention",
                                   "self_attention", "conv_module")}


def q_bf16(x):
    x = np.ascontiguousarray(x, F32)
    u = x.view(np.uint32)
    r = ((u + np.uint32(0x7FFF) + ((u >> 16) & np.uint32(1))) & np.uint32(0xFFFF0000))
    return r.view(F32)


def q_fp16(x):
    return np.asarray(x, F32).astype(np.float16).astype(F32)


QF = {"bf16": q_bf16, "fp16": q_fp16, None: lambda x: np.asarray(x, F32)}
# one-sided formats of a linear's operands (the other side exact): "a16" rounds the activation
# to fp16 and keeps the weight exact (the engine's weight-split product ah.bh + ah.bl), "w16" the
# reverse (activation split: ah.bh + al.bh); outputs stored by the family round as fp16
SIDE = {"a16": ("fp16", None), "w16": (None, "fp16")}


class Emu:
    """Which family rounds its operands to which format."""

    def __init__(self, fam):
        self.fam = fam          # dict family -> format (None = fp32)
        self.cur = "io"
        self.text_exact = False  # text encoder left in fp32

    def q(self, x, fam=None):
        f = self.fam.get(fam or self.cur)
        return QF[SIDE[f][0] if f in SIDE else f](x)

    def qw(self, w, fam=None):
        f = self.fam.get(fam or self.cur)
        return QF[SIDE[f][1] if f in SIDE else f](w)


EMU = Emu({})


KEYS = {}                    # id(weight array) -> state-dict key
FP32_KEYS = ("time_emb", "time_embed", "guidance_scale_embed")   # fp32 small linears in the engine


def linear(x, w, b=None):
    if any(t in KEYS.get(id(w), "") for t in FP32_KEYS):
        return ORIG["linear"](x, w, b)
    y = np.matmul(EMU.q(x), EMU.qw(w).T)
    if b is not None:
        y = y + b
    return y.astype(F32)


def attn_weights(P, x, pe, key_pad, heads, qdim, pdim):
    prev, EMU.cur = EMU.cur, "attn"
    B, L, _ = x.shape
    xp = EMU.q(linear(x, P["in_proj.weight"], P["in_proj.bias"]), "qk")   # q | k | p stored 16-bit
    EMU.cur = prev
    qd = qdim * heads
    qq = xp[..., :qd].reshape(B, L, heads, qdim).transpose(2, 0, 1, 3)
    kk = xp[..., qd:2 * qd].reshape(B, L, heads, qdim).transpose(2, 0, 3, 1)
    pp = xp[..., 2 * qd:].reshape(B, L, heads, pdim).transpose(2, 0, 1, 3)
    scores = np.matmul(qq, kk)
    pos = ORIG["linear"](pe, P["linear_pos.weight"])                 # fp32 in the engine
    pos = pos.reshape(2 * L - 1, heads, pdim).transpose(1, 2, 0)[:, None]
    ps = np.matmul(pp, pos)
    i = np.arange(L)[:, None]
    j = np.arange(L)[None, :]
    scores = scores + ps[:, :, i, L - 1 - i + j]
    if key_pad is not None:
        scores = np.where(key_pad[None, :, None, :], F32(-1000.0), scores)
    m = scores.max(axis=-1, keepdims=True)
    return np.exp(scores - m).astype(F32)      # unnormalised: consumers normalise (engine order)


def _pv(Wu, v, fam):
    """P.V with 16-bit P and V, normalised by the sum of the rounded P (the engine's
    ones-row denominator)."""
    Pq = EMU.q(Wu, fam)
    return (np.matmul(Pq, EMU.q(v, fam)) / Pq.sum(-1, keepdims=True)).astype(F32)


def feed_forward(P, x):
    prev, EMU.cur = EMU.cur, "ff"
    h = linear(x, P["in_proj.weight"], P["in_proj.bias"])
    out = linear(EMU.q(Z.swoosh_l_fwd(h)), P["out_proj.weight"], P["out_proj.bias"])
    EMU.cur = prev
    return out


def nonlin_attention(P, x, w0):
    prev, EMU.cur = EMU.cur, "na"
    h = linear(x, P["in_proj.weight"], P["in_proj.bias"])
    hid = h.shape[-1] // 3
    s, v, y = h[..., :hid], h[..., hid:2 * hid], h[..., 2 * hid:]
    v = (v * np.tanh(s)).astype(F32)
    v = _pv(w0, v, "na")
    v = EMU.q((v * EMU.q(y)).astype(F32))
    out = linear(v, P["out_proj.weight"], P["out_proj.bias"])
    EMU.cur = prev
    return out


def self_attention(P, x, W, vdim):
    # sub-families (round 4; each defaults to "sa"): sa_in the value projection, sa_pv the P and V
    # operands of P.V, sa_out the out-projection
    prev = EMU.cur
    sub = lambda n: n if n in EMU.fam else "sa"  # noqa: E731
    B, L, _ = x.shape
    H = W.shape[0]
    EMU.cur = sub("sa_in")
    v = linear(x, P["in_proj.weight"], P["in_proj.bias"]).reshape(B, L, H, vdim).transpose(2, 0, 1, 3)
    o = _pv(W, v, sub("sa_pv")).transpose(1, 2, 0, 3).reshape(B, L, H * vdim)
    EMU.cur = sub("sa_out")
    out = linear(o, P["out_proj.weight"], P["out_proj.bias"])
    EMU.cur = prev
    return out


def conv_module(P, x, key_pad):
    prev, EMU.cur = EMU.cur, "conv"
    h = linear(x, P["in_proj.weight"], P["in_proj.bias"])
    C = h.shape[-1] // 2
    v, s = h[..., :C], h[..., C:]
    v = EMU.q((v * Z.sigmoid(s)).astype(F32))
    if key_pad is not None:
        v = np.where(key_pad[:, :, None], F32(0.0), v)
    v = Z.depthwise_conv1d(v, P["depthwise_conv.weight"], P["depthwise_conv.bias"])
    out = linear(EMU.q(Z.swoosh_r_fwd(v)), P["out_proj.weight"], P["out_proj.bias"])
    EMU.cur = prev
    return out


def _text_embed_exact(orig):
    def f(self, tokens):
        saved, EMU.fam = EMU.fam, ({} if EMU.text_exact else EMU.fam)
        try:
            return orig(self, tokens)
        finally:
            EMU.fam = saved
    return f


def install():
    Z.ZipVoiceOracle.forward_text_embed = _text_embed_exact(Z.ZipVoiceOracle.forward_text_embed)
    Z.linear = linear
    Z.attn_weights = attn_weights
    Z.feed_forward = feed_forward
    Z.nonlin_attention = nonlin_attention
    Z.self_attention = self_attention
    Z.conv_module = conv_module


def run_sample(o, d):
    fl = d["features_lens"]
    gen, _, prm, _ = o.sample(tokens_list(d["tokens"]), tokens_list(d["prompt_tokens"]),
                              d["prompt_features"], d["prompt_features_lens"], x0=d["x0"],
                              features_lens=fl if fl.size else None, speed=float(d["speed"]),
                              t_shift=float(d["t_shift"]), duration=str(d["duration"]),
                              num_step=int(d["num_step"]),
                              guidance_scale=float(d["guidance_scale"]))
    return gen, prm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r02_precision_study.txt"))
    ap.add_argument("--fixture", default="sample_c1.npz")
    ap.add_argument("--mixed", action="store_true")
    ap.add_argument("--r03", action="store_true")
    ap.add_argument("--velocity", action="store_true",
                    help="round 4: one guided velocity on the random input of tests/test_gpu_ffn.py "
                         "(B=2, T=203, lens 203/150, t=0.4, g=1, seed 11) against the exact oracle")
    args = ap.parse_args()
    from zipvoice_amd.config import default_config
    from zipvoice_amd.weights import synthetic_state_dict
    install()
    d = load(args.fixture)
    cfg = default_config(str(d["variant"]))
    o = Z.ZipVoiceOracle(cfg, synthetic_state_dict(cfg, 0))
    KEYS.update({id(v): k for k, v in o.sd.items()})
    fams = ["attn", "qk", "ff", "na", "sa", "conv", "io"]
    if args.velocity:
        base = {g: "fp16" for g in fams}
        mixed = dict(base, io=None, attn="a16")           # the engine's fp16 parity mode (r03)
        arms = [("fp16 parity mode (io fp32, attn a16, +text fp32)", mixed, True)]
        for g in ("qk", "ff", "na", "sa", "conv", "sa_in", "sa_pv", "sa_out"):
            arms.append((f"parity mode, {g} exact", dict(mixed, **{g: None}), True))
        arms.append(("parity mode, sa_pv + qk exact", dict(mixed, sa_pv=None, qk=None), True))
        arms.append(("parity mode, sa_in + sa_out exact", dict(mixed, sa_in=None, sa_out=None), True))
        arms.append(("parity mode, sa_out exact + sa_in a16", dict(mixed, sa_in="a16", sa_out=None), True))
        arms.append(("parity mode, sa_out w16 + sa_in a16", dict(mixed, sa_in="a16", sa_out="w16"), True))
        arms.append(("parity mode, sa + qk exact", dict(mixed, sa=None, qk=None), True))
        arms.append(("parity mode, sa_out + qk exact", dict(mixed, sa_out=None, qk=None), True))
        arms.append(("parity mode, na + sa_out exact", dict(mixed, na=None, sa_out=None), True))
        cand = dict(mixed, sa_in="a16", sa_out=None)
        arms.append(("cand: sa_in a16 + sa_out exact, io fp16", dict(cand, io="fp16"), True))
        arms.append(("cand: sa_in a16 + sa_out exact, io a16", dict(cand, io="a16"), True))
        arms.append(("cand: sa_in a16 + sa_out exact, io w16", dict(cand, io="w16"), True))
        arms.append(("cand: sa_in a16 + sa_out exact, attn fp16", dict(cand, attn="fp16"), True))
        arms.append(("cand: sa_in a16 + sa_out exact, text fp16", cand, False))
        arms.append(("parity mode, sa_out a16 (W split)", dict(mixed, sa_out="a16"), True))
        arms.append(("parity mode, sa_out w16 (A split)", dict(mixed, sa_out="w16"), True))
        arms.append(("parity mode, sa_in a16 (W split)", dict(mixed, sa_in="a16"), True))
        arms.append(("parity mode, attn exact", dict(mixed, attn=None), True))
        arms.append(("parity mode, text fp16", mixed, False))
        run_velocity(o, cfg, arms, args.out.replace(".txt", "_r04_velocity_T203.txt"))
        return
    if "--r03" in sys.argv:
        # cheaper parity-grade candidates: one-sided split products for the attention-score
        # projection, and dropping the text-encoder / in-out splits
        base = {g: "fp16" for g in fams}
        arms = [("io+attn fp32, rest fp16 +text fp32 (r02 mixed)", dict(base, io=None, attn=None), True),
                ("io fp32, attn w16 (A split), +text fp32", dict(base, io=None, attn="w16"), True),
                ("io fp32, attn a16 (W split), +text fp32", dict(base, io=None, attn="a16"), True),
                ("io+attn fp32, text fp16", dict(base, io=None, attn=None), False),
                ("attn fp32, io fp16, +text fp32", dict(base, attn=None), True),
                ("io w16, attn w16, +text fp32", dict(base, io="w16", attn="w16"), True)]
        run_arms(o, d, arms, args.out.replace(".txt", "_r03_" + args.fixture.replace(".npz", ".txt")))
        return
    if "--mixed" in sys.argv:
        arms = []
        base = {g: "fp16" for g in fams}
        for keep in (["io"], ["io", "attn"], ["io", "qk"], ["io", "attn", "qk"], ["io", "sa"],
                     ["io", "na"], ["io", "attn", "sa"]):
            for tx in ((False, True) if args.fixture == "sample_c1.npz" else (True,)):
                arms.append((f"{'+'.join(keep)} fp32, rest fp16{' +text fp32' if tx else ''}",
                             dict(base, **{g: None for g in keep}), tx))
        run_arms(o, d, arms, args.out.replace(".txt", "_mixed.txt" if args.fixture == "sample_c1.npz"
                                              else "_mixed_" + args.fixture.replace(".npz", ".txt")))
        return
    arms = [("fp32 (emulation off)", {})]
    arms.append(("all bf16", {f: "bf16" for f in fams}))
    arms.append(("all fp16", {f: "fp16" for f in fams}))
    for f in fams:
        arms.append((f"only {f} bf16", {f: "bf16"}))
    for f in fams:
        arms.append((f"all bf16 but {f} fp32", {g: "bf16" for g in fams if g != f}))
    for f in fams:
        arms.append((f"all fp16 but {f} bf16", {g: ("bf16" if g == f else "fp16") for g in fams}))
    # candidate mixed modes: the sensitive families fp32-accurate (bf16x3 in the engine)
    for keep in (["io"], ["io", "attn"], ["io", "attn", "sa"], ["io", "attn", "sa", "na"]):
        for fmt in ("bf16", "fp16"):
            arms.append((f"{'+'.join(keep)} fp32, rest {fmt}",
                         {g: (None if g in keep else fmt) for g in fams}))
    run_arms(o, d, [(n, f, False) for n, f in arms], args.out)


def run_velocity(o, cfg, arms, out):
    rng = np.random.default_rng(11)
    B, T = 2, 203
    x = rng.standard_normal((B, T, cfg.feat_dim), dtype=np.float32)
    tc = rng.standard_normal(x.shape, dtype=np.float32)
    sc = rng.standard_normal(x.shape, dtype=np.float32)
    pm = np.arange(T)[None] >= np.array([203, 150])[:, None]
    EMU.fam, EMU.text_exact = {}, True
    ref = o.velocity(np.float32(0.4), x, tc, sc, pm, 1.0)
    lines = ["# precision study (round 4): oracle with emulated MFMA-operand rounding; one guided "
             "velocity on tests/test_gpu_ffn.py's random input (B=2, T=203, lens 203/150, t=0.4, g=1, "
             "seed 11); metric = mean / max |v - exact oracle| over valid frames"]
    for name, fam, tx in arms:
        EMU.fam, EMU.text_exact = fam, tx
        t0 = time.time()
        v = o.velocity(np.float32(0.4), x, tc, sc, pm, 1.0)
        e = np.abs(v - ref)[~pm]
        line = f"{name:50s} mean {e.mean():.3e} max {e.max():.3e}   ({time.time() - t0:.1f} s)"
        print(line, flush=True)
        lines.append(line)
    with open(out, "w") as f:
        f.write("\n".join(lines) + "\n")


def run_arms(o, d, arms, out):
    lines = ["# precision study: oracle with emulated MFMA-operand rounding; fixture sample_c1 "
             "(reference fp32 output); metric = mean / max |gen - ref| (and prompt part)"]
    for name, fam, tx in arms:
        EMU.fam = fam
        EMU.text_exact = tx
        t0 = time.time()
        gen, prm = run_sample(o, d)
        eg = np.abs(gen - d["gen"])
        ep = np.abs(prm - d["prompt"])
        line = (f"{name:40s} gen mean {eg.mean():.3e} max {eg.max():.3e} | prompt mean "
                f"{ep.mean():.3e} max {ep.max():.3e}   ({time.time() - t0:.1f} s)")
        print(line, flush=True)
        lines.append(line)
    with open(out, "w") as f:
        f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()

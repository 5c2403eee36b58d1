"""ORACLE — test infrastructure only, never the product path.

CPU (numpy, fp32) restatement of the reference ZipVoice inference hot path,
written from the reference's semantics (each function cites the reference
file:line it follows; paths are relative to the reference repository).  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module, and only as the checker / the timed CPU baseline.

Pinned against golden fixtures produced by running the reference's own PyTorch
code in the build container (``tests/golden/make_golden.py``); see
``tests/test_oracle_golden.py``.

Layout convention: activations are (B, L, C) row-major (the reference uses
(L, B, C) inside the Zipformer; this is a layout choice, not a semantic one).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

F32 = np.float32


# ---------------------------------------------------------------------------
# activations & small primitives  (zipvoice/models/modules/scaling.py)
# ---------------------------------------------------------------------------

def swoosh_l_fwd(x: np.ndarray) -> np.ndarray:
    """SwooshLForward, scaling.py:1174-1180 (used inside FeedforwardModule.out_proj)."""
    xo = x - F32(4.0)
    with np.errstate(over="ignore"):
        ls = np.log(F32(1.0) + np.exp(xo))
    ls = np.where(np.isinf(ls), xo, ls)
    return (ls - F32(0.08) * x - F32(0.035)).astype(F32)


def swoosh_r_fwd(x: np.ndarray) -> np.ndarray:
    """SwooshRForward, scaling.py:1185-1191 (ConvolutionModule.out_proj)."""
    xo = x - F32(1.0)
    with np.errstate(over="ignore"):
        ls = np.log(F32(1.0) + np.exp(xo))
    ls = np.where(np.isinf(ls), xo, ls)
    return (ls - F32(0.08) * x - F32(0.313261687)).astype(F32)


def swoosh_r_module(x: np.ndarray) -> np.ndarray:
    """SwooshR nn.Module without k2: SwooshRFunction.forward, scaling.py:1106-1116
    (logaddexp(0, x-1) - 0.08 x - 0.313261687)."""
    return (np.logaddexp(F32(0.0), x - F32(1.0)) - F32(0.08) * x
            - F32(0.313261687)).astype(F32)


def linear(x: np.ndarray, w: np.ndarray, b: Optional[np.ndarray] = None) -> np.ndarray:
    y = np.matmul(x, w.T)
    if b is not None:
        y = y + b
    return y.astype(F32)


def bias_norm(x, bias, log_scale):
    """BiasNormFunction.forward, scaling.py:330-355: x * mean((x-b)^2)^-0.5 * exp(s)."""
    scales = np.mean((x - bias) ** 2, axis=-1, keepdims=True) ** F32(-0.5) * np.exp(
        F32(log_scale))
    return (x * scales).astype(F32)


def bypass(orig, src, scale):
    """BypassModule.forward at eval, zipformer.py:798-804."""
    return (orig + (src - orig) * scale).astype(F32)


def softmax_lastdim(x):
    m = x.max(axis=-1, keepdims=True)
    e = np.exp(x - m)
    return (e / e.sum(axis=-1, keepdims=True)).astype(F32)


def sigmoid(x):
    return (F32(1.0) / (F32(1.0) + np.exp(-x))).astype(F32)


def timestep_embedding(t: np.ndarray, dim: int, max_period: float = 10000.0) -> np.ndarray:
    """zipformer.py:47-69 (cos first, then sin)."""
    half = dim // 2
    freqs = np.exp(-math.log(max_period) * np.arange(half, dtype=F32) / F32(half)).astype(F32)
    args = t.astype(F32)[..., None] * freqs[None]
    emb = np.concatenate([np.cos(args), np.sin(args)], axis=-1).astype(F32)
    if dim % 2:
        emb = np.concatenate([emb, np.zeros_like(emb[..., :1])], axis=-1)
    return emb


def rel_pos_table(L: int, pos_dim: int) -> np.ndarray:
    """CompactRelPositionalEncoding.extend_pe + forward, zipformer.py:983-1056.

    Returns pe of shape (2L-1, pos_dim); row n encodes relative offset n-(L-1).
    """
    x = np.arange(-(L - 1), L, dtype=np.int64).astype(F32)[:, None]
    freqs = (1 + np.arange(pos_dim // 2)).astype(np.int64)
    c = pos_dim ** 0.5
    xc = (F32(c) * np.sign(x) * (np.log(np.abs(x) + F32(c)) - F32(math.log(c)))).astype(F32)
    length_scale = 1.0 * pos_dim / (2.0 * math.pi)
    xa = np.arctan(xc / F32(length_scale)).astype(F32)
    ang = (xa * freqs.astype(F32)).astype(F32)
    pe = np.zeros((x.shape[0], pos_dim), F32)
    pe[:, 0::2] = np.cos(ang)
    pe[:, 1::2] = np.sin(ang)
    pe[:, -1] = 1.0
    return pe


# ---------------------------------------------------------------------------
# Zipformer modules  (zipvoice/models/modules/zipformer.py)
# ---------------------------------------------------------------------------

class Params:
    """Thin accessor over a flat state dict with a key prefix."""

    def __init__(self, sd: Dict[str, np.ndarray], prefix: str = ""):
        self.sd, self.prefix = sd, prefix

    def __getitem__(self, k):
        return self.sd[self.prefix + k]

    def sub(self, p):
        return Params(self.sd, self.prefix + p)


def attn_weights(P: Params, x, pe, key_pad, heads, qdim, pdim):
    """RelPositionMultiheadAttentionWeights.forward, zipformer.py:1149-1306.

    x (B,L,C); pe (2L-1, pos_dim); key_pad (B,L) bool True = padded.
    Returns W (H, B, L, L)."""
    B, L, _ = x.shape
    xp = linear(x, P["in_proj.weight"], P["in_proj.bias"])
    qd = qdim * heads
    q = xp[..., :qd].reshape(B, L, heads, qdim).transpose(2, 0, 1, 3)      # H,B,L,d
    k = xp[..., qd:2 * qd].reshape(B, L, heads, qdim).transpose(2, 0, 3, 1)  # H,B,d,L
    p = xp[..., 2 * qd:].reshape(B, L, heads, pdim).transpose(2, 0, 1, 3)   # H,B,L,pd
    scores = np.matmul(q, k)                                                 # no 1/sqrt(d)
    pos = linear(pe, P["linear_pos.weight"])                                 # (2L-1, H*pd)
    pos = pos.reshape(2 * L - 1, heads, pdim).transpose(1, 2, 0)[:, None]   # H,1,pd,2L-1
    ps = np.matmul(p, pos)                                                   # H,B,L,2L-1
    # as_strided (zipformer.py:1239-1248): out[i,j] = ps[i, L-1-i+j]
    i = np.arange(L)[:, None]
    j = np.arange(L)[None, :]
    scores = scores + ps[:, :, i, L - 1 - i + j]
    if key_pad is not None:
        scores = np.where(key_pad[None, :, None, :], F32(-1000.0), scores)   # :1281-1289
    return softmax_lastdim(scores.astype(F32))


def feed_forward(P: Params, x):
    """FeedforwardModule.forward, zipformer.py:1433-1439 (+ scaling.py:1322-1334)."""
    h = linear(x, P["in_proj.weight"], P["in_proj.bias"])
    return linear(swoosh_l_fwd(h), P["out_proj.weight"], P["out_proj.bias"])


def nonlin_attention(P: Params, x, w0):
    """NonlinAttention.forward, zipformer.py:1499-1544; w0 (B,L,L) = head 0."""
    h = linear(x, P["in_proj.weight"], P["in_proj.bias"])
    hid = h.shape[-1] // 3
    s, v, y = h[..., :hid], h[..., hid:2 * hid], h[..., 2 * hid:]
    v = (v * np.tanh(s)).astype(F32)
    v = np.matmul(w0, v).astype(F32)
    v = (v * y).astype(F32)
    return linear(v, P["out_proj.weight"], P["out_proj.bias"])


def self_attention(P: Params, x, W, vdim):
    """SelfAttention.forward, zipformer.py:1359-1396; W (H,B,L,L)."""
    B, L, _ = x.shape
    H = W.shape[0]
    v = linear(x, P["in_proj.weight"], P["in_proj.bias"]).reshape(B, L, H, vdim)
    v = v.transpose(2, 0, 1, 3)                                             # H,B,L,d
    o = np.matmul(W, v).transpose(1, 2, 0, 3).reshape(B, L, H * vdim).astype(F32)
    return linear(o, P["out_proj.weight"], P["out_proj.bias"])


def depthwise_conv1d(x, w, b):
    """nn.Conv1d(groups=C, padding=k//2) on (B,L,C) layout; w (C,1,k)."""
    B, L, C = x.shape
    k = w.shape[-1]
    pad = k // 2
    xp = np.zeros((B, L + 2 * pad, C), F32)
    xp[:, pad:pad + L] = x
    out = np.zeros((B, L, C), F32)
    for t in range(k):
        out += xp[:, t:t + L, :] * w[:, 0, t]
    return (out + b).astype(F32)


def conv_module(P: Params, x, key_pad):
    """ConvolutionModule.forward, zipformer.py:1638-1680."""
    h = linear(x, P["in_proj.weight"], P["in_proj.bias"])
    C = h.shape[-1] // 2
    v, s = h[..., :C], h[..., C:]
    v = (v * sigmoid(s)).astype(F32)
    if key_pad is not None:
        v = np.where(key_pad[:, :, None], F32(0.0), v)                       # :1669-1670
    v = depthwise_conv1d(v, P["depthwise_conv.weight"], P["depthwise_conv.bias"])
    return linear(swoosh_r_fwd(v), P["out_proj.weight"], P["out_proj.bias"])


def encoder_layer(P: Params, src, pe, temb, key_pad, dims):
    """Zipformer2EncoderLayer.forward at inference, zipformer.py:489-642."""
    heads, qdim, pdim, vdim = dims
    src_orig = src
    W = attn_weights(P.sub("self_attn_weights."), src, pe, key_pad, heads, qdim, pdim)
    if temb is not None:
        src = src + temb
    src = src + feed_forward(P.sub("feed_forward1."), src)
    src = src + nonlin_attention(P.sub("nonlin_attention."), src, W[0])
    src = src + self_attention(P.sub("self_attn1."), src, W, vdim)
    if temb is not None:
        src = src + temb
    src = src + conv_module(P.sub("conv_module1."), src, key_pad)
    src = src + feed_forward(P.sub("feed_forward2."), src)
    src = bypass(src_orig, src, P["bypass_mid.bypass_scale"])
    src = src + self_attention(P.sub("self_attn2."), src, W, vdim)
    if temb is not None:
        src = src + temb
    src = src + conv_module(P.sub("conv_module2."), src, key_pad)
    src = src + feed_forward(P.sub("feed_forward3."), src)
    src = bias_norm(src, P["norm.bias"], P["norm.log_scale"])
    return bypass(src_orig, src, P["bypass.bypass_scale"]).astype(F32)


def zipformer_encoder(P: Params, src, temb, key_pad, num_layers, dims, pos_dim):
    """Zipformer2Encoder.forward, zipformer.py:702-744."""
    L = src.shape[1]
    pe = rel_pos_table(L, pos_dim)
    te = None
    if temb is not None:
        te = linear(swoosh_r_module(temb), P["time_emb.1.weight"], P["time_emb.1.bias"])
        te = te[:, None, :]
    for li in range(num_layers):
        src = encoder_layer(P.sub(f"layers.{li}."), src, pe, te, key_pad, dims)
    return src


def downsampled_encoder(P: Params, src, temb, key_pad, ds, num_layers, dims, pos_dim):
    """DownsampledZipformer2Encoder.forward, zipformer.py:823-870 with
    SimpleDownsample :887-913 and SimpleUpsample :925-935."""
    B, L, C = src.shape
    dL = (L + ds - 1) // ds
    pad = dL * ds - L
    xs = src
    if pad:
        xs = np.concatenate([src, np.repeat(src[:, -1:], pad, axis=1)], axis=1)
    wts = softmax_lastdim(P["downsample.bias"].astype(F32)[None])[0]
    xs = xs.reshape(B, dL, ds, C)
    d = (xs * wts[None, None, :, None]).sum(axis=2).astype(F32)
    kp = key_pad[:, ::ds] if key_pad is not None else None
    d = zipformer_encoder(P.sub("encoder."), d, temb, kp, num_layers, dims, pos_dim)
    up = np.repeat(d, ds, axis=1)[:, :L]
    return bypass(src, up, P["out_combiner.bypass_scale"])


def tts_zipformer(P: Params, x, t, key_pad, cfg_dims, guidance=None, stream=None):
    """TTSZipformer.forward, zipformer.py:242-293 (two-stream variant:
    zipformer_two_stream.py:219-264, projection pair chosen by input width)."""
    (factors, layers, heads, qdim, pdim, vdim, pos_dim, temb_dim) = cfg_dims
    dims = (heads, qdim, pdim, vdim)
    if stream is None:
        src = linear(x, P["in_proj.weight"], P["in_proj.bias"])
    else:
        src = linear(x, P[f"in_proj.{stream}.weight"], P[f"in_proj.{stream}.bias"])
    temb = None
    if t is not None:
        temb = timestep_embedding(t, temb_dim)
        if guidance is not None:
            temb = temb + linear(timestep_embedding(guidance, temb_dim),
                                 P["guidance_scale_embed.weight"])
        temb = linear(temb, P["time_embed.0.weight"], P["time_embed.0.bias"])
        temb = linear(swoosh_r_module(temb), P["time_embed.2.weight"], P["time_embed.2.bias"])
    for s, ds in enumerate(factors):
        if ds == 1:
            src = zipformer_encoder(P.sub(f"encoders.{s}."), src, temb, key_pad,
                                    layers[s], dims, pos_dim)
        else:
            src = downsampled_encoder(P.sub(f"encoders.{s}."), src, temb, key_pad, ds,
                                      layers[s], dims, pos_dim)
    if stream is None:
        return linear(src, P["out_proj.weight"], P["out_proj.bias"])
    return linear(src, P[f"out_proj.{stream}.weight"], P[f"out_proj.{stream}.bias"])


# ---------------------------------------------------------------------------
# host helpers  (zipvoice/utils/common.py)
# ---------------------------------------------------------------------------

def make_pad_mask(lengths: np.ndarray, max_len: int = 0) -> np.ndarray:
    """common.py:395-420 (True = padded)."""
    max_len = max(int(max_len), int(lengths.max()))
    return np.arange(max_len)[None, :] >= lengths[:, None]


def pad_labels(y: List[List[int]], pad_id: int) -> np.ndarray:
    """common.py:255-268: append ONE pad to every row, then pad to max length."""
    y = [list(t) + [pad_id] for t in y]
    n = max(len(t) for t in y)
    return np.array([t + [pad_id] * (n - len(t)) for t in y], dtype=np.int64)


def get_tokens_index(features_lens, tokens_lens, num_frames: int) -> np.ndarray:
    """prepare_avg_tokens_durations + get_tokens_index, common.py:246-252, :271-295."""
    B = len(features_lens)
    ans = np.zeros((B, num_frames), np.int64)
    for b in range(B):
        S = int(tokens_lens[b])
        d = int(features_lens[b]) // S
        durs = [d] * S
        durs.append(num_frames - sum(durs))
        cur = 0
        for i, dd in enumerate(durs):
            ans[b, cur:cur + dd] = i
            cur += dd
        assert cur == num_frames
    return ans


def linspace_f32(start: float, end: float, steps: int) -> np.ndarray:
    """torch.linspace(start, end, steps) in float32 (ATen CPU kernel: forward from
    start for the first half, backward from end for the second)."""
    if steps == 1:
        return np.array([start], F32)
    step = F32((F32(end) - F32(start)) / F32(steps - 1))
    out = np.empty(steps, F32)
    half = steps // 2
    for i in range(steps):
        if i < half:
            out[i] = F32(start) + step * F32(i)
        else:
            out[i] = F32(end) - step * F32(steps - i - 1)
    return out


def get_time_steps(t_start=0.0, t_end=1.0, num_step=10, t_shift=1.0) -> np.ndarray:
    """solver.py:256-281."""
    ts = linspace_f32(t_start, t_end, num_step + 1)
    return (F32(t_shift) * ts / (F32(1.0) + F32(t_shift - 1) * ts)).astype(F32)


# ---------------------------------------------------------------------------
# model wrappers  (zipvoice/models/zipvoice*.py, solver.py)
# ---------------------------------------------------------------------------

class ZipVoiceOracle:
    """fp32 CPU restatement of ZipVoice / -Distill / -Dialog / -DialogStereo inference."""

    def __init__(self, cfg, state_dict: Dict[str, np.ndarray]):
        self.cfg = cfg
        self.sd = {k: np.asarray(v, F32) for k, v in state_dict.items()}
        self.P = Params(self.sd)

    # -- decoder -------------------------------------------------------------
    def _dec_dims(self):
        c = self.cfg
        return (c.fm_decoder_downsampling_factor, c.fm_decoder_num_layers,
                c.fm_decoder_num_heads, c.query_head_dim, c.pos_head_dim, c.value_head_dim,
                c.pos_dim, c.time_embed_dim)

    def forward_fm_decoder(self, t, xt, text_condition, speech_condition, padding_mask,
                           guidance_scale=None):
        """ZipVoice.forward_fm_decoder, zipvoice.py:135-185.  t: scalar or (N,)."""
        x = np.concatenate([xt, text_condition, speech_condition], axis=2).astype(F32)
        N = x.shape[0]
        t = np.broadcast_to(np.asarray(t, F32), (N,)).copy()
        g = None
        if guidance_scale is not None:
            g = np.broadcast_to(np.asarray(guidance_scale, F32), (N,)).copy()
        stream = None
        if self.cfg.stereo:
            stream = 0 if x.shape[2] == self.cfg.decoder_in_dims()[0] else 1
        P = self.P.sub("fm_decoder.")
        # the per-stack conv kernel size is carried by the depthwise weight shape
        return tts_zipformer(P, x, t, padding_mask, self._dec_dims(), guidance=g,
                             stream=stream)

    # -- text side -----------------------------------------------------------
    def forward_text_embed(self, tokens: List[List[int]]):
        """zipvoice.py:187-212 (+ ZipVoiceDialog override zipvoice_dialog.py:127-159)."""
        c = self.cfg
        tp = pad_labels(tokens, c.pad_id)
        emb = self.sd["embed.weight"][tp]
        lens = np.array([len(t) for t in tokens], np.int64)
        kp = make_pad_mask(lens, tp.shape[1])
        dims = ([1], [c.text_encoder_num_layers], c.text_encoder_num_heads, c.query_head_dim,
                c.pos_head_dim, c.value_head_dim, c.pos_dim, -1)
        out = tts_zipformer(self.P.sub("text_encoder."), emb, None, kp, dims)
        if c.dialog:
            turn = ((tp == c.spk_a_id) | (tp == c.spk_b_id)).astype(np.int64)
            spk = np.cumsum(turn, axis=1) % 2
            spk = np.where(tp == c.pad_id, -1, spk)
            se = self.sd["spk_embed.weight"]
            out = out + (spk == 0)[..., None] * se[0] + (spk == 1)[..., None] * se[1]
            out = out.astype(F32)
        return out, lens

    def forward_text_condition(self, embed, tokens_lens, features_lens):
        """zipvoice.py:214-251."""
        num_frames = int(features_lens.max())
        pm = make_pad_mask(features_lens, num_frames)
        idx = get_tokens_index(features_lens, tokens_lens, num_frames)
        tc = np.take_along_axis(embed, idx[..., None], axis=1)
        return tc.astype(F32), pm

    @staticmethod
    def predict_features_lens(prompt_features_lens, prompt_tokens_lens, tokens_lens, speed):
        """zipvoice.py:323-325 in float32 (int64/int64 true-division -> float32)."""
        pf = prompt_features_lens.astype(F32)
        r = pf / prompt_tokens_lens.astype(F32) * tokens_lens.astype(F32) / F32(speed)
        return prompt_features_lens + np.ceil(r).astype(np.int64)

    def text_condition_predict(self, tokens, prompt_tokens, prompt_features_lens, speed):
        """forward_text_inference_ratio_duration, zipvoice.py:290-330."""
        cat = [list(p) + list(t) for p, t in zip(prompt_tokens, tokens)]
        ptl = np.array([len(t) for t in prompt_tokens], np.int64)
        tl = np.array([len(t) for t in tokens], np.int64)
        emb, ctl = self.forward_text_embed(cat)
        fl = self.predict_features_lens(np.asarray(prompt_features_lens, np.int64), ptl, tl,
                                        speed)
        return self.forward_text_condition(emb, ctl, fl)

    def text_condition_real(self, tokens, features_lens, prompt_tokens, prompt_features_lens):
        """forward_text_inference_gt_duration, zipvoice.py:270-288."""
        cat = [list(p) + list(t) for p, t in zip(prompt_tokens, tokens)]
        fl = np.asarray(prompt_features_lens, np.int64) + np.asarray(features_lens, np.int64)
        emb, ctl = self.forward_text_embed(cat)
        return self.forward_text_condition(emb, ctl, fl)

    # -- solver --------------------------------------------------------------
    def velocity(self, t, x, text_c, speech_c, pm, guidance_scale):
        """DiffusionModel.forward / DistillDiffusionModel.forward, solver.py:40-165."""
        g = F32(guidance_scale)
        if self.cfg.distill:
            return self.forward_fm_decoder(t, x, text_c, speech_c, pm, guidance_scale=g)
        if g == 0.0:
            return self.forward_fm_decoder(t, x, text_c, speech_c, pm)
        x2 = np.concatenate([x, x], 0)
        pm2 = np.concatenate([pm, pm], 0)
        tc2 = np.concatenate([np.zeros_like(text_c), text_c], 0)
        if float(t) > 0.5:
            sc2 = np.concatenate([np.zeros_like(speech_c), speech_c], 0)
        else:
            g = F32(g * F32(2.0))
            sc2 = np.concatenate([speech_c, speech_c], 0)
        v = self.forward_fm_decoder(t, x2, tc2, sc2, pm2)
        B = x.shape[0]
        vu, vc = v[:B], v[B:]
        return ((F32(1.0) + g) * vc - g * vu).astype(F32)

    def euler(self, x0, text_c, speech_c, pm, num_step, guidance_scale, t_start=0.0,
              t_end=1.0, t_shift=1.0):
        """EulerSolver.sample, solver.py:182-240."""
        ts = get_time_steps(t_start, t_end, num_step, t_shift)
        x = x0.astype(F32)
        for k in range(num_step):
            v = self.velocity(ts[k], x, text_c, speech_c, pm, guidance_scale)
            x = (x + v * (ts[k + 1] - ts[k])).astype(F32)
        return x

    def sample(self, tokens, prompt_tokens, prompt_features, prompt_features_lens,
               x0=None, features_lens=None, speed=1.0, t_shift=1.0, duration="predict",
               num_step=5, guidance_scale=0.5, seed=0):
        """ZipVoice.sample, zipvoice.py:388-486, with x0 supplied explicitly."""
        pfl = np.asarray(prompt_features_lens, np.int64)
        if duration == "predict":
            tc, pm = self.text_condition_predict(tokens, prompt_tokens, pfl, speed)
        else:
            tc, pm = self.text_condition_real(tokens, features_lens, prompt_tokens, pfl)
        B, T, _ = tc.shape
        F = prompt_features.shape[-1]
        sc = np.zeros((B, T, F), F32)
        n = min(T, prompt_features.shape[1])
        sc[:, :n] = prompt_features[:, :n]
        sc = np.where(make_pad_mask(pfl, T)[..., None], F32(0.0), sc).astype(F32)
        if x0 is None:
            x0 = np.random.default_rng(seed).standard_normal((B, T, F), dtype=F32)
        x1 = self.euler(x0, tc, sc, pm, num_step, guidance_scale, t_shift=t_shift)
        gen_lens = (~pm).sum(-1) - pfl
        gen = np.zeros((B, int(gen_lens.max()), F), F32)
        prm = np.zeros((B, int(pfl.max()), F), F32)
        for i in range(B):
            gen[i, :gen_lens[i]] = x1[i, pfl[i]:pfl[i] + gen_lens[i]]
            prm[i, :pfl[i]] = x1[i, :pfl[i]]
        return gen, gen_lens, prm, pfl

#!/usr/bin/env python3
"""Algorithmic FLOPs of the flow-matching decoder path per guided Euler step, and the path
roofline of a measured step time: the reference's arithmetic (zipformer.py:489-642 per layer),
not what the kernels execute (the fused attention consumers recompute scores per consumer; the
CFG rows are counted, the padding rows of a ragged batch are not).

Per layer and frame of a stack at L frames (D = 512, heads H = 4, query / pos / value head dims
32 / 4 / 12, FF hidden 3/4, 1, 5/4 x feedforward_dim, NonlinAttention hidden 3/4 D):
  feed-forward x3      4 D (F1 + F2 + F3)                       (in + out projections)
  attention weights    2 D H (2 qd + pd)  +  H L (2 qd + 2 pd)   (projection, q.k + positional)
  NonlinAttention      2 D 3 h + 2 h D  +  2 h L                 (in / out projections, P.V)
  SelfAttention x2     2 (2 D H vd + 2 H vd D)  +  2 (2 H vd L)   (projections, P.V)
  ConvolutionModule x2 2 (2 D 2D + 2 D D + 2 k D)                (in / out projections, depthwise)
The text encoder, the stack time embeddings, the down / upsampling and the vocoder are < 1 %
of a C2 step and are left out (the roofline is then a slight under-estimate).

usage: path_flops.py CONFIG MS_PER_STEP [peak TFLOP/s, default 2500 (bf16 dense)]"""
import sys

CONFIGS = {   # rows per decoder pass (CFG doubles), frames, Euler steps per sample()
    "C2": dict(variant="zipvoice", rows=64, T=1219, N=16),
    "C3": dict(variant="zipvoice_distill", rows=16, T=1219, N=8),
    "C4": dict(variant="zipvoice_dialog", rows=32, T=3376, N=16),
    "C5": dict(variant="zipvoice_dialog_stereo", rows=8, T=3376, N=16),
}


def layer_flops(L, D=512, H=4, qd=32, pd=4, vd=12, ff=1536, k=31):
    f1, f2, f3 = ff * 3 // 4, ff, ff * 5 // 4
    h = D * 3 // 4
    per_frame = (4 * D * (f1 + f2 + f3)
                 + 2 * D * H * (2 * qd + pd) + H * L * (2 * qd + 2 * pd)
                 + 2 * D * 3 * h + 2 * h * D + 2 * h * L
                 + 2 * (2 * D * H * vd + 2 * H * vd * D) + 2 * (2 * H * vd * L)
                 + 2 * (2 * D * 2 * D + 2 * D * D + 2 * k * D))
    return per_frame


def decoder_flops(rows, T, ds=(1, 2, 4, 2, 1), layers=(2, 2, 4, 4, 4), kernels=(31, 15, 7, 15, 31)):
    tot = 0.0
    for d, nl, k in zip(ds, layers, kernels):
        L = (T + d - 1) // d
        tot += nl * rows * L * layer_flops(L, k=k)
    return tot


def main():
    name = sys.argv[1]
    ms = float(sys.argv[2])
    peak = float(sys.argv[3]) if len(sys.argv) > 3 else 2500.0
    c = CONFIGS[name]
    fl = decoder_flops(c["rows"], c["T"]) * c["N"]
    tf = fl / (ms * 1e-3) / 1e12
    print(f"{name}: {fl / 1e12:.2f} TFLOP per step ({c['N']} decoder passes of {c['rows']} x {c['T']}), "
          f"{ms:.1f} ms -> {tf:.0f} TFLOP/s = {tf / peak:.3f} of {peak:.0f}")


if __name__ == "__main__":
    main()

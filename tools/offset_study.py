#!/usr/bin/env python3
"""Which per-query offset keeps the fp16 second-generation attention in range (study, CPU only).

The fp16 parity mode's attention consumers (zv_flash2.inc, FA2_OFS) take p = 2^(s - o) with
o = ceil(max of the query's scores over ONE key step) and send a wave / block to the exact path
when some later score rises 16 or more above o (p overflows fp16).  Every such unit costs one
more block-time on its CU.  This script runs the numpy oracle (oracle/zipvoice_np.py) on one
guided velocity at the C2 shape with the bench's synthetic weights, records every layer's
attention weights W (the softmax of the scores: log2 W_ij - log2 W_ik = s_ij - s_ik in base 2,
so offsets can be judged from W alone) and counts, per candidate key set for the offset, the
queries / SelfAttention waves / NonlinAttention blocks that would overflow.

    python tools/offset_study.py [T]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import oracle.zipvoice_np as onp  # noqa: E402
from zipvoice_amd.config import default_config  # noqa: E402
from zipvoice_amd.weights import synthetic_state_dict  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 1219
SA_KS, NA_KS = 64, 32          # key step of sa2 / sa3 and of na2
SA_WAVE, NA_BLOCK = 64, 128    # queries per SelfAttention wave (sa3<4>) / NonlinAttention block
records = []
orig = onp.attn_weights


def capture(P, x, pe, key_pad, heads, qdim, pdim):
    W = orig(P, x, pe, key_pad, heads, qdim, pdim)
    records.append(W.copy())
    return W


onp.attn_weights = capture
cfg = default_config("zipvoice")
o = onp.ZipVoiceOracle(cfg, synthetic_state_dict(cfg, 0))
rng = np.random.default_rng(7)
x = rng.standard_normal((1, T, 100), dtype=np.float32)
tc = rng.standard_normal((1, T, 100), dtype=np.float32)
sc = rng.standard_normal((1, T, 100), dtype=np.float32)
o.velocity(np.float32(0.3), x, tc, sc, np.zeros((1, T), bool), 1.0)


def overflow(lw, ks, keysets):
    """lw (Q, L) log2 weights; for each query the offset o = ceil(max over keysets(q)) in the
    score frame where the query's maximum is 0 (shift-invariant up to the ceil's phase, taken
    at its worst: an offset at the lower integer); overflow when max - o >= 16."""
    Q, L = lw.shape
    ns = (L + ks - 1) // ks
    pad = np.full((Q, ns * ks), -np.inf)
    pad[:, :L] = lw
    stepmax = pad.reshape(Q, ns, ks).max(axis=2)
    qs = np.arange(Q)
    sel = np.full(Q, -np.inf)
    for ks_fn in keysets:
        sel = np.maximum(sel, stepmax[qs, ks_fn(qs, L) // ks])
    return (lw.max(axis=1) - sel) >= 15.0          # ceil adds [0, 1): count the worst case


def strategies(ks):
    step0 = lambda q, L: 0 * q                                                # noqa: E731
    diag = lambda q, L: np.minimum((q // ks) * ks, ((L - 1) // ks) * ks)      # noqa: E731
    last = lambda q, L: 0 * q + ((L - 1) // ks) * ks                          # noqa: E731
    return {"step0": [step0], "step0+diag": [step0, diag], "step0+diag+last": [step0, diag, last],
            "diag": [diag]}


tot = {}
for W in records:                       # (H, B, L, L)
    H, B, L, _ = W.shape
    lw_all = np.log2(np.maximum(W.astype(np.float64), 1e-300))
    for h in range(H):
        for b in range(B):
            lw = lw_all[h, b]
            for kind, ks, unit in (("SA", SA_KS, SA_WAVE), ("NA", NA_KS, NA_BLOCK)):
                if kind == "NA" and h != 0:
                    continue
                for name, kset in strategies(ks).items():
                    ov = overflow(lw, ks, kset)
                    nunit = (L + unit - 1) // unit
                    units = sum(ov[u * unit:(u + 1) * unit].any() for u in range(nunit))
                    t = tot.setdefault((kind, L, name), [0, 0, 0, 0])
                    t[0] += int(ov.sum()); t[1] += L; t[2] += int(units); t[3] += nunit
print(f"# T={T}, one guided velocity (t=0.3, CFG rows 2), synthetic weights (seed 0); "
      f"{len(records)} attention-weight sets")
print(f"{'consumer':8s} {'L':>5s} {'offset from':18s} {'queries over':>14s} {'units over':>14s}")
for (kind, L, name), (nq, qt, nu, ut) in sorted(tot.items()):
    print(f"{kind:8s} {L:5d} {name:18s} {nq:7d}/{qt:<7d} {nu:6d}/{ut:<6d}")

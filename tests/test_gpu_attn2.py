"""The second-generation attention consumers (csrc/zv_flash2.inc: the bf16 / fp8 engines' default
SelfAttention and NonlinAttention) pinned at their own precision, fast path and exact path.

Those kernels take p = 2^s with no running maximum and send a wave (SelfAttention) or block
(NonlinAttention) whose range check fails -- a query denominator outside [2^-60, 2^100] or a
non-finite accumulator -- through an exact path with the row maximum subtracted
(zv_flash2.inc; the reference's softmax, zipformer.py:1257-1306 with masked_fill(-1000) at
:1281-1289; SelfAttention :1359-1396, NonlinAttention :1499-1544).

1. Kernel level (zv_attn2_check, through the C ABI): each kernel form against a float64 softmax of
   the same bf16-rounded operands, for normal scores, with every wave / block forced onto the exact
   path, and with per-query score shifts of +-320 (base 2) that straddle both range edges, with a
   ragged (padded-key) second utterance.  Bound, written here: |out - ref| <= 6e-3 * sum_j w|v| |y|
   + 4e-3 |ref| + 1e-6 per element -- the bf16 rounding of p (2^-9 relative, numerator and
   denominator) and of the output (2^-9), with a 1.5x margin.  A wrong row, block or wave is
   orders of magnitude outside it.
2. Engine level (C ABI velocity, ragged B = 2 at the C2 / C4 lengths): ZV_ATTN2=1 against the
   first-generation consumers (ZV_ATTN2=0), the forced exact path (ZV_ATTN2_EXACT=1) against the
   fast path, the bf16 materialising fallback (ZV_ATTN_MATERIALIZE=1, the path the engine takes
   where the fused images do not fit) against the fused one, and q / p rows scaled x8 so that part
   of the waves take the exact path.  Any bf16 perturbation of attention reaches the velocity at
   the bf16 noise level (the measured pairwise differences, tools/attn2_probe.py /
   profiles/r06_attn2_probe.txt: mean 7.7e-3 .. 9.1e-3, max 4.8e-2 .. 6.1e-2), so these bounds are
   ~1.6x the measured difference, not the 5e-2 model bar.
"""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

LOG2E = 1.4426950408889634
MASKED = -1000.0 * LOG2E
H, QD, PD = 4, 32, 4


def rounded(a, operand):
    dt = torch.bfloat16 if operand == "bf16" else torch.float16
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dt).float().numpy()


def make_inputs(B, L, kernel, nv, seed, straddle=False, ragged=True, operand="bf16", diagonal=False):
    rng = np.random.default_rng(seed)
    q = 0.5 * rng.standard_normal((B, L, H, QD))
    k = 0.5 * rng.standard_normal((B, L, H, QD))
    p = 0.5 * rng.standard_normal((B, L, H, PD))
    if straddle:
        # per-query shift r_i * 8 of the scores (k dim 31 constant 8, q dim 31 = r_i): chunks of
        # 128 queries at 0 / +40 / -40 / 0 ...: denominators 2^320 and 2^-320 beside normal ones
        # (a NonlinAttention block holds at most 128 queries, a SelfAttention wave at most 64).
        # fp16 operands: the kernels' per-query offset (the maximum over the first key step and
        # the step holding the query's own tile) absorbs a shift of every key, so there only keys
        # 64..127 are shifted -- in neither of those steps for the queries of the +40 / -40 chunks:
        # the +40 chunks' scores there rise 320 above the offset (overflow -> the exact path), the
        # -40 chunks' fall 320 below it (their weights vanish, correctly, on the fast path)
        k[..., 31] = 8.0
        if operand != "bf16":
            k[..., 31] = 0.0
            k[:, 64:128, :, 31] = 8.0
        r = np.array([0.0, 40.0, -40.0, 0.0])[(np.arange(L) // 128) % 4]
        q[..., 31] = r[None, :, None]
    if diagonal:
        # the +40 chunks' queries score +320 on their OWN chunk's keys only (k dim 31 = 8 there):
        # the fp16 offsets take the step holding the query tile, so no unit overflows there (with
        # the first step alone every +40 unit would); other queries' weights on those keys vanish.
        # bf16 has no offsets: the same chunks' denominators reach 2^320 (high edge)
        chunk = (np.arange(L) // 128) % 4
        k[..., 31] = np.where(chunk == 1, 8.0, 0.0)[None, :, None]
        q[..., 31] = np.array([0.0, 40.0, -40.0, 0.0])[chunk][None, :, None]
    qkp = np.concatenate([q.reshape(B, L, H * QD), k.reshape(B, L, H * QD), p.reshape(B, L, H * PD)], -1)
    P = 0.5 * rng.standard_normal((2 * L - 1, H * PD))
    pad = np.zeros((B, L), np.uint8)
    if ragged and B > 1:
        pad[1, int(L * 0.82):] = 1
    if kernel == 0:
        v = rng.standard_normal((B, L, H * nv))
        y = None
    else:
        v = rng.standard_normal((B, L, nv))
        y = rng.standard_normal((B, L, nv))
    return [rounded(a, operand) if a is not None else None for a in (qkp, P, v, y)] + [pad]


def reference(qkp, P, v, y, pad, kernel, nv):
    """float64 softmax attention of the bf16-rounded operands (oracle/zipvoice_np.py attn_weights
    in base 2); returns (out, sum_j w |v| |y|) per element."""
    B, L, _ = qkp.shape
    out = np.zeros((B, L, H * nv if kernel == 0 else nv))
    mag = np.zeros_like(out)
    i = np.arange(L)[:, None]
    j = np.arange(L)[None, :]
    heads = range(H) if kernel == 0 else [0]
    for b in range(B):
        for h in heads:
            q = qkp[b, :, h * QD:(h + 1) * QD].astype(np.float64)
            kk = qkp[b, :, H * QD + h * QD:H * QD + (h + 1) * QD].astype(np.float64)
            pp = qkp[b, :, 2 * H * QD + h * PD:2 * H * QD + (h + 1) * PD].astype(np.float64)
            ps = pp @ P[:, h * PD:(h + 1) * PD].astype(np.float64).T          # (L, 2L-1)
            s = q @ kk.T + ps[i, L - 1 - i + j]
            s = np.where(pad[b][None, :] != 0, MASKED, s)
            s -= s.max(1, keepdims=True)
            w = np.exp2(s)
            w /= w.sum(1, keepdims=True)
            if kernel == 0:
                vv = v[b, :, h * nv:(h + 1) * nv].astype(np.float64)
                out[b, :, h * nv:(h + 1) * nv] = w @ vv
                mag[b, :, h * nv:(h + 1) * nv] = w @ np.abs(vv)
            else:
                vv = v[b].astype(np.float64)
                out[b] = (w @ vv) * y[b]
                mag[b] = (w @ np.abs(vv)) * np.abs(y[b])
    return out, mag


def run_check(kernel, form, qkp, P, v, y, pad, nv, force_exact, operand="bf16"):
    from zipvoice_amd import engine
    lib = engine.load_library(operand="f16" if operand == "f16" else "bf16")
    B, L, _ = qkp.shape
    out = np.zeros((B, L, H * nv if kernel == 0 else nv), np.float32)
    cnt = (ctypes.c_int64 * 3)()
    c = lambda a: None if a is None else np.ascontiguousarray(a, np.float32).ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    keep = [np.ascontiguousarray(a, np.float32) if a is not None else None for a in (qkp, P, v, y)]
    rc = lib.zv_attn2_check(kernel, form, B, L, H, nv, c(keep[0]), c(keep[1]),
                            np.ascontiguousarray(pad).ctypes.data_as(ctypes.c_void_p), c(keep[2]), c(keep[3]),
                            int(force_exact), out.ctypes.data_as(ctypes.c_void_p),
                            ctypes.cast(cnt, ctypes.c_void_p))
    if rc != 0:
        raise RuntimeError(lib.zv_last_error().decode())
    return out, tuple(int(x) for x in cnt)


def check_bound(out, ref, mag, what):
    assert np.isfinite(out).all(), what
    err = np.abs(out - ref)
    bound = 6e-3 * mag + 4e-3 * np.abs(ref) + 1e-6
    ratio = (err / bound).max()
    print(f"{what}: max |err| {err.max():.3e}, mean {err.mean():.3e}, max err/bound {ratio:.3f}")
    assert ratio <= 1.0, (what, ratio, np.unravel_index(np.argmax(err / bound), err.shape))


# (kernel, form, L): every form the engine launches, at lengths where it is the engine's choice
# (form 0) and forced (the long-sequence forms at C4's 3376 frames)
SA_CASES = [(0, 1, 305), (0, 3, 610), (0, 5, 1219), (0, 2, 1219), (0, 4, 1688), (0, 2, 3376), (0, 4, 3376)]
NA_CASES = [(1, 1, 305), (1, 1, 844), (1, 2, 1219), (1, 2, 3376)]
NA_BLOCK_Q = {1: 64, 2: 128}


def units(kernel, form, B, L):
    """exact-path units of a launch: SelfAttention waves (4 per block), NonlinAttention blocks"""
    if kernel == 0:
        qpw = {1: 2, 2: 3, 3: 2, 4: 3, 5: 4}[form]
        return 4 * H * B * -(-L // (64 * qpw))
    return B * -(-L // NA_BLOCK_Q[form])


@pytest.mark.parametrize("operand", ["bf16", "f16"])
@pytest.mark.parametrize("regime", ["normal", "forced", "straddle", "diagonal"])
@pytest.mark.parametrize("case", SA_CASES + NA_CASES, ids=lambda c: f"{'SA' if c[0] == 0 else 'NA'}-f{c[1]}-L{c[2]}")
def test_attn2_kernel_vs_float64(case, regime, operand):
    """operand f16: the same kernels in libzipvoice_hip_f16.so (the fp16 parity mode's decoder), with
    the per-query offsets (zv_flash2.inc FA2_OFS)."""
    kernel, form, L = case
    nv = 12 if kernel == 0 else 384
    B = 2
    qkp, P, v, y, pad = make_inputs(B, L, kernel, nv, seed=L * 10 + form, straddle=regime == "straddle",
                                    operand=operand, diagonal=regime == "diagonal",
                                    # (diagonal: both utterances unpadded -- a padded utterance's
                                    # tail queries have a masked diagonal step, so their offsets
                                    # come from step 0 and another +40 chunk's keys overflow them)
                                    ragged=regime != "diagonal")
    out, cnt = run_check(kernel, form, qkp, P, v, y, pad, nv, force_exact=regime == "forced", operand=operand)
    ref, mag = reference(qkp, P, v, y, pad, kernel, nv)
    n = units(kernel, form, B, L)
    print(f"{case} {regime} [{operand}]: exact-path runs (low, high, all) = {cnt} of {n}")
    check_bound(out, ref, mag, f"{case} {regime} [{operand}]")
    if regime == "normal":
        assert cnt == (0, 0, 0), cnt
    elif regime == "forced":
        assert cnt[2] == n and cnt[0] == cnt[1] == 0, (cnt, n)
    elif regime == "diagonal":
        if operand == "bf16":
            assert cnt[1] > 0 and cnt[2] < n, (cnt, n)
        elif kernel == 0 and form in (2, 4):
            # 48-query waves: a wave straddling a chunk edge takes its offset from the step of its
            # first tile, outside the shifted chunk (exact path, counted)
            assert cnt[2] < n, (cnt, n)
        else:
            assert cnt == (0, 0, 0), cnt
    elif operand == "bf16":
        # both edges fire, and the waves / blocks of the unshifted chunks stay on the fast path
        assert cnt[0] > 0 and cnt[1] > 0 and cnt[2] < n, (cnt, n)
    else:
        assert cnt[1] > 0 and cnt[2] < n, (cnt, n)


# ---------------------------------------------------------------------------------------------
# engine level
# ---------------------------------------------------------------------------------------------
def scaled_scores_sd(cfg, sd, S):
    """q and p rows (and biases) of every decoder attention-score projection times S."""
    out = dict(sd)
    for k in sd:
        if k.startswith("fm_decoder.") and "self_attn_weights.in_proj" in k:
            a = np.array(sd[k], dtype=np.float32, copy=True)
            a[:H * QD] *= S
            a[2 * H * QD:2 * H * QD + H * PD] *= S
            out[k] = a
    return out


_sd = {}


def state(S=1.0):
    from zipvoice_amd.config import default_config
    from zipvoice_amd.weights import synthetic_state_dict
    cfg = default_config("zipvoice")
    if S not in _sd:
        base = _sd.get(1.0) or synthetic_state_dict(cfg, 0)
        _sd[1.0] = base
        _sd[S] = base if S == 1.0 else scaled_scores_sd(cfg, base, S)
    return cfg, _sd[S]


def engine_with(monkeypatch, env, S=1.0):
    from zipvoice_amd.models import build_model
    for k in ("ZV_ATTN2", "ZV_ATTN2_EXACT", "ZV_ATTN_MATERIALIZE"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    cfg, sd = state(S)
    m = build_model(cfg, precision="bf16")
    m.load_state_dict(sd)
    m = m.to("cuda:0")
    for k in env:
        monkeypatch.delenv(k)
    return m


def vel_inputs(T):
    rng = np.random.default_rng(T)
    B = 2
    x = rng.standard_normal((B, T, 100), dtype=np.float32)
    tc = rng.standard_normal((B, T, 100), dtype=np.float32)
    sc = (0.3 * rng.standard_normal((B, T, 100)) - 0.5).astype(np.float32)
    pm = np.arange(T)[None] >= np.array([T, int(T * 0.82)])[:, None]
    return x, tc, sc, pm


def velocity(m, ins):
    x, tc, sc, pm = (torch.from_numpy(a).to("cuda:0") for a in ins)
    v = m.engine.velocity(0.3, 1.0, x, tc, sc, pm)
    torch.cuda.synchronize()
    return v.float().cpu().numpy()


def diff(a, b, pm):
    d = np.abs(a - b)[~pm]
    return float(d.mean()), float(d.max())


_v = {}


def v_of(monkeypatch, T, name, env, S=1.0):
    key = (T, name, S)
    if key not in _v:
        m = engine_with(monkeypatch, env, S)
        m.engine.attn_fallbacks(reset=True)
        v = velocity(m, vel_inputs(T))
        _v[key] = (v, m.engine.attn_fallbacks(reset=True))
        del m
        torch.cuda.empty_cache()
    return _v[key]


@pytest.mark.parametrize("T", [1219, 3376])
def test_engine_attn2_vs_first_generation(monkeypatch, T):
    pm = vel_inputs(T)[3]
    v2, c2 = v_of(monkeypatch, T, "attn2", {})
    v1, _ = v_of(monkeypatch, T, "attn1", {"ZV_ATTN2": "0"})
    mean, mx = diff(v2, v1, pm)
    print(f"T={T}: ZV_ATTN2=1 vs 0 mean {mean:.3e} max {mx:.3e}; fallbacks {c2}")
    assert c2 == (0, 0, 0), c2
    assert mean < 1.5e-2 and mx < 0.1, (mean, mx)


def test_engine_attn2_error_vs_oracle_no_worse(monkeypatch):
    """At C2's length both consumer generations against the fp32 oracle: the second generation's
    error is within 1.3x the first generation's (a mean / max bound derived from the first
    generation's own bf16 error, not the model bar)."""
    from oracle.zipvoice_np import ZipVoiceOracle
    T = 1219
    x, tc, sc, pm = vel_inputs(T)
    cfg, sd = state()
    ref = ZipVoiceOracle(cfg, sd).velocity(np.float32(0.3), x, tc, sc, pm, 1.0)
    e2 = diff(v_of(monkeypatch, T, "attn2", {})[0], ref, pm)
    e1 = diff(v_of(monkeypatch, T, "attn1", {"ZV_ATTN2": "0"})[0], ref, pm)
    print(f"vs oracle: second generation mean {e2[0]:.3e} max {e2[1]:.3e}; first {e1[0]:.3e} / {e1[1]:.3e}")
    assert e2[0] <= 1.3 * e1[0] and e2[1] <= 1.3 * e1[1] + 1e-2, (e2, e1)


@pytest.mark.parametrize("T", [1219, 3376])
def test_engine_forced_exact_path(monkeypatch, T):
    pm = vel_inputs(T)[3]
    v2, c2 = v_of(monkeypatch, T, "attn2", {})
    vx, cx = v_of(monkeypatch, T, "exact", {"ZV_ATTN2_EXACT": "1"})
    mean, mx = diff(v2, vx, pm)
    print(f"T={T}: forced exact vs fast mean {mean:.3e} max {mx:.3e}; fallbacks fast {c2} forced {cx}")
    assert c2[2] == 0 and cx[2] > 0 and cx[0] == cx[1] == 0, (c2, cx)
    assert mean < 1.5e-2 and mx < 0.1, (mean, mx)


@pytest.mark.parametrize("T", [1219, 3376])
def test_engine_materialized_bf16(monkeypatch, T):
    """The bf16 W-materialising fallback (base-2 masked value, exp2 softmax) against the fused
    consumers, padding mask included."""
    pm = vel_inputs(T)[3]
    v2, _ = v_of(monkeypatch, T, "attn2", {})
    vm, cm = v_of(monkeypatch, T, "mat", {"ZV_ATTN_MATERIALIZE": "1"})
    mean, mx = diff(v2, vm, pm)
    print(f"T={T}: fused vs materialised (bf16) mean {mean:.3e} max {mx:.3e}")
    assert np.isfinite(vm).all() and cm[2] == 0
    assert mean < 1.5e-2 and mx < 0.1, (mean, mx)


def test_engine_scores_straddling_the_range(monkeypatch):
    """Scores x8 (the attention-score projection's q / p rows): about a quarter of the C2-length
    waves / blocks fail the range check and take the exact path, the rest stay fast.  At this
    scale attention is near-argmax and any bf16 perturbation moves the output by O(0.1-1) (the
    first generation differs from the second by mean 0.94): the check is that the output is
    finite, the counters show a partial fallback, and the forced-exact engine is no further from
    the natural one than the first generation is."""
    T = 1219
    pm = vel_inputs(T)[3]
    v2, c2 = v_of(monkeypatch, T, "attn2", {}, S=8.0)
    vx, cx = v_of(monkeypatch, T, "exact", {"ZV_ATTN2_EXACT": "1"}, S=8.0)
    v1, _ = v_of(monkeypatch, T, "attn1", {"ZV_ATTN2": "0"}, S=8.0)
    print(f"S=8: fallbacks natural {c2} forced {cx}; natural vs forced {diff(v2, vx, pm)}; "
          f"natural vs first generation {diff(v2, v1, pm)}")
    assert np.isfinite(v2).all()
    assert 0 < c2[2] < cx[2] and c2[1] > 0, (c2, cx)
    assert diff(v2, vx, pm)[0] < diff(v2, v1, pm)[0], "forced exact further than the first generation"

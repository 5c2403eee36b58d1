"""MX-fp8 operand format of the fp8 mode, restated in numpy (TEST INFRASTRUCTURE: only tests/
and tools/ import this; the product path is zipvoice_amd/csrc/zv_mx8.inc).

The reference has no fp8 path: BASELINE.json configs[4] ("ZipVoice-Dialog-Stereo ... fp8 MFMA
weights") names the mode, so this module is the format's specification, not a restatement of
reference code.  Values are OCP e4m3fn (bias 7, max 448, subnormals 2^-9 steps, round to
nearest even); each run of 32 consecutive K elements of a row shares an E8M0 scale 2^e, e the
smallest integer with max|x| * 2^-e <= 448, clamped to [-126, 126] (zero blocks: e = -126).
Parity of the fp8 mode against the fp32 reference is a documented tolerance, not bit
equality; the C host quantiser is pinned bit-exactly to this module
(tests/test_cabi.py) and the device quantiser / GEMM to it on the GPU (tests/test_gpu_fp8.py).
"""
import numpy as np

BLOCK = 32


def block_exponents(amax):
    """e per block (int32), amax (..., nblocks) float32."""
    amax = np.asarray(amax, dtype=np.float32)
    with np.errstate(divide="ignore"):
        r = amax.astype(np.float64) / 448.0
        e = np.ceil(np.log2(np.where(r > 0, r, 1.0))).astype(np.int64)
    e = np.where(amax > 0, e, -126)
    # exact: the smallest e with amax <= 448 * 2^e
    e = np.where(amax.astype(np.float64) > 448.0 * np.exp2(e.astype(np.float64)), e + 1, e)
    e = np.where(amax.astype(np.float64) <= 448.0 * np.exp2((e - 1).astype(np.float64)), e - 1, e)
    e = np.where(amax > 0, e, -126)
    return np.clip(e, -126, 126).astype(np.int32)


def e4m3_encode(x):
    """Round-to-nearest-even e4m3fn codes (uint8) of float32 x with |x| <= 448."""
    x = np.asarray(x, dtype=np.float64)
    sign = np.where(np.signbit(x), 0x80, 0).astype(np.uint8)
    a = np.minimum(np.abs(x), 448.0)
    code = np.zeros(a.shape, dtype=np.int64)
    nz = a > 0
    E = np.zeros(a.shape, dtype=np.int64)
    E[nz] = np.floor(np.log2(a[nz])).astype(np.int64)
    # guard log2 rounding at exact powers of two
    E = np.where(nz & (np.exp2(E.astype(np.float64)) > a), E - 1, E)
    E = np.where(nz & (np.exp2((E + 1).astype(np.float64)) <= a), E + 1, E)
    sub = nz & (E < -6)
    q = np.rint(np.ldexp(a, 9))                        # subnormal grid, ties to even
    code = np.where(sub, q, code)
    nrm = nz & ~sub
    m = np.rint(np.ldexp(a, (3 - E).astype(np.int64)))   # in [8, 16]
    E2 = np.where(m == 16, E + 1, E)
    m = np.where(m == 16, 8, m)
    code = np.where(nrm, ((E2 + 7) << 3) | (m.astype(np.int64) - 8), code)
    return (code.astype(np.uint8) | sign).astype(np.uint8)


def e4m3_decode(code):
    code = np.asarray(code, dtype=np.uint8).astype(np.int64)
    s = np.where(code & 0x80, -1.0, 1.0)
    e = (code >> 3) & 15
    m = code & 7
    v = np.where(e > 0, np.ldexp(1.0 + m / 8.0, (e - 7).astype(np.int64)), np.ldexp(m / 8.0, -6))
    return (s * v).astype(np.float64)


def quantize(x, ldq=None):
    """x (rows, K) -> (q (rows, ldq) uint8, s (rows, ldq/32) uint8); ldq = K rounded to 128."""
    x = np.asarray(x, dtype=np.float32)
    rows, K = x.shape
    ldq = ldq or -(-K // 128) * 128
    xp = np.zeros((rows, ldq), dtype=np.float32)
    xp[:, :K] = x
    blocks = xp.reshape(rows, ldq // BLOCK, BLOCK)
    e = block_exponents(np.abs(blocks).max(axis=2))
    scaled = blocks.astype(np.float64) * np.exp2(-e.astype(np.float64))[..., None]
    q = e4m3_encode(scaled.astype(np.float32)).reshape(rows, ldq)
    return q, (e + 127).astype(np.uint8)


def dequantize(q, s):
    rows, ldq = q.shape
    v = e4m3_decode(q).reshape(rows, ldq // BLOCK, BLOCK)
    return (v * np.exp2(s.astype(np.float64) - 127.0)[..., None]).reshape(rows, ldq)


def round_trip(x):
    """x rounded through the MX-fp8 format (float32, same shape)."""
    x = np.asarray(x, dtype=np.float32)
    q, s = quantize(x)
    return dequantize(q, s)[:, :x.shape[1]].astype(np.float32)

"""Host-only check of the fused-attention length rule (zv_attn_plan, no GPU): whenever a
layer takes the fused path, every attention kernel it launches fits one workgroup's
160 KiB of LDS, for every precision mode's kernel set and L up to 5000 frames.  (The
fp16 mode's Toeplitz SelfAttention needs ~36 B per key, the plain kernel ~33 B: sizing
the wrong one let L ~ 4.4k-4.78k through to a launch that throws.)"""
import ctypes

import pytest

LIM = 160 * 1024
# (split, sa_plo, tpm): the kernel sets zv_engine's layer() launches per mode
MODES = {
    "bf16/fp8": (1, 0, 3),        # second generation (zv_flash2.inc): base-2 scores, no stats pass
    "bf16/fp8 ZV_ATTN2=0": (1, 0, 1),   # Toeplitz SA, Toeplitz head-0 stats + NonlinAttention
    "fp16 mixed": (1, 1, 0),      # Toeplitz SA with the table's lo half, fp32-table NA
    "16-bit no-tp": (1, -1, 0),   # ZV_SA_TP=0 A/B arm
    "fp32": (3, -1, 0),
}


@pytest.fixture(scope="module")
def lib():
    from zipvoice_amd.csrc.build import build
    build(verbose=False)
    from zipvoice_amd import engine
    return engine.load_library()


def plan(lib, split, sa_plo, tpm, L, nv):
    o = [ctypes.c_int64() for _ in range(3)]
    fits = ctypes.c_int()
    rc = lib.zv_attn_plan(split, sa_plo, tpm, L, nv, *[ctypes.byref(x) for x in o], ctypes.byref(fits))
    assert rc == 0, lib.zv_last_error()
    return [x.value for x in o], bool(fits.value)


@pytest.mark.parametrize("mode", sorted(MODES))
@pytest.mark.parametrize("nv", [144, 384])   # text encoder (dim 192) / decoder (dim 512) NA width
def test_fused_implies_every_kernel_fits(lib, mode, nv):
    split, sa_plo, tpm = MODES[mode]
    fused_max = 0
    for L in list(range(1, 5001, 7)) + [4400, 4500, 4600, 4700, 4780, 5000]:
        sizes, fits = plan(lib, split, sa_plo, tpm, L, nv)
        assert fits == all(b <= LIM for b in sizes), (mode, L, sizes)
        if fits:
            fused_max = max(fused_max, L)
    # C4/C5 (T = 3376) must stay on the fused path in the 16-bit modes
    if split == 1:
        assert fused_max >= 3376


def test_fp16_mode_long_sequence_falls_back(lib):
    sizes, fits = plan(lib, 1, 1, 0, 4500, 384)
    assert sizes[0] > LIM and not fits       # the advisor's example: 168,400 B SA image


def test_rejects_bad_arguments(lib):
    o = [ctypes.c_int64() for _ in range(3)]
    fits = ctypes.c_int()
    assert lib.zv_attn_plan(3, 1, 0, 100, 384, *[ctypes.byref(x) for x in o], ctypes.byref(fits)) != 0

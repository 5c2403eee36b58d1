"""The C-ABI library builds, loads without a GPU and exports every symbol that
include/zipvoice_hip.h declares (no compute calls here)."""
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "zipvoice_hip.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(zv_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_api():
    syms = declared_symbols()
    for s in ("zv_create", "zv_set_weight", "zv_finalize", "zv_fm_decoder", "zv_velocity",
              "zv_euler_sample", "zv_text_encode", "zv_last_error", "zv_destroy"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from zipvoice_amd.csrc.build import build
    build(verbose=False)
    from zipvoice_amd import engine
    lib = engine.load_library()
    syms = declared_symbols()
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) == set(engine.SIGNATURES), "ctypes signature table out of sync"
    assert lib.zv_version().decode().startswith("zipvoice_hip")


def test_create_rejects_bad_config_without_gpu():
    import ctypes
    from zipvoice_amd import engine
    from zipvoice_amd.config import default_config
    lib = engine.load_library()
    zc = engine.make_zv_config(default_config("zipvoice"), "fp32")
    zc.num_stacks = 0
    assert not lib.zv_create(ctypes.byref(zc))
    assert "num_stacks" in lib.zv_last_error().decode()
    # an engine handle can be created and staged on the host without a GPU
    zc = engine.make_zv_config(default_config("zipvoice"), "bf16")
    h = lib.zv_create(ctypes.byref(zc))
    assert h
    assert lib.zv_finalize(h) != 0           # strict: no weights staged
    assert "missing weight" in lib.zv_last_error().decode()
    lib.zv_destroy(h)


def test_no_cpu_fallback():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from zipvoice_amd.config import default_config
    from zipvoice_amd.models import build_model
    m = build_model(default_config("zipvoice"))
    m.load_synthetic(0)
    with pytest.raises(RuntimeError):
        m.to("cuda:0")
    with pytest.raises(RuntimeError):
        m.to("cpu")


def test_library_built_from_these_sources():
    """Build provenance: each in-tree library (bf16 and fp16 operand builds) carries the
    sha256 of the sources it was compiled from (zv_version "src=..."); it must equal the hash
    of the current tree, so a stale prebuilt .so cannot pass for the sources under test."""
    from zipvoice_amd.csrc.build import VARIANTS, build, library_hash, source_hash
    build(verbose=False)
    for out, defines in VARIANTS:
        assert library_hash(out) == source_hash(defines), out


def test_both_operand_libraries_load_side_by_side():
    """The bf16- and fp16-operand engines export the same entry points; both load into one
    process (RTLD_LOCAL, -Bsymbolic) and each answers for itself."""
    from zipvoice_amd import engine
    a = engine.load_library()
    b = engine.load_library(operand="f16")
    assert a is not b
    va, vb = a.zv_version().decode(), b.zv_version().decode()
    assert "bf16 operands" in va and "fp16 operands" in vb, (va, vb)
    for name in engine.SIGNATURES:
        assert hasattr(b, name), name


@pytest.mark.gpu
def test_gpu_box_library_provenance():
    """On the GPU box (prebuilt library shipped with the tree, no rebuild): the library
    the GPU tests load was compiled from the sources shipped beside it."""
    from zipvoice_amd.csrc.build import VARIANTS, library_hash, source_hash
    for out, defines in VARIANTS:
        assert library_hash(out) == source_hash(defines), f"stale {out}"


def test_mx8_host_quantizer_matches_numpy_spec():
    """The fp8 mode's weight quantiser (csrc/zv_mx8.inc mx8_quantize_host, through the C ABI;
    host only, no GPU) is bit-exact to the numpy specification oracle/mx8_np.py: e4m3 codes
    and E8M0 scale bytes, including zero blocks, subnormal-range values, the 448 maximum,
    rounding ties and a ragged K padded to 128."""
    import numpy as np
    from oracle import mx8_np
    from zipvoice_amd import engine
    lib = engine.load_library()
    rng = np.random.default_rng(7)
    rows, K = 9, 200
    x = rng.standard_normal((rows, K)).astype(np.float32)
    x *= np.exp2(rng.integers(-30, 30, (rows, 1))).astype(np.float32)
    x[0, :32] = 0.0                                   # a zero block
    x[1, :] *= 1e-38                                  # subnormal-range inputs
    x[2, :32] = 448.0 * np.linspace(-1, 1, 32)        # exactly at the e4m3 maximum
    x[3, :16] = np.float32(1.0625)                    # a tie between two e4m3 codes (1.0 / 1.125)
    x[3, 16:32] = np.float32(448.0)
    ldq = 256
    q = np.zeros((rows, ldq), np.uint8)
    s = np.zeros((rows, ldq // 32), np.uint8)
    assert lib.zv_mx8_quantize(x.ctypes.data, rows, K, q.ctypes.data, s.ctypes.data) == 0
    rq, rs = mx8_np.quantize(x, ldq)
    assert np.array_equal(s, rs)
    assert np.array_equal(q, rq)
    # the format round trip: relative error within e4m3's half step of the block maximum
    y = mx8_np.dequantize(q, s)[:, :K]
    blk = np.abs(np.pad(x, ((0, 0), (0, ldq - K)))).reshape(rows, -1, 32).max(2)
    bound = np.repeat(blk, 32, axis=1)[:, :K] * 2.0 ** -4
    assert (np.abs(y - x) <= bound + 1e-45).all()

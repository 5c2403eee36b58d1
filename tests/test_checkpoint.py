"""Checkpoint ingestion: the reference's on-disk weight formats
loaded with loaders that execute nothing from the file.

* ``model.pt``: ``checkpoint.py:87-105`` saves a dict whose ``"model"`` entry is the
  state dict; ``load_checkpoint`` (``checkpoint.py:108-146``) strips the DDP ``module.``
  prefix and loads strictly.  Read here with ``torch.load(weights_only=True)``.
* ``model.safetensors`` (``infer_zipvoice.py:561-566``).

CPU tests: the files round-trip to the exact tensors and strict=True errors.  The GPU
test (marked) checks that the engine built from each file computes bitwise the same
decoder output as the engine built from the in-memory state dict.
"""
import numpy as np
import pytest
import torch

from zipvoice_amd.config import default_config
from zipvoice_amd.weights import (check_state_dict, load_checkpoint_state_dict,
                                  synthetic_state_dict)


def small_cfg(variant="zipvoice"):
    # the base architecture's structure at a size that keeps the files small
    return default_config(variant, fm_decoder_num_layers=[1, 1, 1, 1, 1],
                          fm_decoder_feedforward_dim=512, fm_decoder_dim=256,
                          text_encoder_num_layers=1)


def write_pt(path, sd, ddp=True):
    blob = {"model": {("module." + k if ddp else k): torch.from_numpy(v.copy())
                      for k, v in sd.items()},
            "optimizer": {"state": {}}, "batch_idx_train": 123, "best_valid_loss": 0.5}
    torch.save(blob, path)


def write_safetensors(path, sd):
    from safetensors.numpy import save_file
    save_file({k: np.array(v, np.float32, order="C") for k, v in sd.items()}, path)


@pytest.mark.parametrize("variant", ["zipvoice", "zipvoice_distill", "zipvoice_dialog_stereo"])
@pytest.mark.parametrize("fmt", ["pt_ddp", "pt", "safetensors"])
def test_checkpoint_roundtrip(tmp_path, variant, fmt):
    cfg = small_cfg(variant)
    sd = synthetic_state_dict(cfg, 3)
    if fmt == "safetensors":
        path = str(tmp_path / "model.safetensors")
        write_safetensors(path, sd)
    else:
        path = str(tmp_path / "model.pt")
        write_pt(path, sd, ddp=fmt == "pt_ddp")
    got = load_checkpoint_state_dict(path)
    assert set(got) == set(sd)
    for k in sd:
        assert got[k].dtype == np.float32 and got[k].shape == sd[k].shape
        assert np.array_equal(got[k], sd[k]), k
    check_state_dict(cfg, got)          # strict=True passes
    from zipvoice_amd.models import build_model
    m = build_model(cfg).load_checkpoint(path)
    assert all(np.array_equal(m._state[k], sd[k]) for k in sd)


def test_checkpoint_strict_errors(tmp_path):
    cfg = small_cfg()
    sd = synthetic_state_dict(cfg, 0)
    missing = dict(sd)
    missing.pop("fm_decoder.encoders.1.encoder.layers.0.feed_forward2.in_proj.weight")
    with pytest.raises(KeyError, match="missing"):
        check_state_dict(cfg, missing)
    extra = dict(sd)
    extra["fm_decoder.encoders.9.bogus.weight"] = np.zeros(3, np.float32)
    with pytest.raises(KeyError, match="unexpected"):
        check_state_dict(cfg, extra)
    bad = dict(sd)
    bad["embed.weight"] = np.zeros((5, 5), np.float32)
    with pytest.raises(ValueError, match="shape mismatch"):
        check_state_dict(cfg, bad)
    # a checkpoint of another variant does not load into this one (strict)
    other = str(tmp_path / "distill.pt")
    write_pt(other, synthetic_state_dict(small_cfg("zipvoice_distill"), 0))
    from zipvoice_amd.models import build_model
    with pytest.raises(KeyError):
        build_model(cfg).load_checkpoint(other)
    with pytest.raises(NotImplementedError):
        load_checkpoint_state_dict(str(tmp_path / "model.bin"))


@pytest.mark.gpu
def test_checkpoint_engine_bitwise(tmp_path):
    """Engine from model.pt (DDP prefixes) / model.safetensors == engine from the
    in-memory state dict, bitwise, on a decoder forward."""
    from zipvoice_amd.models import build_model
    cfg = small_cfg()
    sd = synthetic_state_dict(cfg, 5)
    pt = str(tmp_path / "model.pt")
    st = str(tmp_path / "model.safetensors")
    write_pt(pt, sd)
    write_safetensors(st, sd)
    rng = np.random.default_rng(0)
    T = 57
    dev = "cuda:0"
    x = torch.from_numpy(rng.standard_normal((2, T, 100), dtype=np.float32)).to(dev)
    tc = torch.from_numpy(rng.standard_normal((2, T, 100), dtype=np.float32)).to(dev)
    sc = torch.from_numpy(rng.standard_normal((2, T, 100), dtype=np.float32)).to(dev)
    pm = torch.from_numpy(np.arange(T)[None] >= np.array([T, 40])[:, None]).to(dev)
    outs = []
    for load in (lambda m: m.load_state_dict(sd), lambda m: m.load_checkpoint(pt),
                 lambda m: m.load_checkpoint(st)):
        m = build_model(cfg, precision="bf16")
        load(m)
        m = m.to(dev)
        outs.append(m.forward_fm_decoder(torch.tensor(0.4), x, tc, sc, pm).cpu())
        del m
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])

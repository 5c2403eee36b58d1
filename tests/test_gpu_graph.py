"""HIP-graph replay of the Euler loop (zv_euler_sample): the first call of a
shape runs uncaptured, later calls replay a captured graph over staging copies.
Replays must be bit-identical to the uncaptured run, and must not alias the
caller's buffers (different inputs of the same shape give different outputs)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from zipvoice_amd.config import default_config  # noqa: E402
from zipvoice_amd.models import build_model  # noqa: E402
from zipvoice_amd.weights import synthetic_state_dict  # noqa: E402


@pytest.mark.parametrize("variant,precision", [("zipvoice", "bf16"), ("zipvoice_distill", "fp32")])
def test_graph_replay_bit_identical(variant, precision):
    cfg = default_config(variant)
    m = build_model(cfg, precision=precision)
    m.load_state_dict(synthetic_state_dict(cfg, 0))
    m = m.to("cuda:0")
    rng = np.random.default_rng(0)
    B, T = 3, 150
    mk = lambda: torch.from_numpy(rng.standard_normal((B, T, 100), dtype=np.float32)).cuda()  # noqa: E731
    x0, tc, sc = mk(), mk(), mk()
    pm = (torch.arange(T)[None] >= torch.tensor([150, 120, 90])[:, None]).cuda()
    kw = dict(text_condition=tc, speech_condition=sc, padding_mask=pm, num_step=4,
              guidance_scale=1.5 if variant == "zipvoice" else 3.0, t_shift=0.5)
    outs = [m.solver.sample(x=x0.clone(), **kw) for _ in range(4)]   # warm-up(s), capture, replay
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    x1 = mk()
    other = m.solver.sample(x=x1, **kw)
    ref = m.solver.sample(x=x1.clone(), **kw)
    assert torch.equal(other, ref) and not torch.equal(other, outs[0])
    assert torch.equal(x0, outs[0]) is False

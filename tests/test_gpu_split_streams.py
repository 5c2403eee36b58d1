"""Decoder row blocks on 2-4 streams (ZV_SPLIT_STREAMS, zv_engine::decoder; default 3)
against the single-stream decoder (ZV_SPLIT_STREAMS=1): rows never interact on the path
(every kernel is per row, per (row, head) or per output element with a fixed K order), so
the velocity, a guided Euler solve replayed from its graph, and the per-utterance-guidance
/ Distill variants must be bitwise equal."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _inputs(B, T, lens, seed):
    rng = np.random.default_rng(seed)
    dev = "cuda:0"
    f = lambda: torch.from_numpy(rng.standard_normal((B, T, 100), dtype=np.float32)).to(dev)
    x, tc, sc = f(), f(), f()
    pm = torch.from_numpy(np.arange(T)[None] >= np.array(lens)[:, None]).to(dev)
    return x, tc, sc, pm


@pytest.mark.parametrize("variant,precision,parts", [("zipvoice", "bf16", "2"), ("zipvoice", "fp32", "2"),
                                                     ("zipvoice_distill", "bf16", "2"),
                                                     ("zipvoice", "bf16", "3"), ("zipvoice", "bf16", "4"),
                                                     ("zipvoice", "fp16", "4")])
def test_split_streams_bitwise(monkeypatch, variant, precision, parts):
    from zipvoice_amd.config import default_config
    from zipvoice_amd.models import build_model
    from zipvoice_amd.weights import synthetic_state_dict
    cfg = default_config(variant)
    sd = synthetic_state_dict(cfg, 0)
    B, T = 3, 1500                                   # 6 CFG rows x 1500 >= the split threshold
    x, tc, sc, pm = _inputs(B, T, [1500, 1200, 777], seed=3)
    g_rows = torch.tensor([1.0, 0.0, 2.0]).reshape(B, 1, 1)
    outs = []
    # single stream, split + graph replay, split + plain launches (ZV_GRAPH=2, the default:
    # split shapes are not replayed from a graph)
    for flag, graph in (("1", "1"), (parts, "1"), (parts, "2")):
        monkeypatch.setenv("ZV_SPLIT_STREAMS", flag)
        monkeypatch.setenv("ZV_SPLIT_MIN_ROWS", "2048")
        monkeypatch.setenv("ZV_GRAPH", graph)
        monkeypatch.setenv("ZV_FFN_MIN_ROWS", "0")    # one FeedForward kernel at every block size
        m = build_model(cfg, precision=precision)
        m.load_state_dict(sd)
        m = m.to("cuda:0")
        r = [m.engine.velocity(0.3, 1.0, x, tc, sc, pm).cpu(),
             m.engine.velocity(0.7, g_rows, x, tc, sc, pm).cpu()]
        for _ in range(2):                           # warm-up run, then the captured graph
            xs = m.solver.sample(x=x, text_condition=tc, speech_condition=sc, padding_mask=pm,
                                 num_step=3, guidance_scale=1.0, t_shift=0.5)
        r.append(xs.cpu())
        outs.append(r)
        del m
    for arm in outs[1:]:
        for i, (a, b) in enumerate(zip(outs[0], arm)):
            d = (a - b).abs().max().item()
            print(f"{variant} {precision} output {i}: max |split - single| = {d:.3e}")
            assert torch.equal(a, b), (i, d)


@pytest.mark.parametrize("precision", ["bf16", "fp16"])
def test_ffn_persistent_bitwise(monkeypatch, precision):
    """The fused FeedForward's persistent line schedule (ZV_FFN_PERSIST, zv_ffn.inc: row blocks cut
    into P / C items whose out^T tiles are handed over through memory, one flag word per line)
    against one row block per block, on one stream and on the split decoder's three streams, with
    the default thresholds: bitwise equal velocities.
    16 utterances = 32 CFG rows x 1219 frames: 39008 rows (305 row blocks) at the full-rate stacks,
    19504 at the half-rate ones -- lines cut row blocks at every stack that runs fused.
    Two different velocities run back to back on each engine (and every call launches the kernel
    48 times on one scratch): a flag word left set by one launch would let the next launch's C
    item skip its wait and start from the previous launch's tiles -- the second output would then
    differ (the round-4 hand-off faults, DESIGN.md §3, were of this family)."""
    from zipvoice_amd.config import default_config
    from zipvoice_amd.models import build_model
    from zipvoice_amd.weights import synthetic_state_dict
    cfg = default_config("zipvoice")
    sd = synthetic_state_dict(cfg, 0)
    B, T = 16, 1219
    x, tc, sc, pm = _inputs(B, T, [1219 - 37 * i for i in range(B)], seed=5)
    outs = []
    for env in ({"ZV_SPLIT_STREAMS": "1", "ZV_FFN_PERSIST": "0"},
                {"ZV_SPLIT_STREAMS": "1", "ZV_FFN_PERSIST": "1"},
                {"ZV_SPLIT_STREAMS": "3", "ZV_FFN_PERSIST": "1"}):
        for k in ("ZV_SPLIT_STREAMS", "ZV_FFN_PERSIST", "ZV_FFN_MIN_ROWS", "ZV_GRAPH"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        m = build_model(cfg, precision=precision)
        m.load_state_dict(sd)
        m = m.to("cuda:0")
        outs.append([m.engine.velocity(0.3, 1.0, x, tc, sc, pm).cpu(),
                     m.engine.velocity(0.8, 1.0, x, tc, sc, pm).cpu()])
        del m
    for j, arm in enumerate(outs[1:], 1):
        for i, (a, b) in enumerate(zip(outs[0], arm)):
            d = (a - b).abs().max().item()
            print(f"{precision} arm {j} output {i}: max |arm - classic one-stream| = {d:.3e}")
            assert torch.isfinite(b).all()
            assert torch.equal(a, b), (j, i, d)

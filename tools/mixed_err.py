#!/usr/bin/env python3
"""Mean |velocity - oracle| of one precision mode on small seeded cases (the shapes of
tests/test_gpu_sa_tp.py and the parity fixtures' lengths), under the policy environment in
effect: a quick probe of how close a parity-grade variant sits to north_star's 1e-3 bar.

usage: python tools/mixed_err.py [fp16] [B,T,len1,len2 ...]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "fp16"
    cases = [tuple(int(v) for v in a.split(",")) for a in sys.argv[2:]] or [(2, 203, 203, 150),
                                                                         (2, 422, 422, 300),
                                                                         (1, 1219, 1219)]
    from oracle.zipvoice_np import ZipVoiceOracle
    from zipvoice_amd.config import default_config
    from zipvoice_amd.models import build_model
    from zipvoice_amd.weights import synthetic_state_dict
    for variant in ("zipvoice", "zipvoice_dialog_stereo"):
        cfg = default_config(variant)
        sd = synthetic_state_dict(cfg, 0)
        m = build_model(cfg, precision=prec)
        m.load_state_dict(sd)
        m = m.to("cuda:0")
        o = ZipVoiceOracle(cfg, sd)
        F = cfg.io_feat_dim
        for case in cases:
            B, T, lens = case[0], case[1], list(case[2:]) or [case[1]] * case[0]
            rng = np.random.default_rng(11 + T)
            x = rng.standard_normal((B, T, F), dtype=np.float32)
            tc = rng.standard_normal((B, T, cfg.feat_dim), dtype=np.float32)
            sc = rng.standard_normal((B, T, F), dtype=np.float32)
            pm = np.arange(T)[None] >= np.array(lens)[:, None]
            cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")  # noqa: E731
            v = m.engine.velocity(0.4, 1.0, cu(x), cu(tc), cu(sc), cu(pm)).cpu().numpy()
            ref = o.velocity(np.float32(0.4), x, tc, sc, pm, 1.0)
            e = np.abs(v - ref)[~pm]
            print(f"{variant} {prec} B={B} T={T} lens={lens}: mean {e.mean():.3e} max {e.max():.3e}", flush=True)
        del m
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

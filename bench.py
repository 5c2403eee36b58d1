#!/usr/bin/env python3
"""Benchmark: generated mel-frames/s (whole job) + RTF of ZipVoice sampling.

Workload (BASELINE.json configs[1], "C2"): ZipVoice 123M (synthetic seeded
weights — no pretrained weights offline), bf16 MFMA, N_steps=16, batch of 32
utterances per GPU, each a 3 s prompt (281 frames, 40 prompt tokens) + 10 s of
generated speech (938 frames, 134 text tokens; duration="real"), so T = 1219
frames, classifier-free guidance 1.0 (batch doubled to 64 inside the engine),
t_shift 0.5.  One "step" = what the reference's RTF times
(``infer_zipvoice.py:359-386``): one full ``ZipVoice.sample()`` of the batch
(text encoder, conditions, the 16-step guided Euler loop) followed by the
vocoder on the generated features (post-processing + Vocos decode + clamp,
``:374-378``; synthetic vocos-mel-24khz weights, fp32-accurate mode), plus, for
N > 1 GPUs, the RCCL all-gather that reassembles the output wav batch on every
rank.

Launch: python bench.py [--gpus N --steps K --warmup W]
        (N > 1 under torch.distributed.run, one process per GPU).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

# C2 shapes
B_PER_GPU = 32
T_PROMPT = 281
S_PROMPT = 40
S_TEXT = 134
T_GEN = 938
NUM_STEP = 16
GUIDANCE = 1.0
T_SHIFT = 0.5
SAMPLE_RATE = 24000
HOP = 256
BF16_DENSE_PEAK_TFLOPS = 2500.0     # MI355X_MICROARCH.md: ~2.5 PF dense bf16
FP32_MFMA_PEAK_TFLOPS = 157.3
HBM_PEAK_GBS = 8000.0
# PMC traffic per launch (tools/pmc_traffic.py, tools/gpu/final.sh) of the two GEMM instantiations
# the roofline reports: the residual-stream linears (ROLE = 1) and the plain / activation linears
TRAFFIC_FILES = {"gemm_bf16_resid": "r01_gemm_resid_traffic.json", "gemm_bf16": "r01_gemm_traffic.json"}


def make_inputs(rank, device):
    rng = np.random.default_rng(1000 + rank)
    tokens = [[int(v) for v in rng.integers(1, 360, S_TEXT)] for _ in range(B_PER_GPU)]
    ptokens = [[int(v) for v in rng.integers(1, 360, S_PROMPT)] for _ in range(B_PER_GPU)]
    pf = (0.3 * rng.standard_normal((B_PER_GPU, T_PROMPT, 100)) - 0.5).astype(np.float32)
    plens = np.full(B_PER_GPU, T_PROMPT, np.int64)
    flens = np.full(B_PER_GPU, T_GEN, np.int64)
    T = T_PROMPT + T_GEN
    x0 = np.random.default_rng(666 + rank).standard_normal((B_PER_GPU, T, 100), dtype=np.float32)
    to = lambda a: torch.from_numpy(a).to(device)  # noqa: E731
    return dict(tokens=tokens, prompt_tokens=ptokens, prompt_features=to(pf),
                prompt_features_lens=to(plens), features_lens=to(flens), x0=to(x0))


def build(precision, device):
    from zipvoice_amd.config import default_config
    from zipvoice_amd.models import build_model
    from zipvoice_amd.weights import synthetic_state_dict
    cfg = default_config("zipvoice")
    m = build_model(cfg, precision=precision)
    m.load_state_dict(synthetic_state_dict(cfg, 0))
    return m.to(device)


def build_vocoder(device):
    from zipvoice_amd.vocoder import Vocos
    return Vocos(precision="fp32").load_synthetic(0).to(device)


def run_step(model, vocoder, inp, world, rank):
    gen, gen_lens, _, _ = model.sample(
        tokens=inp["tokens"], prompt_tokens=inp["prompt_tokens"],
        prompt_features=inp["prompt_features"], prompt_features_lens=inp["prompt_features_lens"],
        features_lens=inp["features_lens"], t_shift=T_SHIFT, duration="real",
        num_step=NUM_STEP, guidance_scale=GUIDANCE, x0=inp["x0"])
    wav = vocoder.decode_features(gen, gen_lens, feat_scale=0.1, feat_bias=0.0, clamp=True)
    if world > 1:
        # the one exchange of the data-parallel path: reassemble the output wav
        # batch on every rank (RCCL all-gather over xGMI), zipvoice_amd/dist.py
        from zipvoice_amd.dist import all_gather_padded
        wav, _ = all_gather_padded(wav.unsqueeze(-1), gen_lens * HOP)
    return wav


def timed(model, vocoder, inp, steps, warmup, world, rank):
    import torch.distributed as dist
    for _ in range(warmup):
        run_step(model, vocoder, inp, world, rank)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        run_step(model, vocoder, inp, world, rank)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt / steps


def _kernel_roofline(name, r, total_ms):
    """Roofline object of one tagged kernel.  Residual-stream linears (tag *_resid) sit
    below the bf16 ridge point (<= ~250 FLOP/B vs 2500 TF/s / 8 TB/s = 312): bound HBM,
    achieved = algorithmic bytes per launch / average launch duration.  The others are
    priced on the dense MFMA peak of their dtype."""
    hbm = name.endswith("_resid")
    sec = r["ms"] * 1e-3
    if hbm:
        achieved, peak, unit = r["bytes"] / sec / 1e9, HBM_PEAK_GBS, "GB/s"
    else:
        achieved = r["flops"] / sec / 1e12
        peak = BF16_DENSE_PEAK_TFLOPS if "bf16" in name else FP32_MFMA_PEAK_TFLOPS
        unit = "TFLOP/s"
    traffic, tsrc = None, None
    tfile = TRAFFIC_FILES.get(name)
    tpath = os.path.join(REPO, "profiles", tfile) if tfile else None
    if tpath and os.path.exists(tpath):
        with open(tpath) as f:
            t = json.load(f)
        traffic = t.get("traffic_bytes_per_launch")
        tsrc = (f"profiles/{tfile}: rocprofv3 PMC FETCH_SIZE(x2, gfx950) + WRITE_SIZE "
                f"per launch of {t['kernel_regex']} over one guided forward")
    out = {
        "kernel": name, "bound": "hbm" if hbm else "mfma", "achieved": round(achieved, 2), "peak": peak,
        "unit": unit, "frac": round(achieved / peak, 4), "traffic": traffic,
        "traffic_unit": "bytes per launch", "traffic_source": tsrc,
        "launches_per_step": r["launches"], "avg_launch_us": round(r["ms"] * 1e3 / r["launches"], 2),
        "flops_per_launch": r["flops"] / r["launches"],
        "tflops_achieved": round(r["flops"] / sec / 1e12, 2),
        "share_of_profiled_time": round(r["ms"] / total_ms, 3),
    }
    if hbm:
        out["algorithmic_bytes_per_launch"] = r["bytes"] / r["launches"]
    return out


def roofline(model, vocoder, inp):
    """One extra, untimed step with the engine's per-launch HIP-event profiler on:
    the dominant kernel's algorithmic work per launch / its average duration (HIP events
    on the launch stream), plus the same object for the plain GEMM family."""
    from zipvoice_amd import engine
    torch.cuda.synchronize()
    engine.profile(True)
    run_step(model, vocoder, inp, 1, 0)
    torch.cuda.synchronize()
    rep = engine.profile_report()
    engine.profile(False)
    total_ms = sum(v["ms"] for v in rep.values())
    name, r = max(rep.items(), key=lambda kv: kv[1]["ms"])
    res = _kernel_roofline(name, r, total_ms)
    if name != "gemm_bf16" and "gemm_bf16" in rep:
        res["secondary"] = _kernel_roofline("gemm_bf16", rep["gemm_bf16"], total_ms)
    res["per_kernel_ms_per_step"] = {k: round(v["ms"], 3) for k, v in rep.items()}
    return res


def cpu_baseline(budget_s=12.0):
    """Oracle (numpy fp32 restatement, oracle/zipvoice_np.py) on the host cores: one
    utterance of the same workload (CFG batch of 2, T=1219), guided velocity
    evaluations repeated until ~budget_s, scaled to generated frames/s."""
    from threadpoolctl import threadpool_limits

    from oracle.zipvoice_np import ZipVoiceOracle
    from zipvoice_amd.config import default_config
    from zipvoice_amd.weights import synthetic_state_dict
    cores = min(16, len(os.sched_getaffinity(0)))
    cfg = default_config("zipvoice")
    o = ZipVoiceOracle(cfg, synthetic_state_dict(cfg, 0))
    rng = np.random.default_rng(7)
    T = T_PROMPT + T_GEN
    x = rng.standard_normal((1, T, 100), dtype=np.float32)
    tc = rng.standard_normal((1, T, 100), dtype=np.float32)
    sc = rng.standard_normal((1, T, 100), dtype=np.float32)
    pm = np.zeros((1, T), bool)
    n = 0
    with threadpool_limits(limits=cores):
        t0 = time.perf_counter()
        while True:
            o.velocity(np.float32(0.3), x, tc, sc, pm, GUIDANCE)
            n += 1
            if time.perf_counter() - t0 > budget_s or n >= 8:
                break
        dt = (time.perf_counter() - t0) / n
    frames_per_s = T_GEN / (NUM_STEP * dt)
    return {"value": round(frames_per_s, 2), "unit": "mel-frames/s", "cores": cores,
            "kind": "port",
            "sample": f"{n} guided velocity evaluations (CFG batch 2 x T={T}) of one utterance; "
                      f"{dt:.2f} s each; frames/s = {T_GEN} / (16 steps x time per evaluation)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fp32-mode", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=device)

    model = build(args.precision, device)
    vocoder = build_vocoder(device)
    inp = make_inputs(rank, device)
    ms = timed(model, vocoder, inp, args.steps, args.warmup, world, rank) * 1e3
    frames = B_PER_GPU * T_GEN * world
    value = frames / (ms * 1e-3)
    audio_s_per_gpu = B_PER_GPU * T_GEN * HOP / SAMPLE_RATE
    rtf = (ms * 1e-3) / audio_s_per_gpu
    result = {
        "metric": "generated mel-frames/s (whole job) + RTF, ZipVoice 123M N_steps=16 batch=32/GPU",
        "value": round(value, 1), "unit": "mel-frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 2), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": args.precision, "data": "synthetic",
        "rtf_per_gpu": round(rtf, 6), "x_realtime_per_gpu": round(1.0 / rtf, 1),
        "config": {"workload": "C2: ZipVoice 123M, N_steps=16, batch=32x(3 s prompt + 10 s "
                               "generated; T=1219 frames), CFG g=1.0 (64 rows), t_shift=0.5",
                   "model": "ZipVoice-123M (zipvoice_base.json, synthetic seeded weights)",
                   "global_batch": B_PER_GPU * world, "seq_len": T_PROMPT + T_GEN,
                   "parallelism": f"dp{world}"},
    }
    if rank == 0:
        result["roofline"] = roofline(model, vocoder, inp)
        if world == 1 and not args.no_fp32_mode and args.precision == "bf16":
            del model
            torch.cuda.empty_cache()
            m32 = build("fp32", device)
            ms32 = timed(m32, vocoder, inp, 1, 1, 1, 0) * 1e3
            result["fp32_accurate_mode"] = {
                "ms_per_step": round(ms32, 2),
                "value": round(B_PER_GPU * T_GEN / (ms32 * 1e-3), 1), "unit": "mel-frames/s",
                "note": "bf16x3 split-product GEMMs; the parity mode (mean |err| ~3e-5 vs reference)"}
            del m32
        if world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline()
        print(json.dumps(result), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

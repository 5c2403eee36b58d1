"""Data-parallel batch sharding across the GPUs of one node.

The reference runs inference on a single device, one sentence at a time
(``infer_zipvoice.py:568-577``, ``:431-452``); utterances are independent, so the
MI355X build shards a batch across one process per GPU with no data-path
collective, and uses exactly one exchange at the end: an all-gather (RCCL over
xGMI on GPUs, gloo in the CPU tests) of the per-utterance output lengths and the
padded outputs, which reassembles the batch in its original order on every rank.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def shard_bounds(costs: Sequence[float], world: int) -> List[Tuple[int, int]]:
    """Split items 0..n-1 into `world` contiguous ranges of roughly equal total
    cost (e.g. frames per utterance).  Every rank gets a range (possibly empty)."""
    n = len(costs)
    total = float(sum(costs))
    bounds = []
    start, acc = 0, 0.0
    for r in range(world - 1):
        target = total * (r + 1) / world
        end = start
        while end < n and acc + costs[end] <= target + 1e-9:
            acc += costs[end]
            end += 1
        # take one more item when that lands closer to the ideal boundary
        if end < n and abs(acc + costs[end] - target) < abs(acc - target):
            acc += costs[end]
            end += 1
        bounds.append((start, end))
        start = end
    bounds.append((start, n))
    return bounds


def local_slice(items: Sequence, costs: Sequence[float], rank: int, world: int):
    lo, hi = shard_bounds(costs, world)[rank]
    return lo, hi, list(items[lo:hi])


def all_gather_padded(x: torch.Tensor, lens: torch.Tensor, group=None):
    """All-gather a (b_r, T_r, F) tensor with per-row lengths (b_r,) from every
    rank, where b_r and T_r may differ per rank.  Returns the concatenated
    (sum b_r, max T, F) tensor (rows in rank order, zero padded) and lengths."""
    world = dist.get_world_size(group)
    dev = x.device
    shape = torch.tensor([x.shape[0], x.shape[1]], dtype=torch.int64, device=dev)
    shapes = [torch.zeros_like(shape) for _ in range(world)]
    dist.all_gather(shapes, shape, group=group)
    shapes = [tuple(int(v) for v in s.tolist()) for s in shapes]
    bmax = max(s[0] for s in shapes)
    tmax = max(s[1] for s in shapes)
    F = x.shape[2]
    pad = torch.zeros((bmax, tmax, F), dtype=x.dtype, device=dev)
    pad[:x.shape[0], :x.shape[1]] = x
    lpad = torch.zeros((bmax,), dtype=torch.int64, device=dev)
    lpad[:lens.shape[0]] = lens.to(torch.int64)
    outs = [torch.empty_like(pad) for _ in range(world)]
    louts = [torch.empty_like(lpad) for _ in range(world)]
    dist.all_gather(outs, pad, group=group)
    dist.all_gather(louts, lpad, group=group)
    rows = [o[:s[0]] for o, s in zip(outs, shapes)]
    lrows = [l[:s[0]] for l, s in zip(louts, shapes)]
    return torch.cat(rows, 0), torch.cat(lrows, 0)


def _world_rank(group=None) -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def generate_batch_dp(items: Sequence, compute: Callable[[Sequence], Tuple[torch.Tensor, torch.Tensor]],
                      costs: Optional[Sequence[float]] = None, group=None):
    """Data-parallel generation of one GLOBAL batch, the multi-GPU replacement of the
    reference's single-device sentence loop (``infer_zipvoice.py:568-577``, ``:431-452``).

    Every rank holds the same ``items`` list (one entry per utterance).  Rank r takes its
    contiguous cost-balanced shard (:func:`shard_bounds` over ``costs``, e.g. frames per
    utterance), runs ``compute(shard) -> (wav (b, n), lens (b,))`` on its own GPU (the
    whole ``sample()`` + vocoder path; nothing crosses ranks inside it), and the single
    exchange of the path, :func:`all_gather_padded` (RCCL over xGMI on GPUs, gloo on CPU),
    reassembles the (B, n_max) wav batch and its lengths in the original item order on
    every rank.  Multi-channel output (ZipVoice-Dialog-Stereo: one wav per channel,
    ``infer_zipvoice_dialog.py:483-490``) comes as wav (b, n, C) channel-last with lens in
    samples per channel and is gathered as (B, n_max, C).  Returns (wav, lens, (lo, hi)) with
    (lo, hi) this rank's shard."""
    world, rank = _world_rank(group)
    if costs is None:
        costs = [1.0] * len(items)
    if len(costs) != len(items):
        raise ValueError("costs must have one entry per item")
    lo, hi = shard_bounds(costs, world)[rank]
    wav, lens = compute(items[lo:hi])
    if (wav.dim() not in (2, 3) or lens.dim() != 1 or wav.shape[0] != lens.shape[0]
            or wav.shape[0] != hi - lo):
        raise ValueError("compute must return (wav (b, n) or (b, n, C), lens (b,)) for its "
                         "b = hi - lo items")
    if world == 1:
        return wav, lens, (lo, hi)
    mono = wav.dim() == 2
    out, olens = all_gather_padded(wav.unsqueeze(-1) if mono else wav.contiguous(), lens, group)
    return (out.squeeze(-1) if mono else out), olens, (lo, hi)

"""Multi-process data-parallel path on CPU (gloo, world_size 2): sharding is
balanced and covers every item once; the final all-gather reassembles ragged
per-rank outputs in the original order."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from zipvoice_amd.dist import all_gather_padded, shard_bounds


def test_shard_bounds_cover_and_balance():
    for costs in ([1] * 32, [5, 1, 1, 1, 1, 1, 1, 5], list(range(1, 20)), [3], [], [2, 2]):
        for world in (1, 2, 4, 8):
            b = shard_bounds(costs, world)
            assert len(b) == world
            assert b[0][0] == 0 and b[-1][1] == len(costs)
            for (lo, hi), (lo2, _) in zip(b, b[1:]):
                assert hi == lo2 and lo <= hi
    b = shard_bounds([1] * 32, 8)
    assert all(hi - lo == 4 for lo, hi in b)
    # ragged costs: no rank above the ideal share + one max item
    costs = [int(c) for c in torch.randint(100, 3000, (64,), generator=torch.Generator().manual_seed(0))]
    for world in (2, 4, 8):
        b = shard_bounds(costs, world)
        loads = [sum(costs[lo:hi]) for lo, hi in b]
        assert max(loads) <= sum(costs) / world + max(costs)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        costs = [10 + 7 * i % 13 for i in range(7)]
        lo, hi = shard_bounds(costs, world)[rank]
        # each "utterance" i produces costs[i] frames of value i (3 features)
        T = max([costs[i] for i in range(lo, hi)], default=1)
        x = torch.zeros((hi - lo, T, 3))
        for j, i in enumerate(range(lo, hi)):
            x[j, :costs[i]] = float(i)
        lens = torch.tensor([costs[i] for i in range(lo, hi)], dtype=torch.int64)
        allx, alll = all_gather_padded(x, lens)
        q.put((rank, allx.numpy().tolist(), alll.tolist()))
    finally:
        dist.destroy_process_group()


def test_all_gather_reassembles_batch_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    costs = [10 + 7 * i % 13 for i in range(7)]
    for rank, allx, alll in res:
        assert alll == costs
        allx = torch.tensor(allx)
        assert allx.shape[0] == 7
        for i in range(7):
            assert torch.all(allx[i, :costs[i]] == float(i))
            assert torch.all(allx[i, costs[i]:] == 0)


def _dp_worker(rank, world, port, q, n_items=9, channels=1):
    """generate_batch_dp — the function bench.py's data-parallel step runs — with a CPU
    compute stub in place of sample() + vocoder: utterance i yields costs[i] samples of
    value i (channels == 2: the stereo form, channel c = (-1)^c i, as bench.py's C5 step
    returns (b, n, 2))."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from zipvoice_amd.dist import generate_batch_dp
        items = list(range(n_items))
        costs = [5 + (3 * i) % 7 for i in items]
        seen = []

        def compute(shard):
            seen.extend(shard)
            n = max([costs[i] for i in shard], default=1)
            wav = torch.zeros((len(shard), n) if channels == 1 else (len(shard), n, channels))
            for j, i in enumerate(shard):
                if channels == 1:
                    wav[j, :costs[i]] = float(i)
                else:
                    for c in range(channels):
                        wav[j, :costs[i], c] = float(i) * (-1) ** c
            return wav, torch.tensor([costs[i] for i in shard], dtype=torch.int64)

        wav, lens, (lo, hi) = generate_batch_dp(items, compute, costs)
        q.put((rank, wav.numpy().tolist(), lens.tolist(), seen, lo, hi))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_items,channels", [(9, 1), (32, 2)], ids=["mono", "stereo-C5"])
def test_generate_batch_dp_world2(n_items, channels):
    """mono, and the C5 shape (bench.py --config C5: 32 Dialog-Stereo utterances, (b, n, 2))."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q, n_items, channels)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    costs = [5 + (3 * i) % 7 for i in range(n_items)]
    # each rank computed exactly its own contiguous shard; together every item once
    assert sorted(res[0][3] + res[1][3]) == list(range(n_items))
    assert res[0][3] == list(range(res[0][4], res[0][5]))
    assert res[0][5] == res[1][4]
    for rank, wav, lens, _, _, _ in res:
        assert lens == costs
        wav = torch.tensor(wav)
        assert wav.shape[0] == n_items and wav.dim() == (2 if channels == 1 else 3)
        for i in range(n_items):
            if channels == 1:
                assert torch.all(wav[i, :costs[i]] == float(i))
                assert torch.all(wav[i, costs[i]:] == 0)
            else:
                for c in range(channels):
                    assert torch.all(wav[i, :costs[i], c] == float(i) * (-1) ** c)
                assert torch.all(wav[i, costs[i]:] == 0)


def test_generate_batch_dp_single_process():
    from zipvoice_amd.dist import generate_batch_dp
    wav, lens, (lo, hi) = generate_batch_dp(
        [0, 1, 2], lambda s: (torch.ones((len(s), 4)), torch.full((len(s),), 4)))
    assert (lo, hi) == (0, 3) and wav.shape == (3, 4) and lens.tolist() == [4, 4, 4]
    with pytest.raises(ValueError):
        generate_batch_dp([0, 1], lambda s: (torch.ones((1, 4)), torch.ones(1)))

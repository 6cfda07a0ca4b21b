"""Multi-process replica exchange (smore_amd/dist.py) on CPU with gloo,
world_size 2: the snapshot-delta all-reduce applies every rank's updates
exactly once (sum), averages them (mean) or scales them per row (adaptive)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mean, out, overlap=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from smore_amd.dist import DeltaAllReduce, OverlapSync
    torch.manual_seed(0)
    base = [torch.randn(50, 8), torch.randn(50, 8)]
    tabs = [b.clone() for b in base]
    sync = OverlapSync(tabs, mean=mean) if overlap else DeltaAllReduce(tabs, mean=mean)
    expect = [b.clone() for b in base]
    for step in range(3):
        # each rank updates disjoint and overlapping rows with its own deltas
        deltas = []
        for r in range(world):
            g = torch.Generator().manual_seed(100 * step + r)
            deltas.append([torch.randn(50, 8, generator=g) * 0.01 for _ in tabs])
        for t, d in zip(tabs, deltas[rank]):
            t.add_(d)
        if overlap:
            sync.begin()     # folds the previous exchange in, starts this one
        else:
            sync.allreduce()
        for i in range(len(tabs)):
            tot = sum(deltas[r][i] for r in range(world))
            expect[i] += tot / world if mean else tot
    if overlap:
        sync.end()
    ok = all(torch.allclose(t, e, atol=1e-5) for t, e in zip(tabs, expect))
    same = [torch.empty_like(tabs[0]) for _ in range(world)]
    dist.all_gather(same, tabs[0])
    # synchronous: snap + sum on every rank, bit-identical replicas; overlapped:
    # each rank adds (sum - own delta) to its own values, equal within rounding
    if overlap:
        ok = ok and all(torch.allclose(same[0], x, atol=1e-6, rtol=0) for x in same)
    else:
        ok = ok and all(torch.equal(same[0], x) for x in same)
    out[rank] = int(ok)
    dist.destroy_process_group()


@pytest.mark.parametrize("overlap", [False, True])
@pytest.mark.parametrize("mean", [False, True])
def test_delta_allreduce_gloo_world2(mean, overlap):
    """Synchronous (DeltaAllReduce) and one-exchange-late (OverlapSync)
    schedules end with every rank's updates applied once on every rank."""
    ctx = mp.get_context("spawn")
    out = ctx.Array("i", [0, 0])
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, mean, out, overlap)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert list(out) == [1, 1]


def _hot_worker(rank, world, port, out):
    """Hub-row exchange between launches + the one-late full exchange."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from smore_amd.dist import OverlapSync
    torch.manual_seed(0)
    base = [torch.randn(60, 8), torch.randn(60, 8)]
    tabs = [b.clone() for b in base]
    hot = [torch.tensor([3, 17, 0, 44]), torch.tensor([59, 1, 30])]
    sync = OverlapSync(tabs, hot_idx=hot)
    expect = [b.clone() for b in base]
    for step in range(4):
        for sub in range(3):
            deltas = []
            for r in range(world):
                g = torch.Generator().manual_seed(1000 * step + 10 * sub + r)
                deltas.append([torch.randn(60, 8, generator=g) * 0.01 for _ in tabs])
            for t, d in zip(tabs, deltas[rank]):
                t.add_(d)
            sync.hot()
            for i in range(len(tabs)):
                expect[i] += sum(deltas[r][i] for r in range(world))
                # after hot(): the hub rows already hold every rank's updates
                agreed = [torch.empty_like(tabs[i][hot[i]]) for _ in range(world)]
                dist.all_gather(agreed, tabs[i][hot[i]].contiguous())
                if not all(torch.allclose(agreed[0], x, atol=1e-6, rtol=0) for x in agreed):
                    out[rank] = 0
                    return
        sync.begin()
    sync.end()
    ok = all(torch.allclose(t, e, atol=1e-5) for t, e in zip(tabs, expect))
    same = [torch.empty_like(tabs[1]) for _ in range(world)]
    dist.all_gather(same, tabs[1])
    ok = ok and all(torch.allclose(same[0], x, atol=1e-6, rtol=0) for x in same)
    out[rank] = int(ok)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_hot_row_exchange_gloo(world):
    """ReplicaSync's hub-row exchange (dist.py OverlapSync.hot) between the
    launches of a step, composed with the one-late full exchange: after every
    hot() the hub rows agree on all ranks, and at the end every rank holds
    base + every rank's every delta exactly once."""
    ctx = mp.get_context("spawn")
    out = ctx.Array("i", [0] * world)
    port = _free_port()
    procs = [ctx.Process(target=_hot_worker, args=(r, world, port, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert list(out) == [1] * world


def _adaptive_worker(rank, world, port, out):
    """The adaptive rule: OverlapSync with one per-row scale tensor per table."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from smore_amd.dist import OverlapSync
    torch.manual_seed(0)
    base = [torch.randn(40, 8), torch.randn(40, 8)]
    tabs = [b.clone() for b in base]
    g0 = torch.Generator().manual_seed(7)
    scale = [1.0 / world + (1.0 - 1.0 / world) * torch.rand(40, generator=g0) for _ in tabs]
    sync = OverlapSync(tabs, row_scale=scale)
    expect = [b.clone() for b in base]
    for step in range(3):
        deltas = []
        for r in range(world):
            g = torch.Generator().manual_seed(100 * step + r)
            deltas.append([torch.randn(40, 8, generator=g) * 0.01 for _ in tabs])
        for t, d in zip(tabs, deltas[rank]):
            t.add_(d)
        sync.begin()
        for i in range(len(tabs)):
            expect[i] += scale[i].view(-1, 1) * sum(deltas[r][i] for r in range(world))
    sync.end()
    ok = all(torch.allclose(t, e, atol=1e-5) for t, e in zip(tabs, expect))
    same = [torch.empty_like(tabs[0]) for _ in range(world)]
    dist.all_gather(same, tabs[0])
    ok = ok and all(torch.allclose(same[0], x, atol=1e-6, rtol=0) for x in same)
    out[rank] = int(ok)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_adaptive_exchange_gloo(world):
    """The adaptive exchange rule (dist.py, smore_hip.h SMORE_SYNC_ADAPTIVE):
    each row's summed one-late delta is scaled by its own factor, and at the
    end every rank holds base + sum over steps of scale * (all ranks' deltas)."""
    ctx = mp.get_context("spawn")
    out = ctx.Array("i", [0] * world)
    port = _free_port()
    procs = [ctx.Process(target=_adaptive_worker, args=(r, world, port, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert list(out) == [1] * world


def test_adaptive_scale_law():
    """s = min(1, c0 / k), scale = s + (1 - s) / N with k = rate * updates * N:
    the sum for rows with at most c0 updates per exchange, -> 1/N for hubs."""
    import numpy as np
    from smore_amd.dist import adaptive_scale
    rate = np.array([0.0, 1e-9, 64.0 / (8 * 1000), 128.0 / (8 * 1000), 1.0])
    sc = adaptive_scale(rate, 1000, 8, c0=64.0)
    assert sc[0] == 1.0 and sc[1] == 1.0 and sc[2] == 1.0
    np.testing.assert_allclose(sc[3], 0.5 + 0.5 / 8, rtol=1e-6)
    np.testing.assert_allclose(sc[4], 64.0 / 8000 + (1 - 64.0 / 8000) / 8, rtol=1e-6)

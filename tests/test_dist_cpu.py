"""bench.py's multi-rank path on CPU: world_size 2 over gloo (127.0.0.1).  Ranks hold
disjoint env shards; the only collective is the MAX-reduction of the timings."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    elapsed, kern = bench.reduce_max([1.0 + rank, 0.5 - 0.1 * rank], torch.device("cpu"))
    value = bench.throughput(dist.get_world_size(), 8192, 10, 200, elapsed)
    # per-rank synthetic action streams differ (seed 1234 + rank), as in bench.main
    g = torch.Generator().manual_seed(1234 + rank)
    a = torch.rand(4, generator=g)
    gathered = [torch.zeros(4) for _ in range(world)]
    dist.all_gather(gathered, a)
    q.put((rank, elapsed, kern, value, not torch.equal(gathered[0], gathered[1])))
    dist.destroy_process_group()


def test_bench_reduction_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, elapsed, kern, value, distinct in res:
        assert elapsed == 2.0 and kern == pytest.approx(0.5)
        assert value == pytest.approx(2 * 8192 * 10 * 200 / 2.0)
        assert distinct


def _record(rank, step, E, C, K):
    """synthetic record of `rank` for pushes step*K .. step*K + K - 1: obs [K, E, C, 38] etc. (K = 1: no step dim)"""
    import torch
    ks = torch.arange(K, dtype=torch.float32) + step * K
    obs = (100.0 * rank + ks).view(K, 1, 1, 1) + torch.arange(38.0) + torch.zeros(K, E, C, 38)
    rew = (-0.05 * (rank + 1) + ks).view(K, 1, 1) + torch.zeros(K, E, C)
    cf = (4 * rank + ks.to(torch.uint8)).view(K, 1, 1).expand(K, E, C).contiguous()
    ef = torch.stack([torch.tensor([rank, int(k), 8 + rank], dtype=torch.uint8) for k in ks.tolist()])
    if K == 1:
        return obs[0], rew[0], cf[0], ef[0]
    return obs, rew, cf, ef


def _gather_worker(rank, world, port, q, K):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from nascargymnasium_amd.gather import ObsGather
    E, C = 3, 2
    g = ObsGather(E, C, torch.device("cpu"), steps=K)
    got, held = [], None
    for step in range(3):
        g.push(*_record(rank, step, E, C, K))
        if held is not None:    # the previous record's views survive one more push (double-buffered receive)
            got.append(("held", step - 1, {k: v.numpy().copy() for k, v in held.items()}))
        r = g.received()
        if r is not None:
            # numpy copies: tensors in an mp queue travel by shared-memory handle, which dies with this process
            got.append(("now", step, {k: v.numpy().copy() for k, v in r.items()}))
        held = r
    q.put((rank, got))
    dist.destroy_process_group()


@pytest.mark.parametrize("K", [1, 4])
def test_obs_gather_world2(K):
    """ObsGather (the optional cfg4 gather of obs/reward/flags to rank 0) over gloo, world size 2: per-step records
    (K = 1) and K-step trajectory records; received() returns exactly the last push, and the views of the push before
    it still hold that record after the next push."""
    import torch
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_gather_worker, args=(r, 2, port, q, K)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[1] == []
    assert [(w, s) for w, s, _ in res[0]] == [("now", 0), ("held", 0), ("now", 1), ("held", 1), ("now", 2)]
    lead = (K,) if K > 1 else ()
    for _, step, r in res[0]:
        assert r["obs"].shape == (2,) + lead + (3, 2, 38)
        for rank in range(2):
            obs, rew, cf, ef = _record(rank, step, 3, 2, K)
            assert torch.equal(torch.from_numpy(r["obs"][rank]), obs)
            assert torch.equal(torch.from_numpy(r["reward"][rank]), rew)
            assert torch.equal(torch.from_numpy(r["car_flags"][rank]), cf)
            assert torch.equal(torch.from_numpy(r["env_flags"][rank]), ef)

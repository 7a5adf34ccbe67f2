"""Experiment: the headline workload (daytona 8192x10, noisy driver, staggered ages) split into S engine handles
of E/S envs, each stepped on its own HIP stream, vs one handle.  Kernel tails of one shard can overlap the bulk
of another's.  Usage: python tools/streams_exp.py S [S ...]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from nascargymnasium_amd.batched import BatchedCarEnv  # noqa: E402
from nascargymnasium_amd.track import track_path  # noqa: E402


def run(S, E=8192, C=10, settle=10800, W=20, K=200, barrier=False):
    dev = torch.device("cuda", 0)
    n = E // S
    envs = [BatchedCarEnv(n, C, track_path("daytona"), device=dev) for _ in range(S)]
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    at = bench.stagger_schedule(E, settle)
    plans = []
    for s, env in enumerate(envs):
        env.reset()
        a = at[s * n:(s + 1) * n]
        plans.append((torch.from_numpy(a).to(dev), set(int(x) for x in a[a >= 0])))
    torch.cuda.synchronize()
    t = time.perf_counter()
    for k in range(settle):
        for s, env in enumerate(envs):
            with torch.cuda.stream(streams[s]):
                if k in plans[s][1]:
                    env.reset((plans[s][0] == k).to(torch.uint8))
                env.step_driven(3, seed=s, step=k)
    torch.cuda.synchronize()
    ts = time.perf_counter() - t

    main = torch.cuda.current_stream(dev)
    fork = torch.cuda.Event()
    joins = [torch.cuda.Event() for _ in range(S)]

    def steps(first, m):
        for i in range(first, first + m):
            if barrier:                   # per-step fork from / join into the caller's stream (engine semantics)
                fork.record(main)
            for s, env in enumerate(envs):
                with torch.cuda.stream(streams[s]):
                    if barrier:
                        streams[s].wait_event(fork)
                    env.step_driven(3, seed=s, step=i)
                    if barrier:
                        joins[s].record(streams[s])
            if barrier:
                for j in joins:
                    main.wait_event(j)

    steps(settle, W)
    torch.cuda.synchronize()
    t = time.perf_counter()
    steps(settle + W, K)
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    dis = sum(float(((e.car_flags & 1) != 0).float().mean()) for e in envs) / S
    print(f"S={S}{' barrier' if barrier else ''}: {el / K * 1e3:.4f} ms/step  {E * C * K / el:.3e} car-steps/s  settle {ts:.1f}s  disabled {dis:.3f}",
          flush=True)
    for e in envs:
        e.close()


if __name__ == "__main__":
    for s in sys.argv[1:]:
        run(int(s.rstrip("b")), barrier=s.endswith("b"))

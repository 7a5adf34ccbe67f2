"""Benchmark: batched CarEnv.step throughput (car-steps/s = envs x cars x steps / s).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs E] [--cars C] [--track daytona]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, weak scaling)

Workload (BASELINE.json metric "env-steps/sec (cars x envs), daytona 10-car"): E=8192 envs x C=10
cars on daytona.track per GPU, synthetic uniform U[-1,1]^2 actions pre-generated in HBM, SB3-style
auto-reset on done.  A "step" = one fused kernel launch over all E*C cars of a rank.
Prints ONE JSON line on rank 0 (schema: see DESIGN.md "Measurement").
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

ALGO_BYTES_PER_CAR_STEP = 1221      # 2 x 528 B state + 8 B action + 152 B obs + 4 B reward + 1 B flags
HBM_PEAK_GBS = 8000.0               # MI355X HBM3E spec (MI355X_MICROARCH.md)


def _oracle_shard(track, cars, E, seed, budget_s, out, slot):
    """One host thread: its own OracleEnv shard of E envs x C cars, uniform actions, ~budget_s of stepping
    (the oracle's C step releases the GIL inside ctypes, so shards on threads run in parallel)."""
    import numpy as np
    from oracle_lib import OracleEnv
    env = OracleEnv(track, E, cars)
    env.reset()
    acts = np.random.default_rng(seed).uniform(-1, 1, (64, E, cars, 2)).astype(np.float32)
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        env.step(acts[steps % 64])
        steps += 1
    out[slot] = (E * cars * steps, time.perf_counter() - t0)
    env.close()


def cpu_baseline(track, cars, budget_s=12.0, threads=None):
    """The CPU oracle (C restatement of the reference path) on a bounded sample of the same workload:
    16 envs x C cars per shard, uniform actions.  First 1 thread for budget_s / 2, then one shard per
    host thread (threads = the box's CPU share, at most 16) for budget_s / 2 of wall time; `value` is the
    multi-thread rate (car-steps over the slowest shard's time), the 1-thread rate is in `sample`."""
    import threading
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    E = 16
    if threads is None:
        threads = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()))
    one = [None]
    _oracle_shard(track, cars, E, 0, budget_s / 2, one, 0)
    rate1 = one[0][0] / one[0][1]
    res = [None] * threads
    th = [threading.Thread(target=_oracle_shard, args=(track, cars, E, k, budget_s / 2, res, k)) for k in range(threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    rate = sum(r[0] for r in res) / max(r[1] for r in res)
    return {"value": rate, "unit": "car-steps/s", "cores": threads, "kind": "port",
            "sample": f"oracle (C restatement of the reference path incl. Box2D subset) on {os.path.basename(track)}, "
                      f"uniform actions: {threads} host threads x one shard of {E} envs x {cars} cars, "
                      f"~{budget_s / 2:.0f} s each; 1 thread alone: {rate1:.0f} car-steps/s"}


def reduce_max(values, device):
    """MAX over ranks of per-rank timings (no-op at world size 1).  Ranks own disjoint env shards and
    never exchange simulation data: this is the only collective in the benchmark."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [float(v) for v in values]
    t = torch.tensor([float(v) for v in values], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.tolist()]


def throughput(world, envs, cars, steps, elapsed_max):
    """whole-job car-steps/s under weak scaling: every rank steps its own envs x cars."""
    return world * envs * cars * steps / elapsed_max


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--envs", type=int, default=8192)
    ap.add_argument("--cars", type=int, default=10)
    ap.add_argument("--track", default="daytona")
    ap.add_argument("--policy", default="uniform", choices=["uniform", "driver", "sac"],
                    help="uniform: U[-1,1]^2 resident in HBM; driver: device rule driver; sac: fused SAC actor "
                         "(random-init weights of the reference architecture) on the previous observation")
    ap.add_argument("--mixed", action="store_true", help="env e on track e mod 8 of the sorted bundled tracks "
                    "(BASELINE cfg5: mixed batch, divergent geometry); --track is ignored")
    ap.add_argument("--gather", action="store_true", help="gather every step's obs/reward/flags of all ranks to "
                    "rank 0 (RCCL, side stream; BASELINE cfg4 single-learner layout)")
    ap.add_argument("--cpu-threads", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from nascargymnasium_amd.batched import BatchedCarEnv
    from nascargymnasium_amd.track import track_path

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    E, C, K, W = args.envs, args.cars, args.steps, args.warmup
    tpath = track_path(args.track)
    if args.mixed:
        from nascargymnasium_amd.track import available_tracks
        names = available_tracks()
        env = BatchedCarEnv(E, C, [names[e % len(names)] for e in range(E)], device=dev)
    else:
        env = BatchedCarEnv(E, C, tpath, device=dev)
    gather = None
    if args.gather:
        from nascargymnasium_amd.gather import ObsGather
        gather = ObsGather(E, C, dev)
    if args.policy == "sac":
        from nascargymnasium_amd.policy import random_actor
        env.set_actor(random_actor(rank))
    env.reset()
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + rank)
    if args.policy == "uniform":
        acts = torch.rand((W + K, E, C, 2), generator=gen, device=dev) * 2 - 1     # resident before timing
    torch.cuda.synchronize()

    pol = {"driver": 1, "sac": 2}.get(args.policy)

    def one_step(i):
        a = acts[i] if args.policy == "uniform" else env.policy_actions(pol, seed=rank, step=i)
        env.launch_step(a, auto_reset=True)
        if gather is not None:
            gather.push(env.obs, env.reward, env.car_flags, env.env_flags)

    for i in range(W):
        one_step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # timed region: K steps back to back (no per-step events: each event record costs ~5 us of device
    # time between kernels on this stack, which would be charged to the throughput)
    t0 = time.perf_counter()
    for i in range(W, W + K):
        one_step(i)
    if gather is not None:
        gather.wait()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # roofline pass (after the timed region): HIP events on the launch stream around each env step's
    # kernels (model_kernel + logic_kernel + sensor_kernel), averaged over KR further steps
    KR = min(K, 50)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(KR)]
    for i in range(KR):
        a = acts[W + i] if args.policy == "uniform" else env.policy_actions(pol, seed=rank, step=W + K + i)
        ev[i][0].record()
        env.launch_step(a, auto_reset=True)
        ev[i][1].record()
    torch.cuda.synchronize()
    kern_ms = sum(s.elapsed_time(e) for s, e in ev) / KR
    errs = int(((env.car_flags & 128) != 0).sum().item())
    elapsed, kern_ms = reduce_max([elapsed, kern_ms], dev)
    value = throughput(world, E, C, K, elapsed)
    achieved = E * C * ALGO_BYTES_PER_CAR_STEP / (kern_ms * 1e-3) / 1e9
    traffic = None
    tfile = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tfile):
        try:
            tj = json.load(open(tfile))
            if tj.get("envs") == E and tj.get("cars") == C and tj.get("track") == os.path.basename(tpath):
                traffic = tj.get("bytes_per_step")
        except Exception:
            traffic = None
    out = {
        "metric": "env-steps/sec (cars x envs), daytona 10-car",
        "value": value, "unit": "car-steps/s", "n_gpus": world, "steps": K, "warmup": W,
        "ms_per_step": elapsed / K * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f32+f64", "data": "synthetic",
        "config": {"workload": f"{'mixed 8-track' if args.mixed else os.path.basename(tpath)[:-6]} {C}-car: {E} envs x {C} cars per GPU, "
                               f"{ {'uniform': 'uniform U[-1,1]^2 actions resident in HBM', 'driver': 'on-device rule driver', 'sac': 'fused SAC actor (random-init) closed loop'}[args.policy]}, auto-reset",
                   "envs_per_gpu": E, "cars_per_env": C, "track": "mixed (env e: track e mod 8)" if args.mixed else os.path.basename(tpath),
                   "parallelism": f"dp{world} (env shards" + (", RCCL gather of obs/reward/flags to rank 0 per step)" if gather else ", no collective)")},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "model_kernel + logic_kernel + ray_sensor_kernel (one env step)", "kernel_ms": kern_ms,
                     "algo_bytes_per_car_step": ALGO_BYTES_PER_CAR_STEP},
        "engine_errors": errs,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(tpath, C, args.cpu_budget, args.cpu_threads)
    if rank == 0:
        print(json.dumps(out), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

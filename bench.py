"""Benchmark: batched CarEnv.step throughput (car-steps/s = envs x cars x steps / s).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs E] [--cars C] [--track daytona] [--policy noisy]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, weak scaling)

Headline workload (BASELINE.json metric "env-steps/sec (cars x envs), daytona 10-car"; SURVEY.md 8(d) action
source (B)): E=8192 envs x C=10 cars on daytona.track per GPU, driven closed loop by the on-device noisy rule
driver (BaseController._fallback_control, game/control/base_controller.py:39-103, with 15 % of car-steps
replaced by a counter-hash uniform action), SB3-style auto-reset.  Before timing, the envs are SETTLED to a
steady state: 10 800 steps (one 180 s episode) during which env e is reset at a staggered step, so that the
env ages at the start of the timed window are spread uniformly over the episode -- cars are spread round the
track, touch walls, complete laps, get disabled and auto-reset inside the timed window (the rates are reported
in `workload_stats`).  A "step" = one env step over all E*C cars of a rank: model_logic_kernel (the noisy driver,
the vehicle + tyre model, the Box2D step and the env logic in one launch; nascar_set_fused_logic(h, 0) splits it
into model_kernel + logic_kernel) then ray_sensor_kernel, issued on the sharded rollout schedule (4 env shards on 4
streams, 50 steps per nascar_rollout call; bit-identical to one whole-batch launch per step).  The uniform-U[-1,1]^2-from-reset number of round 1 is kept
only as the labelled secondary field `uniform_from_reset`.
Prints ONE JSON line on rank 0 (schema: see DESIGN.md "Measurement").
"""
import argparse
import glob
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

ALGO_BYTES_PER_CAR_STEP = 1221      # 2 x 528 B state + 8 B action + 152 B obs + 4 B reward + 1 B flags
# model_kernel's own share (the dominant kernel's roofline): the SURVEY Appendix B state it reads and writes -- Box2D
# body 7 + contacts 56 + listener 4 + car 27 + tyres 12 = 106 words, read + written -- plus the 8 B action
MODEL_ALGO_BYTES_PER_CAR = 2 * 106 * 4 + 8
# model_logic_kernel (the default: vehicle model + Box2D step + env logic in one launch): the whole step's bytes but
# the sensor kernel's 64 B of obs[22:38] -- every state word read and written, the action, obs[0:22], reward, flags
FUSED_ALGO_BYTES_PER_CAR = ALGO_BYTES_PER_CAR_STEP - 16 * 4
HBM_PEAK_GBS = 8000.0               # MI355X HBM3E spec (MI355X_MICROARCH.md)
EPISODE_STEPS = 10800               # 180 s time limit at dt = 1/60 (src/car_env.py:1154)
POLICY_ID = {"uniform": 0, "driver": 1, "sac": 2, "noisy": 3}
POLICY_TEXT = {"uniform": "uniform U[-1,1]^2 actions resident in HBM",
               "driver": "on-device rule driver (BaseController._fallback_control), closed loop",
               "noisy": "on-device noisy rule driver (BaseController._fallback_control, 15% of car-steps "
                        "uniform), closed loop",
               "sac": "fused SAC actor (random-init weights of the reference architecture), closed loop"}


def source_sha():
    """sha256 over the HIP sources: tags the PMC traffic file so a stale one is never reported as current."""
    h = hashlib.sha256()
    for p in sorted(glob.glob(os.path.join(ROOT, "nascargymnasium_amd", "csrc", "*"))):
        h.update(open(p, "rb").read())
    return h.hexdigest()[:16]


def _oracle_shard(track, cars, E, seed, budget_s, out, slot, init=None, init_seed=0):
    """One host thread: its own OracleEnv shard of E envs x C cars driven by the host restatement of the
    noisy rule driver (tests/drivers.py, same counter hash as the device), auto-reset, ~budget_s of stepping
    (the oracle's C step releases the GIL inside ctypes, so shards on threads run in parallel)."""
    import numpy as np
    from drivers import NoisyRuleDriver
    from oracle_lib import OracleEnv, inject_gpu_state
    env = OracleEnv(track, E, cars)
    step0 = 0
    if init is None:
        drv = NoisyRuleDriver(E * cars, seed)
        obs = env.reset()[0]
    else:   # continue from the GPU's steady state: envs `genvs` of the GPU's E_gpu x cars engine, driver state included
        blob, E_gpu, genvs, gobs, step0 = init
        # the driver's noise keyed by the cars' global ids on the GPU, from the GPU's next step index: the sample
        # continues the GPU run's own action stream (tests/test_gpu_configs.py pins this host driver at full size)
        drv = NoisyRuleDriver(E * cars, init_seed, ids=[g * cars + c for g in genvs for c in range(cars)])
        rows = inject_gpu_state(env, blob, E_gpu, cars, genvs)
        drv.tb = rows[:, 0].copy()
        drv.steer, drv.last, drv.lim = (rows[:, j].astype(np.float32) for j in (1, 2, 3))
        obs = np.ascontiguousarray(gobs[genvs])
    steps, contact, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        obs, _, cf, ef = env.step(drv.actions(obs, step0 + steps))
        contact += int(((cf & 4) != 0).sum())   # car flag bit 2: collision impulse this step (as the GPU tally)
        for e in np.nonzero((ef[:, 0] != 0) | (ef[:, 1] != 0))[0]:
            env.reset(int(e))
            obs = env.outputs()[0]
        steps += 1
    out[slot] = (E * cars * steps, time.perf_counter() - t0, steps, contact)
    env.close()


def host_cores():
    """(threads to use, description): every core this process may run on -- its affinity mask, capped by a cgroup
    CPU quota and by the host's declared CPU share when set: NASCAR_CPU_SHARE, else OMP_NUM_THREADS (on the GPU box the
    affinity mask lists the whole machine while the job's share, OMP_NUM_THREADS, is 16 cores, and more threads than the
    share only time-slice).  When the share is what binds, the description says so: an OMP_NUM_THREADS set for another
    reason (e.g. 1) would shrink the baseline -- override with NASCAR_CPU_SHARE or --cpu-threads."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        pass
    model = "unknown CPU"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    share, share_var = None, None
    for var in ("NASCAR_CPU_SHARE", "OMP_NUM_THREADS"):
        try:
            if os.environ.get(var):
                share, share_var = int(os.environ[var]), var
                break
        except ValueError:
            pass
    n = min([aff] + [x for x in (quota, share) if x])
    binding = share is not None and share == n and share < min([aff] + ([quota] if quota else []))
    return n, (f"{model}; affinity {aff} cores" + (f", cgroup quota {quota} cores" if quota else ", no cgroup quota")
               + (f", declared CPU share {share_var}={share}" if share else "")
               + (f" (the binding limit; NASCAR_CPU_SHARE or --cpu-threads override it)" if binding else "")
               + f"; {n} threads used")


def cpu_baseline(track, cars, budget_s=12.0, threads=None, steady=None):
    """The CPU oracle (C restatement of the reference path) on a bounded sample of the same workload:
    16 envs x C cars per shard, noisy rule driver -- from the GPU run's steady state when `steady` = (state blob,
    E, obs [E][C][38], step, driver seed) is given (each shard continues 16 of the GPU's envs, every field, contact
    and driver state injected: tests/oracle_lib.inject_gpu_state, tested bit-exact against the GPU), else from
    reset.  First 1 thread for budget_s / 2, then one shard per host thread (threads = every core the process may
    use, host_cores()) for budget_s / 2 of wall time; `value` is the multi-thread rate (car-steps over the slowest
    shard's time), the 1-thread rate is in `sample`."""
    import threading
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    E = 16
    n_host, host_txt = host_cores()
    if threads is None:
        threads = n_host

    def init(k):
        if steady is None:
            return None
        blob, E_gpu, gobs, step0, _ = steady
        stride = max(1, E_gpu // (E * (threads + 1)))   # shards spread over the GPU's envs (ages uncorrelated)
        genvs = [((k * E + i) * stride) % E_gpu for i in range(E)]
        return blob, E_gpu, genvs, gobs, step0
    seed = steady[4] if steady is not None else 0
    one = [None]
    _oracle_shard(track, cars, E, 0, budget_s / 2, one, 0, init(threads), seed)
    rate1 = one[0][0] / one[0][1]
    res = [None] * threads
    th = [threading.Thread(target=_oracle_shard, args=(track, cars, E, k, budget_s / 2, res, k, init(k), seed))
          for k in range(threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    rate = sum(r[0] for r in res) / max(r[1] for r in res)
    contact = sum(r[3] for r in res) / max(1, sum(r[0] for r in res))
    return {"value": rate, "unit": "car-steps/s", "cores": threads, "kind": "port",
            "host": host_txt,
            "sample": f"oracle (C restatement of the reference path incl. Box2D subset) on {os.path.basename(track)}, "
                      + (f"noisy rule driver continuing the GPU run's steady state ({min(r[2] for r in res)}+ steps; "
                         f"each shard's 16 envs injected from the GPU's state, driver state included)"
                         if steady is not None else
                         f"noisy rule driver from reset (first ~{min(r[2] for r in res)} steps)")
                      + f": {threads} host threads x one shard of {E} envs x {cars} cars, "
                      f"~{budget_s / 2:.0f} s each; 1 thread alone: {rate1:.0f} car-steps/s; wall contact in "
                      f"{100 * contact:.2f} % of the sample's car-steps (the GPU window's workload_stats.contact_frac "
                      f"is the steady state's); host: {host_txt}"}


COLLECTIVES = []    # this rank's collective calls in issue order (reported by --plumbing runs; every rank must match)


def _dist_on():
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def barrier():
    import torch.distributed as dist
    if _dist_on():
        COLLECTIVES.append("barrier")
        dist.barrier()


def sync(dev):
    """wait for the device's queued work (no-op for the --plumbing engine on the CPU)"""
    import torch
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


class HostEvent:
    """torch.cuda.Event's record / elapsed_time on the host clock (the --plumbing engine has no device)"""

    def __init__(self):
        self.t = None

    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, end):
        return (end.t - self.t) * 1e3


def new_event(dev):
    import torch
    return torch.cuda.Event(enable_timing=True) if dev.type == "cuda" else HostEvent()


def reduce_max(values, device):
    """MAX over ranks of per-rank timings (no-op at world size 1).  Ranks own disjoint env shards and
    never exchange simulation data: this is the only collective in the benchmark."""
    import torch
    import torch.distributed as dist
    if not _dist_on():
        return [float(v) for v in values]
    COLLECTIVES.append(f"all_reduce_max[{len(values)}]")
    t = torch.tensor([float(v) for v in values], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.tolist()]


def reduce_sum(values, device):
    import torch
    import torch.distributed as dist
    if not _dist_on():
        return [float(v) for v in values]
    COLLECTIVES.append(f"all_reduce_sum[{len(values)}]")
    t = torch.tensor([float(v) for v in values], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(x) for x in t.tolist()]


def gather_all(value, device):
    """every rank's value (rank order; [value] at world size 1) -- the per-rank timings the MAX is taken over"""
    import torch
    import torch.distributed as dist
    if not _dist_on():
        return [float(value)]
    COLLECTIVES.append("all_gather[1]")
    t = torch.tensor([float(value)], device=device, dtype=torch.float64)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(x.item()) for x in out]


def launch_ranks(n, argv):
    """`bench.py --gpus N` (N > 1) outside a torchrun environment: start the N ranks as one child
    `python -m torch.distributed.run --nproc-per-node N ... bench.py <same args>` (the driver's own launch line),
    rendezvous on 127.0.0.1, and return its exit code.  The parent never initialises the GPU and never execs (a
    process that has touched the GPU must not replace itself); it only waits.  The reference scales the same way, by
    processes (learn/ppo.py:77, SubprocVecEnv)."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def track_cache_prebuild(files, rank, world, beam_cell):
    """Multi-rank runs share one build per track (verdict r05 item 5): the host-built track tables go to an on-disk cache
    (NASCAR_TRACK_CACHE, default <tmp>/nascargymnasium_amd_tracks_<uid> when world > 1) and each rank prebuilds the
    job's tracks there before its engine starts -- host only, in an order rotated by the rank, so the ranks build
    different tracks at once and load the others' (a lock file per track: each is built once per node).  Returns
    (directory, built, loaded, seconds) or None (world 1 with no cache set: the engine builds in memory)."""
    import tempfile
    d = os.environ.get("NASCAR_TRACK_CACHE")
    if not d:
        if world <= 1:
            return None
        d = os.path.join(tempfile.gettempdir(), f"nascargymnasium_amd_tracks_{os.getuid()}")
        os.environ["NASCAR_TRACK_CACHE"] = d
    from nascargymnasium_amd import _lib
    _lib.set_track_cache(int(os.environ.get("NASCAR_TRACK_RETAIN", "8")), d)
    uniq = sorted(set(files))
    t0, built, loaded = time.perf_counter(), 0, 0
    for k in range(len(uniq)):
        if _lib.prebuild_track(uniq[(k + rank) % len(uniq)], beam_cell if beam_cell is not None else 1.0):
            loaded += 1
        else:
            built += 1
    return d, built, loaded, time.perf_counter() - t0


def throughput(world, envs, cars, steps, elapsed_max):
    """whole-job car-steps/s under weak scaling: every rank steps its own envs x cars."""
    return world * envs * cars * steps / elapsed_max


def stagger_schedule(E, settle):
    """settle step at which env e is reset so that its age when timing starts is floor(pi(e) * 10800 / E) steps,
    pi a fixed (seeded) random permutation: ages spread uniformly over one episode and uncorrelated with the env
    index -- as after many episodes that end at different times -- rather than adjacent envs (one workgroup's)
    being one step apart and driving the same stretch of track together.  Envs whose age would exceed the settle
    length are not reset."""
    import numpy as np
    perm = np.random.default_rng(20261016).permutation(E).astype(np.int64)
    age = (perm * EPISODE_STEPS) // E
    at = settle - age
    return np.where(age < settle, at, -1)


class Stepper:
    """bench steps on a BatchedCarEnv.  Per-step path (rollout == 0): actions from the chosen source, then one env
    step with auto-reset (nascar_policy_actions + nascar_step).  Fused path (rollout = R > 0, device action sources
    0/1/3): R steps per nascar_rollout launch, identical results (tests/test_gpu_rollout.py)."""

    def __init__(self, env, policy, seed, acts=None, gather=None, rollout=0):
        self.env, self.pol, self.seed, self.acts, self.gather = env, POLICY_ID[policy], seed, acts, gather
        # device action sources (policy 2, the SAC actor, only on the sharded schedule) step through nascar_rollout
        self.R = rollout if (acts is None and (self.pol != 2 or env.rollout_streams > 0)) else 0
        self.traj = None
        self.gtraj = None

    def actions(self, i):
        if self.acts is not None:
            return self.acts[i % self.acts.shape[0]]
        return self.env.policy_actions(self.pol, seed=self.seed, step=i)

    def __call__(self, i):
        if self.gather is not None and self.R:
            self.run(i, 1)
            return
        if self.acts is None and self.pol != 2:   # device driver computed inside the step launch (nascar_step_driven)
            self.env.step_driven(self.pol, seed=self.seed, step=i, auto_reset=True)
        else:
            self.env.launch_step(self.actions(i), auto_reset=True)
        if self.gather is not None:
            self.gather.push(self.env.obs, self.env.reward, self.env.car_flags, self.env.env_flags)

    def run(self, first, K, trajectory=False):
        """K steps starting at step index `first` (trajectory: per-step records of a fused launch in self.traj)"""
        if not self.R:
            for i in range(first, first + K):
                self(i)
            return
        import torch
        if self.gather is not None:   # K-step trajectory records (obs after every step + rewards / flags) to rank 0
            e = self.env
            if self.gtraj is None:
                self.gtraj = (torch.empty(self.R + 1, e.E, e.C, 38, dtype=torch.float32, device=e.device),
                              torch.empty(self.R, e.E, e.C, dtype=torch.float32, device=e.device),
                              torch.empty(self.R, e.E, e.C, dtype=torch.uint8, device=e.device),
                              torch.empty(self.R, e.E, dtype=torch.uint8, device=e.device))
            k = 0
            while k < K:
                n = min(self.R, K - k)
                ot, rew, cf, ef = e.rollout(self.pol, n, seed=self.seed, step0=first + k, auto_reset=True,
                                            trajectory=True, obs_trajectory=True, out=self.gtraj)
                self.gather.push(ot[1:n + 1], rew[:n], cf[:n], ef[:n])
                k += n
            return
        if trajectory and (self.traj is None or self.traj[0].shape[0] < K):
            e = self.env
            self.traj = (torch.empty(K, e.E, e.C, dtype=torch.float32, device=e.device),
                         torch.empty(K, e.E, e.C, dtype=torch.uint8, device=e.device),
                         torch.empty(K, e.E, dtype=torch.uint8, device=e.device))
        k = 0
        while k < K:
            n = min(self.R, K - k) if not trajectory else K
            self.env.rollout(self.pol, n, seed=self.seed, step0=first + k, auto_reset=True, trajectory=trajectory,
                             out=self.traj if trajectory else None)
            k += n


class PlumbingEngine:
    """--plumbing (CPU tests): a stand-in for BatchedCarEnv with exactly the interface main() uses, on the CPU.  A step
    sleeps (rank + 1) ms and writes deterministic outputs, so a gloo world-2 run goes through main()'s own settle,
    timing, statistics and kernel passes, per-step pass, secondary pass, every collective and the JSON line without a
    GPU.  Not a measurement (the line's metric says so)."""

    def __init__(self, E, C, rank, device):
        import torch
        self.E, self.C, self.N, self.rank, self.device = E, C, E * C, rank, torch.device(device)
        self.obs = torch.zeros(E, C, 38, dtype=torch.float32)
        self.reward = torch.zeros(E, C, dtype=torch.float32)
        self.car_flags = torch.zeros(E, C, dtype=torch.uint8)
        self.env_flags = torch.zeros(E, dtype=torch.uint8)
        self._actions = torch.zeros(E, C, 2, dtype=torch.float32)
        self.envs_per_block, self.fused_logic, self.rollout_streams = max(1, 128 // C), True, 4
        self._events, self.steps_done = None, 0

    def set_rollout_streams(self, streams=4):
        self.rollout_streams = int(streams)

    def set_rollout_pipe(self, sensor_workgroups=0):
        self.rollout_pipe = int(sensor_workgroups)

    def set_car_contact(self, enable=True):
        pass

    def set_actor(self, weights, precision="fp32"):
        pass

    def reset(self, env_mask=None):
        if env_mask is None:
            self.obs.zero_()
        else:
            self.obs[env_mask.bool()] = 0.0
        return self.obs

    def _advance(self, step):
        import torch
        ev = self._events
        if ev:
            ev[0].record()
        time.sleep((self.rank + 1) * 1e-3)
        if ev:
            ev[1].record()
            ev[2].record()
        n = torch.arange(self.N).view(self.E, self.C)
        self.obs.fill_(float(step))
        self.obs[..., 4] = 0.25
        self.reward.fill_(float(self.rank))
        self.car_flags.copy_((((n + step) % 7 == 0).to(torch.uint8) * 4) | (((n + step) % 11 == 0).to(torch.uint8) * 8))
        self.env_flags.copy_(((torch.arange(self.E) + step) % 50 == 0).to(torch.uint8) * 8)
        self.steps_done += 1
        if ev:
            ev[3].record()

    def policy_actions(self, policy, seed=0, step=0, obs=None):
        return self._actions

    def launch_step(self, actions, auto_reset=False, terminal_obs=False):
        self._advance(self.steps_done)

    def step_driven(self, policy, seed=0, step=0, auto_reset=True, terminal_obs=False):
        self._advance(step)
        return self.obs, self.reward

    def rollout(self, policy, steps, seed=0, step0=0, auto_reset=True, trajectory=False, out=None,
                obs_trajectory=False):
        import torch
        E, C = self.E, self.C
        if trajectory:
            if out is None:
                out = ((torch.empty(steps + 1, E, C, 38),) if obs_trajectory else ()) + (
                    torch.empty(steps, E, C), torch.empty(steps, E, C, dtype=torch.uint8),
                    torch.empty(steps, E, dtype=torch.uint8))
            ot = out[0] if obs_trajectory else None
            rew, cf, ef = out[-3:]
            if ot is not None:
                ot[0].copy_(self.obs)
        for k in range(steps):
            self._advance(step0 + k)
            if trajectory:
                rew[k].copy_(self.reward); cf[k].copy_(self.car_flags); ef[k].copy_(self.env_flags)
                if ot is not None:
                    ot[k + 1].copy_(self.obs)
        if not trajectory:
            return self.obs, self.reward, self.car_flags, self.env_flags
        return (ot if ot is not None else self.obs), rew, cf, ef

    def set_step_events(self, events=None):
        self._events = events

    def get_state(self):
        return self.obs.clone().view(-1).view(__import__("torch").uint8)

    def set_state(self, buf):
        self.obs.view(-1).view(__import__("torch").uint8).copy_(buf)

    def close(self):
        pass


def settle(env, step, n, stagger, dev):
    """bring the envs to the steady state of the workload (not timed): n closed-loop steps, env e reset at
    its staggered step."""
    import torch
    if n <= 0:
        return
    at = stagger_schedule(env.E, n) if stagger else None
    at_dev = torch.from_numpy(at).to(dev) if stagger else None
    steps_with_reset = set(int(x) for x in at[at >= 0]) if stagger else set()
    if step.R:   # fused path: launches of up to R steps, the staggered resets applied at launch boundaries
        k = 0
        while k < n:
            m = min(step.R, n - k)
            lo, hi = k, k + m
            if stagger:
                sel = (at_dev >= lo) & (at_dev < hi)
                if bool(sel.any()):
                    env.reset(sel.to(torch.uint8))
            step.run(k, m)
            k += m
        return
    for k in range(n):
        if k in steps_with_reset:
            env.reset((at_dev == k).to(torch.uint8))
        step(k)


def timed(step, first, K, world):
    """K steps back to back between a barrier + device synchronisation on both sides; this rank's wall time"""
    dev = step.env.device
    sync(dev)
    barrier()
    sync(dev)
    # K steps back to back (no per-step events: each event record costs ~5 us of device time between kernels
    # on this stack, which would be charged to the throughput)
    diag = os.environ.get("NASCAR_BENCH_DIAG")
    if diag:      # where the window's wall time goes: GPU span (2 events) vs host enqueue vs sync
        e0, e1 = new_event(dev), new_event(dev)
        e0.record()
    t0 = time.perf_counter()
    step.run(first, K)
    t_enq = time.perf_counter() - t0
    if diag:
        e1.record()
    if step.gather is not None:
        step.gather.wait()
    sync(dev)
    barrier()
    el = time.perf_counter() - t0
    if diag:
        print(f"[diag] K={K} wall {el * 1e3:.3f} ms, gpu span {e0.elapsed_time(e1):.3f} ms, host enqueue "
              f"{t_enq * 1e3:.3f} ms", file=sys.stderr, flush=True)
    if getattr(step.env, "rollout_pipe", 0) and hasattr(step.env, "rollout_pipe_status") and step.env.rollout_pipe_status():
        raise RuntimeError("a pipelined rollout gave up on a bounded device wait: the timed steps are not valid")
    return el


def stats_pass(env, step, first, KR):
    """after the timed region, KR further steps of the same workload: HIP events on the launch stream around
    one KR-step rollout call on the timed schedule (or, on the per-step path, around each env step's
    model_logic_kernel + ray_sensor_kernel launches), and device-side tallies of what happened in those car-steps."""
    import torch
    dev = env.device
    tally = torch.zeros(7, dtype=torch.float64, device=dev)
    KR_timed = KR
    if step.R:
        e0, e1 = new_event(dev), new_event(dev)
        step.run(first, KR, trajectory=True)         # allocates the trajectory buffers outside the bracket
        e0.record()
        step.run(first + KR, KR, trajectory=True)
        e1.record()
        if step.gather is not None:                  # the gathered path: its last rollout call's records
            n = KR % step.R or step.R
            cf, ef = step.gtraj[2][:n], step.gtraj[3][:n]
            KR = n
        else:
            rew, cf, ef = step.traj
            cf, ef = cf[:KR], ef[:KR]
        tally += torch.stack([((cf & 4) != 0).sum(), ((cf & 8) != 0).sum(), ((cf & 1) != 0).sum(),
                              ((cf & 2) != 0).sum(), ((ef & 8) != 0).sum(), ((cf & 128) != 0).sum(),
                              torch.zeros((), device=env.device)]).double()
        tally[6] = env.obs[..., 4].double().sum() * KR    # speed sampled at the window's last step
        sync(dev)
        return e0.elapsed_time(e1) / KR_timed, tally.tolist(), KR
    ev = [(new_event(dev), new_event(dev)) for _ in range(KR)]
    for i in range(KR):
        a = step.actions(first + i)
        ev[i][0].record()
        env.launch_step(a, auto_reset=True)
        ev[i][1].record()
        cf, ef = env.car_flags, env.env_flags
        tally += torch.stack([((cf & 4) != 0).sum(), ((cf & 8) != 0).sum(), ((cf & 1) != 0).sum(),
                              ((cf & 2) != 0).sum(), ((ef & 8) != 0).sum(), ((cf & 128) != 0).sum(),
                              env.obs[..., 4].double().sum()]).double()
    sync(dev)
    kern_ms = sum(s.elapsed_time(e) for s, e in ev) / KR
    return kern_ms, tally.tolist(), KR


def kernel_pass(env, step, first, KR):
    """per-kernel durations of the whole-grid step (the per-step path, nascar_step_driven / nascar_step): HIP events
    recorded by the engine before model_kernel, after it, after logic_kernel and after the sensor launch, on the launch
    stream (nascar_set_step_events), over KR steps of the same workload.  Returns mean ms per launch of each kernel."""
    dev = env.device
    evs = [[new_event(dev) for _ in range(4)] for _ in range(KR)]
    for i in range(KR):
        step.env.set_step_events(evs[i])
        step(first + i)
    step.env.set_step_events(None)
    sync(dev)
    t = [[e[k].elapsed_time(e[k + 1]) for k in range(3)] for e in evs]
    return {name: sum(r[k] for r in t) / KR for k, name in enumerate(("model_kernel", "logic_kernel", "ray_sensor_kernel"))}


def _window(fn, first, K, dev):
    """K calls fn(i) back to back between device synchronisations (this rank only): seconds"""
    sync(dev)
    t0 = time.perf_counter()
    for i in range(first, first + K):
        fn(i)
    sync(dev)
    return time.perf_counter() - t0


def drop_in_pass(E, C, track, rank, dev, steady, K=100, W=10, settle_steps=EPISODE_STEPS):
    """The drop-in API's throughput (secondary, beside the headline): VecCarEnv.step -- the SB3 VecEnv that replaces
    learn/ppo.py's SubprocVecEnv(Monitor(CarEnv)) -- with device tensors (return_tensors=True), actions from the device
    noisy rule driver on the observation the previous step returned (one nascar_policy_actions launch: the learner's
    policy stands here), timed against the engine's per-step path on the same state and actions
    (policy_actions + BatchedCarEnv.launch_step with auto-reset and terminal observations).
      single_track: `track`, E x C, from the headline's settled state `steady`;
      random_track_{C}car: track_file=None, learn/ppo.py's configuration (every reset draws a new track, on the
        device), E x C, settled by its own 10 800 noisy-driver steps with staggered resets; the engine's per-step path
        is timed with random tracks on (the draws / fresh worlds / layout kernels after each step) and off.
    Each variant starts from the same state (engine arena, obs, env -> track map, draw counters)."""
    import numpy as np
    import torch
    from nascargymnasium_amd import VecCarEnv
    from nascargymnasium_amd.batched import BatchedCarEnv
    out = {}

    def vec_rate(venv):
        eng = venv.engine
        n = eng.E * eng.C
        holder = [eng.obs]

        def one(i):
            o = holder[0]
            a = eng.policy_actions(3, seed=rank, step=i, obs=o)
            holder[0] = venv.step(a)[0]
        _window(one, 0, W, dev)
        return n * K / _window(one, W, K, dev)

    def eng_rate(eng):
        def one(i):
            eng.launch_step(eng.policy_actions(3, seed=rank, step=i), auto_reset=True, terminal_obs=True)
        _window(one, 0, W, dev)
        return eng.E * eng.C * K / _window(one, W, K, dev)

    def load(eng, snap, random_tracks=None):
        """an engine that has not stepped yet, brought to snapshot (state, obs, track files, draws)"""
        state, obs, files, draws, seeds = snap
        if eng.random_track_ids is not None:
            eng.clear_random_tracks()
        eng.set_env_tracks(files)          # (applies at once: the engine has not been reset or stepped)
        eng.set_state(state)
        eng.obs.copy_(obs)
        if random_tracks is not None:
            eng.set_random_tracks(random_tracks, seeds, draws=draws)

    # single track, from the headline's steady state
    if steady is not None:
        blob, _, gobs, _, _ = steady
        venv = VecCarEnv(E, track, num_cars=C, return_tensors=True, device=dev)
        snap = (torch.from_numpy(blob).to(dev), torch.from_numpy(gobs).to(dev), [track] * E, None, None)
        load(venv.engine, snap)
        rv = vec_rate(venv)
        venv.close()
        eng = BatchedCarEnv(E, C, track, device=dev)
        load(eng, snap)
        re = eng_rate(eng)
        eng.close()
        out["single_track"] = {"config": f"{os.path.basename(track)[:-6]} {E} envs x {C} cars, steady state",
                               "vec_env": rv, "engine_per_step": re, "ratio": re / rv}
    from nascargymnasium_amd.track import available_tracks
    tracks = available_tracks()
    for c in sorted({1, C}):
        venv = VecCarEnv(E, None, num_cars=c, return_tensors=True, seed=1000 + rank, device=dev)
        eng = venv.engine
        venv.reset()
        t0 = time.perf_counter()
        settle(eng, Stepper(eng, "noisy", rank, None, None, 0), settle_steps, True, dev)
        sync(dev)
        t_settle = time.perf_counter() - t0
        ids, draws = eng.env_track_ids()
        snap = (eng.get_state(), eng.obs.clone(), [eng._track_files_by_id[int(i)] for i in ids], draws, venv._seeds)
        resets0 = int(draws.sum())
        rv = vec_rate(venv)
        resets = int(eng.env_track_ids()[1].sum()) - resets0
        venv.close()
        e2 = BatchedCarEnv(E, c, snap[2], device=dev)
        load(e2, snap, tracks)
        re = eng_rate(e2)
        e2.close()
        e3 = BatchedCarEnv(E, c, snap[2], device=dev)
        load(e3, snap)
        r_off = eng_rate(e3)
        e3.close()
        out[f"random_track_{c}car"] = {
            "config": f"track_file=None (learn/ppo.py:65-78), {E} envs x {c} cars, steady state after {settle_steps} "
                      f"noisy-driver steps ({t_settle:.1f} s)",
            "vec_env": rv, "engine_per_step": re, "ratio": re / rv, "engine_per_step_tracks_fixed": r_off,
            "track_switches_in_vec_window": resets}
    out["note"] = (f"car-steps/s of the drop-in VecCarEnv.step (device tensors, SB3 Monitor bookkeeping and action checks "
                   f"on the device, lazy infos) vs the engine's per-step path (policy_actions + launch_step, auto-reset, "
                   f"terminal obs) on the same state; ratio = engine / vec_env; {K} steps after {W} warm-up each")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of this node; without a torchrun environment N > 1 launches N ranks itself "
                         "(default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--envs", type=int, default=8192)
    ap.add_argument("--cars", type=int, default=10)
    ap.add_argument("--track", default="daytona")
    ap.add_argument("--policy", default="noisy", choices=list(POLICY_ID),
                    help="noisy (default): device noisy rule driver; driver: device rule driver; uniform: U[-1,1]^2 "
                         "resident in HBM; sac: fused SAC actor (random-init weights) on the previous observation")
    ap.add_argument("--settle", type=int, default=None,
                    help="closed-loop steps run before the warm-up to reach the steady state (default 10800 for the "
                         "closed-loop policies, 0 for uniform)")
    ap.add_argument("--no-stagger", action="store_true", help="all envs start together (no staggered resets)")
    ap.add_argument("--save-state", default=None, help="write the settled state (engine arena + obs) to this file")
    ap.add_argument("--load-state", default=None, help="start from a state written by --save-state (no settle)")
    ap.add_argument("--rollout", type=int, default=50,
                    help="steps per nascar_rollout call for the device action sources (default 50: the sharded rollout, "
                         "bit-identical to the per-step path, which is timed beside it); 0: per-step path only "
                         "(nascar_step_driven per step)")
    ap.add_argument("--rollout-pipe", type=int, default=0,
                    help="pipelined rollout with this many sensor workgroups (0: off; BatchedCarEnv.set_rollout_pipe)")
    ap.add_argument("--rollout-streams", type=int, default=None,
                    help="shards (internal streams) of the --rollout path; 0: the fused rollout kernel (default: engine's 4)")
    ap.add_argument("--mixed", action="store_true", help="env e on track e mod 8 of the sorted bundled tracks "
                    "(BASELINE cfg5: mixed batch, divergent geometry); --track is ignored")
    ap.add_argument("--gather", action="store_true", help="gather every step's obs/reward/flags of all ranks to "
                    "rank 0 (RCCL, side stream; BASELINE cfg4 single-learner layout)")
    ap.add_argument("--car-contact", action="store_true", help="BUILD-ONLY EXTENSION: car-car contact inside each env "
                    "(cfg3's 'car-car collision on'; no reference counterpart, reported as its own row)")
    ap.add_argument("--no-secondary", action="store_true", help="skip the uniform-from-reset secondary measurement")
    ap.add_argument("--no-drop-in", action="store_true", help="skip the drop-in API (VecCarEnv) secondary measurement")
    ap.add_argument("--beam-cell", type=float, default=None, help="the sensors' beam-list cell size in m (default 1; "
                    "identical results at any size)")
    ap.add_argument("--cpu-threads", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--plumbing", action="store_true", help="CPU tests: main() unchanged on a CPU stand-in engine "
                    "(PlumbingEngine: sleeps per step), gloo between the ranks; not a measurement")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ:
        if args.gpus is not None and args.gpus > 1:      # one rank per GPU, started before anything touches a GPU
            sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
        world = 1
    else:
        world = int(os.environ["WORLD_SIZE"])
        if args.gpus is not None and args.gpus != world:
            print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} ranks were launched", file=sys.stderr)
            sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))

    import torch
    import torch.distributed as dist
    from nascargymnasium_amd.track import track_path

    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.plumbing:      # CPU tests: the same main() on the CPU stand-in engine, gloo between the ranks
        dev = torch.device("cpu")
    else:
        torch.cuda.set_device(local)   # before the process group, so RCCL's barrier binds this rank's GPU
        dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("gloo" if args.plumbing else "nccl")
    E, C, K, W = args.envs, args.cars, args.steps, args.warmup
    closed = args.policy != "uniform"
    S = args.settle if args.settle is not None else (EPISODE_STEPS if closed else 0)
    if args.load_state:
        S = 0
    tpath = track_path(args.track)
    if args.mixed:
        from nascargymnasium_amd.track import available_tracks
        names = available_tracks()
        env_files = [names[e % len(names)] for e in range(E)]
    else:
        env_files = [tpath] * E
    tcache = track_cache_prebuild(env_files, rank, world, args.beam_cell)

    def make_env():
        if args.plumbing:
            return PlumbingEngine(E, C, rank, dev)
        from nascargymnasium_amd.batched import BatchedCarEnv
        return BatchedCarEnv(E, C, env_files if args.mixed else tpath, device=dev, beam_cell=args.beam_cell)

    env = make_env()
    if args.rollout_streams is not None:
        env.set_rollout_streams(args.rollout_streams)
    if args.rollout_pipe:
        env.set_rollout_pipe(args.rollout_pipe)
    if args.car_contact:
        env.set_car_contact(True)
    gather = None
    if args.gather:
        from nascargymnasium_amd.gather import ObsGather
        gather = ObsGather(E, C, dev, steps=max(1, args.rollout))
    if args.policy == "sac":
        from nascargymnasium_amd.policy import random_actor
        env.set_actor(random_actor(rank))
    env.reset()
    acts = None
    if args.policy == "uniform":
        gen = torch.Generator(device=dev)
        gen.manual_seed(1234 + rank)
        acts = torch.rand((W + K, E, C, 2), generator=gen, device=dev) * 2 - 1     # resident before timing
    step = Stepper(env, args.policy, rank, acts, None, args.rollout)
    t_settle = time.perf_counter()
    if args.load_state:
        blob = torch.load(args.load_state, map_location=dev, weights_only=True)
        env.set_state(blob["state"])
        env.obs.copy_(blob["obs"])
        base = int(blob["step"])
    else:   # per-step settle whatever the timed path: each staggered reset lands on its exact step
        settle(env, Stepper(env, args.policy, rank, acts, None, 0), S, closed and not args.no_stagger, dev)
        base = S
    sync(dev)
    t_settle = time.perf_counter() - t_settle
    if args.save_state:
        torch.save({"state": env.get_state().cpu(), "obs": env.obs.cpu(), "step": base}, args.save_state)
    step.gather = gather
    step.run(base, W)
    elapsed = timed(step, base + W, K, world)
    KR = min(K, 50)
    kern_ms, tally, KT = stats_pass(env, step, base + W + K, KR)   # KT: the steps the tallies cover
    ktimes = kernel_pass(env, Stepper(env, args.policy, rank, acts, None, 0), base + W + K + 2 * KR, KR)
    per_step = None
    next_step = base + W + K + 3 * KR        # the driver's next step index (its counter-hash key)
    if step.R:   # the per-step path on the same envs, timed the same way (labelled secondary)
        ps = Stepper(env, args.policy, rank, acts, None, 0)
        first = next_step
        ps.run(first, W)
        per_step = timed(ps, first + W, K, world)
        next_step = first + W + K
    rank_elapsed = gather_all(elapsed, dev)
    elapsed, kern_ms = reduce_max([elapsed, kern_ms], dev)
    fused = env.fused_logic
    if fused:   # model_logic_kernel between events 0 and 1 (events 1 and 2 are recorded back to back)
        ktimes = {"model_logic_kernel": ktimes["model_kernel"], "ray_sensor_kernel": ktimes["ray_sensor_kernel"]}
    kt_names = tuple(ktimes)
    ktimes = dict(zip(kt_names, reduce_max([ktimes[k] for k in kt_names], dev)))
    dom = "model_logic_kernel" if fused else "model_kernel"
    dom_bytes = FUSED_ALGO_BYTES_PER_CAR if fused else MODEL_ALGO_BYTES_PER_CAR
    if per_step is not None:
        per_step = reduce_max([per_step], dev)[0]
    tally = reduce_sum(tally, dev)
    value = throughput(world, E, C, K, elapsed)
    # dominant kernel (model_kernel, whole grid): ITS algorithmic bytes per car (the state it reads and writes + the
    # action) x the cars one launch processes, over its mean launch duration (HIP events around it on its stream,
    # per-step path).  The whole step's bytes over the timed window's step time are `roofline.step`.
    achieved = E * C * dom_bytes / (ktimes[dom] * 1e-3) / 1e9
    step_achieved = E * C * ALGO_BYTES_PER_CAR_STEP / (elapsed / K) / 1e9      # the timed window itself
    traffic, tnote = None, "no PMC file for this workload"
    tfile = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tfile):
        tj = json.load(open(tfile))
        same = (tj.get("envs") == E and tj.get("cars") == C and tj.get("track") == os.path.basename(tpath)
                and tj.get("policy", "uniform") == args.policy and not args.mixed)
        if not same:
            tnote = f"profiles/pmc_traffic.json is for another workload ({tj.get('tag')})"
        elif tj.get("source_sha") != source_sha():
            tnote = f"stale: profiles/pmc_traffic.json ({tj.get('tag')}) was measured on other kernel sources"
        elif tj.get(f"{dom}_bytes") is None:
            tnote = f"profiles/pmc_traffic.json ({tj.get('tag')}) has no {dom} dispatches"
        else:
            traffic = tj.get(f"{dom}_bytes")
            tnote = f"{dom} HBM bytes per whole-grid launch from the rocprofv3 FETCH_SIZE/WRITE_SIZE passes of this " \
                    f"build and workload ({tj.get('tag')}, profiles/pmc_traffic.json; not re-measured in this run); whole " \
                    f"step {tj.get('bytes_per_step', 0) / 1e6:.1f} MB"
    ncs = world * E * C * KT
    wstats = {"source": POLICY_TEXT[args.policy], "settle_steps": S if not args.load_state else f"state file {args.load_state}",
              "staggered_env_ages": closed and not args.no_stagger, "window_car_steps": ncs,
              "contact_frac": tally[0] / ncs, "lap_completed_frac": tally[1] / ncs, "disabled_frac": tally[2] / ncs,
              "just_disabled_frac": tally[3] / ncs, "env_reset_frac": tally[4] / (world * E * KT),
              "mean_speed_ms": tally[6] / ncs * 111.1, "settle_s": t_settle}
    track_name = "mixed 8-track" if args.mixed else os.path.basename(tpath)[:-6]
    settle_txt = (f", steady state after {S} settle steps" + (" (env ages staggered over the 180 s episode)"
                  if closed and not args.no_stagger else "")) if S else (", from a saved steady state" if args.load_state
                                                                        else ", from reset")
    nshard = env.rollout_streams if step.R else 0
    step_kernels = ("model_logic_kernel + ray_sensor_kernel" if fused
                    else "model_kernel + logic_kernel + ray_sensor_kernel")
    if not step.R:
        launch_txt = "per-step kernels (nascar_step_driven)"
        kernel_txt = f"{step_kernels} (one env step)"
    elif nshard == 0:
        launch_txt = f"fused rollout kernel, {step.R} steps per launch"
        kernel_txt = f"rollout_kernel ({step.R} fused env steps per launch; per-step time)"
    else:
        launch_txt = (f"sharded rollout: {step.R} steps per nascar_rollout call, envs in {nshard} shards on {nshard} "
                      f"streams (bit-identical to the per-step path)")
        kernel_txt = (f"{step_kernels} over {nshard} env shards on {nshard} streams "
                      f"(per-step time of a {step.R}-step rollout, HIP events on the caller's stream)")
    out = {
        "metric": "env-steps/sec (cars x envs), daytona 10-car",
        "value": value, "unit": "car-steps/s", "n_gpus": world, "steps": K, "warmup": W,
        "ms_per_step": elapsed / K * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f32+f64", "data": "synthetic",
        "config": {"workload": f"{track_name} {C}-car: {E} envs x {C} cars per GPU, {POLICY_TEXT[args.policy]}"
                               f"{settle_txt}, auto-reset",
                   "envs_per_gpu": E, "cars_per_env": C, "policy": args.policy,
                   "launch": launch_txt,
                   "car_contact": "on (build-only extension, no reference counterpart)" if args.car_contact else "off (reference)",
                   "track": "mixed (env e: track e mod 8)" if args.mixed else os.path.basename(tpath),
                   "parallelism": f"dp{world} (env shards" + ((", RCCL gather to rank 0 of every step's obs/reward/flags, one trajectory record per rollout call)" if step.R
                                   else ", RCCL gather of obs/reward/flags to rank 0 per step)") if gather else ", no collective)")},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": tnote,
                     "kernel": f"{dom} (dominant kernel; whole-grid launch on the per-step path, HIP events around "
                               "each launch on its stream)",
                     "kernel_ms": ktimes[dom], "units_per_launch": E * C,
                     "algo_bytes_per_unit": dom_bytes,
                     "algo_bytes_note": ("model_logic_kernel's share of SURVEY 8(d)'s 1221 B per car-step: every state "
                                         "word read and written (2 x 528 B), the 8 B action, obs[0:22] (88 B), reward and "
                                         "flags (5 B) -- all but the sensor kernel's 64 B of obs[22:38]" if fused else
                                         "model_kernel's share of SURVEY Appendix B: body + contacts + listener + car + "
                                         "tyre state read and written (848 B) + 8 B action")
                                        + "; the whole step's 1221 B per car-step are used in roofline.step",
                     "kernel_times_ms": ktimes,
                     "step": {"achieved": step_achieved, "frac": step_achieved / HBM_PEAK_GBS, "ms": elapsed / K * 1e3,
                              "algo_bytes_per_car_step": ALGO_BYTES_PER_CAR_STEP,
                              "note": "the whole step's algorithmic bytes (1221 B per car-step) over the timed window's "
                                      "time per step (" + launch_txt + ")"},
                     "timed_path_event_ms": kern_ms,
                     "timed_path_event_note": kernel_txt},
        "workload_stats": wstats,
        "engine_errors": int(tally[5]),
        "ranks": {"world_size": dist.get_world_size() if world > 1 else 1,
                  "backend": dist.get_backend() if world > 1 else None,
                  "elapsed_s": rank_elapsed, "envs_per_block": env.envs_per_block,
                  "note": "one process per GPU; each rank times its own K steps between barriers, value uses the MAX"},
    }
    if per_step is not None:
        out["per_step"] = {"value": throughput(world, E, C, K, per_step), "ms_per_step": per_step / K * 1e3,
                           "note": "secondary: the same envs and driver stepped by one whole-batch launch per step "
                                   "(nascar_step_driven), every step waiting for the batch's slowest car"}
    steady = None   # the steady state the CPU baseline and the drop-in pass continue from (rank 0 of a 1-GPU run)
    cpu_leg = rank == 0 and world == 1 and not args.no_cpu_baseline and not args.plumbing
    drop_in = (rank == 0 and world == 1 and not args.no_drop_in and not args.plumbing and args.policy == "noisy"
               and not args.mixed and not args.gather and not args.car_contact)
    if (cpu_leg or drop_in) and args.policy == "noisy" and not args.mixed:
        sync(dev)
        steady = (env.get_state().cpu().numpy(), E, env.obs.cpu().numpy().reshape(E, C, 38).copy(), next_step, rank)
    if drop_in:
        out["drop_in"] = drop_in_pass(E, C, tpath, rank, dev, steady)
    if not args.no_secondary and args.policy != "uniform" and not args.gather:
        # secondary, labelled: round 1's workload (uniform U[-1,1]^2 from reset) on a fresh engine
        del step
        env.close()
        env2 = make_env()
        env2.reset()
        gen = torch.Generator(device=dev)
        gen.manual_seed(1234 + rank)
        acts2 = torch.rand((W + K, E, C, 2), generator=gen, device=dev) * 2 - 1
        s2 = Stepper(env2, "uniform", rank, acts2, None)
        s2.run(0, W)
        el2 = reduce_max([timed(s2, W, K, world)], dev)[0]
        out["uniform_from_reset"] = {"value": throughput(world, E, C, K, el2), "ms_per_step": el2 / K * 1e3,
                                     "note": "secondary: uniform actions from reset (cars stay on the start "
                                             "straight; no contacts, laps or resets) -- an upper bound, not the headline"}
        env = env2
    if tcache is not None:   # (after every timed window: the per-rank cache statistics of the engine starts)
        out["track_cache"] = {"dir": tcache[0], "built": gather_all(tcache[1], dev), "loaded": gather_all(tcache[2], dev),
                              "prebuild_s": gather_all(tcache[3], dev),
                              "note": "per rank: tracks built into / loaded from the node's on-disk track cache before "
                                      "the engine started (each track built once per node)"}
    if args.plumbing:   # every rank must have issued the same collectives in the same order
        seq = list(COLLECTIVES)
        h = int(hashlib.sha256("|".join(seq).encode()).hexdigest()[:12], 16)
        hs = gather_all(h, dev)
        out["metric"] = "plumbing (no GPU, not a measurement)"
        out["collectives"] = {"rank0": seq, "all_ranks_equal": len(set(hs)) == 1, "ranks": len(hs)}
    if cpu_leg:
        out["cpu_baseline"] = cpu_baseline(tpath, C, args.cpu_budget, args.cpu_threads,
                                           steady if args.policy == "noisy" and not args.mixed else None)
    if rank == 0:
        print(json.dumps(out), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

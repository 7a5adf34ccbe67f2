"""Optional observation / reward / done gather to one learner rank (BASELINE cfg4).

Each rank steps its own env shard (BatchedCarEnv); a single learner on rank 0 may want every rank's
step outputs.  ObsGather packs a rank's outputs of `steps` consecutive env steps (1: one step; K: the
trajectory of a K-step sharded rollout, BatchedCarEnv.rollout(trajectory=True, obs_trajectory=True))
into one flat float32 record

    [K*E*C*38 obs | K*E*C reward | K*E*C car flags | K*E env flags]     (flags as exact small floats)

and gathers the records of all ranks to rank `dst` with torch.distributed (RCCL over xGMI on the GPU
box; gloo on CPU in the tests).

Ordering.  On the CPU (gloo) push() is synchronous.  On a GPU push() packs the record into one of two
staging buffers on the current (env) stream and runs the gather on a side stream, so it overlaps the
next env steps.  Both sides are double
buffered: staging buffer and receive buffer i are reused by push n+2 only after push n's gather has
finished (event waits on the streams, no host sync), so the views that received() returns stay valid
until two more pushes.  received() makes the current stream wait for the gather it returns, so
anything enqueued on that stream afterwards -- or a host copy such as .cpu() -- sees the whole record.

The reference has no counterpart (one process per env, SB3 SubprocVecEnv pipes, learn/ppo.py:77-78);
rank dst's `received` views are laid out [world, (K,) E, C, ...] like a VecEnv over world*E envs.
"""
from typing import Optional

import torch
import torch.distributed as dist

OBS_DIM = 38


class ObsGather:
    def __init__(self, num_envs: int, num_cars: int, device: torch.device, dst: int = 0, steps: int = 1):
        """steps: the most env steps one record holds (records of fewer steps are allowed; all ranks push the same
        number of steps per record)."""
        self.E, self.C, self.K = int(num_envs), int(num_cars), int(steps)
        if self.K < 1:
            raise ValueError("steps must be >= 1")
        self.N = self.E * self.C
        self.device = torch.device(device)
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.dst = dst
        self.rec = self._layout(self.K)[-1]
        self.cuda = self.device.type == "cuda"
        nbuf = 2
        self.stage = [torch.zeros(self.rec, dtype=torch.float32, device=self.device) for _ in range(nbuf)]
        self.recv = ([torch.zeros(self.world, self.rec, dtype=torch.float32, device=self.device) for _ in range(nbuf)]
                     if self.rank == dst else None)
        self.side = torch.cuda.Stream(device=self.device) if self.cuda else None
        self.done_ev = [None] * nbuf
        self.steps_of = [0] * nbuf
        self.k = 0

    def _layout(self, k):
        """offsets of a k-step record: obs, reward, car flags, env flags, end"""
        n = self.N
        o_rew = k * n * OBS_DIM
        return 0, o_rew, o_rew + k * n, o_rew + 2 * k * n, o_rew + 2 * k * n + k * self.E

    def _pack(self, buf, k, obs, reward, car_flags, env_flags):
        n, e = self.N, self.E
        for name, t, size in (("obs", obs, k * n * OBS_DIM), ("reward", reward, k * n),
                              ("car_flags", car_flags, k * n), ("env_flags", env_flags, k * e)):
            if t.numel() != size:
                raise ValueError(f"{name}: {t.numel()} elements, expected {size} ({k} step(s) of {e} envs x {self.C} cars)")
        _, o_rew, o_cf, o_ef, end = self._layout(k)
        buf[:o_rew].copy_(obs.reshape(-1))
        buf[o_rew:o_cf].copy_(reward.reshape(-1))
        buf[o_cf:o_ef].copy_(car_flags.reshape(-1))
        buf[o_ef:end].copy_(env_flags.reshape(-1))

    def _gather(self, buf, recv, size):
        if not dist.is_initialized():
            recv[0, :size].copy_(buf[:size])
            return
        parts = [row[:size] for row in recv.unbind(0)] if self.rank == self.dst else None
        dist.gather(buf[:size], gather_list=parts, dst=self.dst)

    def push(self, obs, reward, car_flags, env_flags):
        """Stage one record and start its gather (asynchronous on a GPU): this step's outputs (obs [E, C, 38], reward
        / car_flags [E, C], env_flags [E]) or a k-step trajectory, k <= steps (obs [k, E, C, 38], reward / car_flags
        [k, E, C], env_flags [k, E]).  With a rollout's obs trajectory of k + 1 records pass obs[1:] (the
        observation after each step)."""
        k = reward.numel() // self.N if self.N else 0
        if k < 1 or k > self.K:
            raise ValueError(f"a record holds 1 .. {self.K} steps, got {k}")
        i = self.k % len(self.stage)
        self.k += 1
        self.steps_of[i] = k
        buf = self.stage[i]
        recv = self.recv[i] if self.recv is not None else None
        size = self._layout(k)[-1]
        if not self.cuda:
            self._pack(buf, k, obs, reward, car_flags, env_flags)
            self._gather(buf, recv, size)
            return
        main = torch.cuda.current_stream(self.device)
        if self.done_ev[i] is not None:
            main.wait_event(self.done_ev[i])       # staging / receive buffer i: push n-2's gather has finished
        self._pack(buf, k, obs, reward, car_flags, env_flags)
        ready = torch.cuda.Event()
        ready.record(main)
        self.side.wait_event(ready)               # also orders the gather after reads of recv[i] enqueued before
        with torch.cuda.stream(self.side):
            self._gather(buf, recv, size)
            buf.record_stream(self.side)
            ev = torch.cuda.Event()
            ev.record(self.side)
        self.done_ev[i] = ev

    def wait(self):
        """Make the current stream wait until every started gather has landed on rank dst."""
        if self.cuda:
            torch.cuda.current_stream(self.device).wait_stream(self.side)

    def received(self) -> Optional[dict]:
        """rank dst: the last pushed record as views [world, E, C, 38] / [world, E, C] / [world, E] (a one-step
        record of an ObsGather with steps == 1) or [world, k, E, C, 38] / [world, k, E, C] / [world, k, E]
        (k-step records), ordered on the current stream after its gather (valid until two more pushes); None on
        other ranks or before the first push."""
        if self.recv is None or self.k == 0:
            return None
        i = (self.k - 1) % len(self.recv)
        if self.cuda:
            torch.cuda.current_stream(self.device).wait_event(self.done_ev[i])
        k = self.steps_of[i]
        _, o_rew, o_cf, o_ef, end = self._layout(k)
        r = self.recv[i]
        w, lead = self.world, ((k,) if self.K > 1 else ())
        return {
            "obs": r[:, :o_rew].reshape(w, *lead, self.E, self.C, OBS_DIM),
            "reward": r[:, o_rew:o_cf].reshape(w, *lead, self.E, self.C),
            "car_flags": r[:, o_cf:o_ef].reshape(w, *lead, self.E, self.C).to(torch.uint8),
            "env_flags": r[:, o_ef:end].reshape(w, *lead, self.E).to(torch.uint8),
        }

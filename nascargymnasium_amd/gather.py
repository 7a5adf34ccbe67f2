"""Optional observation / reward / done gather to one learner rank (BASELINE cfg4).

Each rank steps its own env shard (BatchedCarEnv); a single learner on rank 0 may want every rank's
step outputs.  ObsGather packs one step's outputs of a rank into a flat float32 record

    [E*C*38 obs | E*C reward | E*C car flags | E env flags]     (flags as exact small floats)

and gathers the records of all ranks to rank 0 with torch.distributed (RCCL over xGMI on the GPU
box; gloo on CPU in the tests).  On a GPU the record is copied into one of two staging buffers on the
env's stream and the gather runs on a side stream, so it overlaps the next env step; the staging
buffer of step k is reused at step k+2 only after its gather has finished (event wait).

The reference has no counterpart (one process per env, SB3 SubprocVecEnv pipes, learn/ppo.py:77-78);
rank 0's `received` view is laid out [world, E, C, ...] like a VecEnv over world*E envs.
"""
from typing import Optional

import torch
import torch.distributed as dist

OBS_DIM = 38


class ObsGather:
    def __init__(self, num_envs: int, num_cars: int, device: torch.device, dst: int = 0):
        self.E, self.C = int(num_envs), int(num_cars)
        self.N = self.E * self.C
        self.device = torch.device(device)
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.dst = dst
        self.rec = self.N * (OBS_DIM + 2) + self.E
        self.cuda = self.device.type == "cuda"
        nbuf = 2 if self.cuda else 1
        self.stage = [torch.zeros(self.rec, dtype=torch.float32, device=self.device) for _ in range(nbuf)]
        self.recv = (torch.zeros(self.world, self.rec, dtype=torch.float32, device=self.device)
                     if self.rank == dst else None)
        self.side = torch.cuda.Stream(device=self.device) if self.cuda else None
        self.done_ev = [None] * nbuf
        self.k = 0

    def _pack(self, buf, obs, reward, car_flags, env_flags):
        n, e = self.N, self.E
        buf[:n * OBS_DIM].copy_(obs.reshape(-1))
        buf[n * OBS_DIM:n * (OBS_DIM + 1)].copy_(reward.reshape(-1))
        buf[n * (OBS_DIM + 1):n * (OBS_DIM + 2)].copy_(car_flags.reshape(-1))
        buf[n * (OBS_DIM + 2):n * (OBS_DIM + 2) + e].copy_(env_flags.reshape(-1))

    def _gather(self, buf):
        if not dist.is_initialized():
            self.recv[0].copy_(buf)
            return
        parts = list(self.recv.unbind(0)) if self.rank == self.dst else None
        dist.gather(buf, gather_list=parts, dst=self.dst)

    def push(self, obs, reward, car_flags, env_flags):
        """Stage this step's outputs and start the gather (asynchronous on a GPU)."""
        i = self.k % len(self.stage)
        self.k += 1
        buf = self.stage[i]
        if not self.cuda:
            self._pack(buf, obs, reward, car_flags, env_flags)
            self._gather(buf)
            return
        main = torch.cuda.current_stream(self.device)
        if self.done_ev[i] is not None:
            main.wait_event(self.done_ev[i])       # staging buffer i's previous gather has finished
        self._pack(buf, obs, reward, car_flags, env_flags)
        ready = torch.cuda.Event()
        ready.record(main)
        self.side.wait_event(ready)
        with torch.cuda.stream(self.side):
            self._gather(buf)
            buf.record_stream(self.side)
            ev = torch.cuda.Event()
            ev.record(self.side)
        self.done_ev[i] = ev

    def wait(self):
        """Block the current stream until every started gather has landed on rank dst."""
        if self.cuda:
            torch.cuda.current_stream(self.device).wait_stream(self.side)

    def received(self) -> Optional[dict]:
        """rank dst: the last gathered step as views [world, E, C, 38] / [world, E, C] / [world, E]."""
        if self.recv is None:
            return None
        n, e, w = self.N, self.E, self.world
        r = self.recv
        return {
            "obs": r[:, :n * OBS_DIM].reshape(w, self.E, self.C, OBS_DIM),
            "reward": r[:, n * OBS_DIM:n * (OBS_DIM + 1)].reshape(w, self.E, self.C),
            "car_flags": r[:, n * (OBS_DIM + 1):n * (OBS_DIM + 2)].reshape(w, self.E, self.C).to(torch.uint8),
            "env_flags": r[:, n * (OBS_DIM + 2):n * (OBS_DIM + 2) + e].reshape(w, self.E).to(torch.uint8),
        }

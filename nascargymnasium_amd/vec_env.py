"""SB3-style vectorised env over the batched engine.

The reference trains with ``SubprocVecEnv([make_env]*8)`` / ``DummyVecEnv`` over
``Monitor(CarEnv(...))`` (learn/ppo.py:65-78).  ``VecCarEnv`` replaces the whole stack
with one ``BatchedCarEnv``: E envs step in one launch, auto-reset happens in the same
launch, and the final observation of a finished episode is returned in
``info["terminal_observation"]`` exactly as SB3's VecEnv convention, with
``info["TimeLimit.truncated"]`` and Monitor's ``info["episode"] = {"r", "l", "t"}``.

``return_tensors=False`` (default) returns numpy arrays like an SB3 VecEnv;
``return_tensors=True`` keeps obs / rewards / dones on the device (GPU-resident
rollouts) and builds info dicts only for the envs that finished.
"""
import time
from typing import List, Optional, Sequence, Union

import numpy as np

from . import _lib
from .car_env import BaseEnv


class VecCarEnv:
    def __init__(self, num_envs: int, track_file: Union[str, Sequence[str]] = "daytona", num_cars: int = 1,
                 discrete_action_space: bool = False, reset_on_lap: bool = False, device="cuda",
                 return_tensors: bool = False):
        import torch
        from .batched import BatchedCarEnv
        self._torch = torch
        self.num_envs = int(num_envs)
        self.num_cars = int(num_cars)
        spaces = BaseEnv(discrete_action_space=discrete_action_space, num_cars=num_cars)
        self.action_space, self.observation_space = spaces.action_space, spaces.observation_space
        self.discrete_action_space = discrete_action_space
        self.return_tensors = return_tensors
        self.engine = BatchedCarEnv(self.num_envs, self.num_cars, track_file, reset_on_lap=reset_on_lap, device=device)
        self.device = self.engine.device
        self._actions = None
        self._t0 = time.time()
        self._ep_ret = torch.zeros(self.num_envs, self.num_cars, dtype=torch.float64, device=self.device)
        self._ep_len = torch.zeros(self.num_envs, dtype=torch.int64, device=self.device)

    # ------------------------------------------------------------------ SB3 VecEnv API
    def reset(self):
        obs = self.engine.reset()
        self._ep_ret.zero_()
        self._ep_len.zero_()
        return self._out(obs.clone())

    def step_async(self, actions):
        torch = self._torch
        if isinstance(actions, torch.Tensor):
            a = actions.to(self.device)
        else:
            a = torch.as_tensor(np.asarray(actions), device=self.device)
        if self.discrete_action_space:
            a = a.to(torch.int32).reshape(self.num_envs, self.num_cars)
            if bool(((a < 0) | (a > 4)).any()):
                raise AssertionError("Invalid action: discrete actions must be in {0..4}")
        else:
            a = a.to(torch.float32).reshape(self.num_envs, self.num_cars, 2)
            if bool(((a < -1) | (a > 1) | torch.isnan(a)).any()):
                raise AssertionError("Invalid action: continuous actions must be in [-1, 1]")
        self._actions = a.contiguous()

    def step_wait(self):
        if self._actions is None:
            raise RuntimeError("step_async() must be called before step_wait()")
        eng = self.engine
        obs, rew, term, trunc = eng.step(self._actions, auto_reset=True, terminal_obs=True)
        self._actions = None
        done = term | trunc
        self._ep_ret += rew.to(self._torch.float64)
        self._ep_len += 1
        done_idx = self._torch.nonzero(done).flatten().tolist()
        infos: List[dict] = [{} for _ in range(self.num_envs)]
        if done_idx:
            term_obs = eng.terminal_obs[done_idx].cpu().numpy()
            rets = self._ep_ret[done_idx].cpu().numpy()
            lens = self._ep_len[done_idx].cpu().numpy()
            tr = trunc[done_idx].cpu().numpy()
            te = term[done_idx].cpu().numpy()
            reasons = eng.termination_reason()[done_idx].cpu().numpy()
            now = round(time.time() - self._t0, 6)
            for k, e in enumerate(done_idx):
                r = rets[k] if self.num_cars > 1 else rets[k][0]
                infos[e] = {
                    "terminal_observation": term_obs[k] if self.num_cars > 1 else term_obs[k][0],
                    "TimeLimit.truncated": bool(tr[k] and not te[k]),
                    "termination_reason": _lib.REASONS.get(int(reasons[k])),
                    "episode": {"r": np.round(r, 6) if self.num_cars > 1 else round(float(r), 6), "l": int(lens[k]),
                                "t": now},
                }
            self._ep_ret[done_idx] = 0.0
            self._ep_len[done_idx] = 0
        if self.return_tensors:
            r = rew if self.num_cars > 1 else rew[:, 0]
            return self._out(obs.clone()), r.clone(), done.clone(), infos
        r = rew.cpu().numpy()
        return self._out(obs), (r if self.num_cars > 1 else r[:, 0]), done.cpu().numpy(), infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def _out(self, obs):
        if self.num_cars == 1:
            obs = obs[:, 0]
        return obs if self.return_tensors else obs.cpu().numpy()

    def seed(self, seed: Optional[int] = None):
        return [seed] * self.num_envs

    def get_attr(self, name, indices=None):
        n = self.num_envs if indices is None else len(indices)
        return [getattr(self, name)] * n

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False] * (self.num_envs if indices is None else len(indices))

    def render(self, mode=None):
        return None

    def close(self):
        if self.engine is not None:
            self.engine.close()
            self.engine = None

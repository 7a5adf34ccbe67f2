"""SB3-style vectorised env over the batched engine.

The reference trains with ``SubprocVecEnv([make_env]*8)`` / ``DummyVecEnv`` over
``Monitor(CarEnv(...))`` (learn/ppo.py:65-78).  ``VecCarEnv`` replaces the whole stack
with one ``BatchedCarEnv``: E envs step in one launch, auto-reset happens in the same
launch, and the final observation of a finished episode is returned in
``info["terminal_observation"]`` exactly as SB3's VecEnv convention, with
``info["TimeLimit.truncated"]`` and Monitor's ``info["episode"] = {"r", "l", "t"}``.

``track_file=None`` is the reference's random-track mode (``CarEnv(track_file=None)``,
src/car_env.py:243-303, 331-398, as learn/ppo.py:67-72 trains): every env draws a new
track at each reset -- any bundled track but the one it just drove -- from its own
generator, seeded ``seed + env index`` (``seed()``), as SB3 seeds sub-envs.  Finished
envs are then reset after the step (their workgroups regroup by track between launches)
instead of inside it, since one workgroup never mixes tracks.

``return_tensors=False`` (default) returns numpy arrays like an SB3 VecEnv;
``return_tensors=True`` keeps obs / rewards / dones on the device and makes no host
synchronisation per step in single-track mode: actions are validated on the device
(an invalid action raises AssertionError, as the reference's ``assert
self.action_space.contains(action)``, src/car_env.py:694, at the next point that reads
the host: ``infos``, ``reset``, ``check_actions()``, or at the latest ``check_every``
steps later -- one small host read per ``check_every`` steps), and ``infos`` is a list
built from device copies the first time it is read.  The env state after an invalid
action is undefined (the reference never steps one).
"""
import random
import time
from collections import deque
from typing import List, Optional, Sequence, Union

import numpy as np

from . import _lib
from .car_env import BaseEnv
from .track import available_tracks, track_path


class _LazyInfos(list):
    """SB3's per-env info list, materialised from the step's device tensors on first use (any list operation fills
    it first, so it reads exactly like the eager list)."""

    def __init__(self, build):
        super().__init__()
        self._build = build

    def _fill(self):
        if self._build is not None:
            b, self._build = self._build, None
            super().extend(b())

    def __reduce__(self):
        self._fill()
        return (list, (list(self),))


def _filled(name):
    base = getattr(list, name)

    def method(self, *args, **kwargs):
        self._fill()
        for a in args:          # list's C methods read another list's storage directly: fill a lazy operand too
            if isinstance(a, _LazyInfos):
                a._fill()
        return base(self, *args, **kwargs)
    method.__name__ = name
    return method


for _name in ("__getitem__", "__iter__", "__len__", "__repr__", "__str__", "__eq__", "__ne__", "__lt__", "__le__",
              "__gt__", "__ge__", "__contains__", "__reversed__", "__add__", "__mul__", "__rmul__", "__iadd__",
              "__imul__", "__setitem__", "__delitem__", "copy", "index", "count", "append", "extend", "insert", "pop",
              "remove", "reverse", "sort", "clear"):
    setattr(_LazyInfos, _name, _filled(_name))
_LazyInfos.__hash__ = None


class VecCarEnv:
    def __init__(self, num_envs: int, track_file: Optional[Union[str, Sequence[str]]] = "daytona", num_cars: int = 1,
                 discrete_action_space: bool = False, reset_on_lap: bool = False, device="cuda",
                 return_tensors: bool = False, seed: Optional[int] = None, check_every: int = 64):
        import torch
        from .batched import BatchedCarEnv
        self._torch = torch
        self.num_envs = int(num_envs)
        self.num_cars = int(num_cars)
        spaces = BaseEnv(discrete_action_space=discrete_action_space, num_cars=num_cars)
        self.action_space, self.observation_space = spaces.action_space, spaces.observation_space
        self.discrete_action_space = discrete_action_space
        self.return_tensors = return_tensors
        self.random_tracks = track_file is None
        self._tracks = available_tracks()
        self.seed(seed)
        if self.random_tracks:
            # CarEnv.__init__ in random mode picks a track (src/car_env.py:158-163); reset() draws again
            self.env_tracks = [self._rngs[e].choice(self._tracks) for e in range(self.num_envs)]
            files = self.env_tracks
        else:
            files = track_file
            self.env_tracks = ([track_path(track_file)] * self.num_envs if isinstance(track_file, str)
                               else [track_path(f) for f in track_file])
        self.engine = BatchedCarEnv(self.num_envs, self.num_cars, files, reset_on_lap=reset_on_lap, device=device)
        self.device = self.engine.device
        self._actions = None
        self._t0 = time.time()
        self._ep_ret = torch.zeros(self.num_envs, self.num_cars, dtype=torch.float64, device=self.device)
        self._ep_len = torch.zeros(self.num_envs, dtype=torch.int64, device=self.device)
        self._bad = torch.zeros((), dtype=torch.bool, device=self.device)    # invalid action seen (device flag)
        self.check_every = max(1, int(check_every))   # return_tensors: read the flag at least this often
        self._unchecked = 0
        self._attrs = [dict() for _ in range(self.num_envs)]
        # per env, the tracks of its last 64 episodes (random-track mode)
        self.episode_tracks = [deque(maxlen=64) for _ in range(self.num_envs)]

    # ------------------------------------------------------------------ random-track mode (src/car_env.py:243-303)
    def _draw_track(self, e: int) -> str:
        """CarEnv._select_random_track: any bundled track but the current one, from env e's generator."""
        cands = self._tracks
        if len(cands) > 1 and self.env_tracks[e] in cands:
            cands = [t for t in cands if t != self.env_tracks[e]]
        return self._rngs[e].choice(cands)

    def _redraw(self, envs):
        for e in envs:
            self.env_tracks[e] = self._draw_track(e)
        self.engine.set_env_tracks(self.env_tracks)     # applied by the masked reset that follows

    # ------------------------------------------------------------------ SB3 VecEnv API
    def reset(self):
        self.check_actions()
        if self.random_tracks:
            self._redraw(range(self.num_envs))
        obs = self.engine.reset()
        if self.random_tracks:
            for e in range(self.num_envs):
                self.episode_tracks[e].append(self.env_tracks[e])
        self._ep_ret.zero_()
        self._ep_len.zero_()
        return self._out(obs.clone())

    def step_async(self, actions):
        torch = self._torch
        a = actions.to(self.device) if isinstance(actions, torch.Tensor) else \
            torch.as_tensor(np.asarray(actions), device=self.device)
        if self.discrete_action_space:
            a = a.reshape(self.num_envs, self.num_cars)
            bad = (a < 0) | (a > 4) | (a != a.trunc()) if a.is_floating_point() else (a < 0) | (a > 4)
            a = a.to(torch.int32)
        else:
            a = a.to(torch.float32).reshape(self.num_envs, self.num_cars, 2)
            bad = (a < -1) | (a > 1) | torch.isnan(a)
        self._bad |= bad.any()             # device-side check, read at the next host synchronisation
        self._actions = a.contiguous()
        self._unchecked += 1
        if not self.return_tensors or self._unchecked >= self.check_every:
            self.check_actions()

    def check_actions(self):
        """Raise AssertionError (the reference's `assert self.action_space.contains(action)`, src/car_env.py:694)
        if any action handed to step_async since the last check was outside the action space."""
        self._unchecked = 0
        if bool(self._bad):
            self._bad.zero_()
            raise AssertionError("Invalid action: continuous actions must be in [-1, 1], discrete in {0..4}")

    def step_wait(self):
        if self._actions is None:
            raise RuntimeError("step_async() must be called before step_wait()")
        torch = self._torch
        eng = self.engine
        auto = not self.random_tracks
        obs, rew, term, trunc = eng.step(self._actions, auto_reset=auto, terminal_obs=auto)
        self._actions = None
        done = term | trunc
        self._ep_ret += rew.to(torch.float64)
        self._ep_len += 1
        now = round(time.time() - self._t0, 6)
        if self.random_tracks:
            # host sync: the finished envs draw their next tracks, then a masked reset moves them there
            done_np = done.cpu().numpy()
            idx = np.nonzero(done_np)[0].tolist()
            snap = self._snapshot(idx, eng.obs, term, trunc)
            if idx:
                self._redraw(idx)
                eng.reset(done.to(torch.uint8))
                for e in idx:
                    self.episode_tracks[e].append(self.env_tracks[e])
            infos = self._infos(snap, now)
        elif self.return_tensors:
            # no host sync: device copies of what the finished envs' infos need, materialised on first read
            snap = (done.clone(), eng.terminal_obs.clone(), self._ep_ret.clone(), self._ep_len.clone(), term.clone(),
                    trunc.clone(), eng.termination_reason().clone())
            infos = _LazyInfos(lambda: self._infos(self._snapshot_dev(*snap), now))
        else:
            idx = torch.nonzero(done).flatten().tolist()
            infos = self._infos(self._snapshot(idx, eng.terminal_obs, term, trunc), now)
        self._ep_ret.masked_fill_(done[:, None], 0.0)     # masked fills: no host sync
        self._ep_len.masked_fill_(done, 0)
        if self.return_tensors:
            r = rew if self.num_cars > 1 else rew[:, 0]
            return self._out(obs.clone()), r.clone(), done.clone(), infos
        r = rew.cpu().numpy()
        return self._out(obs), (r if self.num_cars > 1 else r[:, 0]), done.cpu().numpy(), infos

    def _snapshot(self, idx, term_obs, term, trunc):
        if not idx:
            return idx, None, None, None, None, None, None
        return (idx, term_obs[idx].cpu().numpy(), self._ep_ret[idx].cpu().numpy(), self._ep_len[idx].cpu().numpy(),
                term[idx].cpu().numpy(), trunc[idx].cpu().numpy(), self.engine.termination_reason()[idx].cpu().numpy())

    def _snapshot_dev(self, done, term_obs, ret, length, term, trunc, reason):
        self.check_actions()
        idx = self._torch.nonzero(done).flatten().tolist()
        if not idx:
            return idx, None, None, None, None, None, None
        return (idx, term_obs[idx].cpu().numpy(), ret[idx].cpu().numpy(), length[idx].cpu().numpy(),
                term[idx].cpu().numpy(), trunc[idx].cpu().numpy(), reason[idx].cpu().numpy())

    def _infos(self, snap, now):
        idx, tobs, rets, lens, te, tr, reasons = snap
        infos: List[dict] = [{} for _ in range(self.num_envs)]
        for k, e in enumerate(idx):
            r = rets[k] if self.num_cars > 1 else rets[k][0]
            infos[e] = {
                "terminal_observation": tobs[k] if self.num_cars > 1 else tobs[k][0],
                "TimeLimit.truncated": bool(tr[k] and not te[k]),
                "termination_reason": _lib.REASONS.get(int(reasons[k])),
                "episode": {"r": np.round(r, 6) if self.num_cars > 1 else round(float(r), 6), "l": int(lens[k]),
                            "t": now},
            }
        return infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def _out(self, obs):
        if self.num_cars == 1:
            obs = obs[:, 0]
        return obs if self.return_tensors else obs.cpu().numpy()

    # ------------------------------------------------------------------ the rest of SB3's VecEnv surface
    def seed(self, seed: Optional[int] = None) -> list:
        """SB3 VecEnv.seed: sub-env i is seeded seed + i (the generators of the random-track draws)."""
        if seed is None:
            seed = random.randint(0, 2 ** 31 - 1)
        self._rngs = [random.Random(seed + e) for e in range(self.num_envs)]
        return [seed + e for e in range(self.num_envs)]

    def _indices(self, indices):
        if indices is None:
            return list(range(self.num_envs))
        return [indices] if isinstance(indices, int) else list(indices)

    def get_attr(self, name, indices=None):
        out = []
        for e in self._indices(indices):
            if name in self._attrs[e]:
                out.append(self._attrs[e][name])
            elif name == "track_file":
                out.append(self.env_tracks[e])
            else:
                out.append(getattr(self, name))
        return out

    def set_attr(self, name, value, indices=None):
        for e in self._indices(indices):
            self._attrs[e][name] = value

    def env_method(self, method_name, *args, indices=None, **kwargs):
        """Per-env methods of the reference CarEnv that make sense on a batched engine."""
        fn = getattr(self, "_env_" + method_name, None)
        if fn is None:
            raise AttributeError(f"VecCarEnv sub-envs have no method {method_name!r}")
        return [fn(e, *args, **kwargs) for e in self._indices(indices)]

    def _env_seed(self, e, seed_value=None):
        self._rngs[e] = random.Random(seed_value)
        return [seed_value]

    def _env_render(self, e, *a, **k):
        return None

    def _env_check_quit_requested(self, e):
        return False

    def get_images(self):
        return [None] * self.num_envs       # no rendering on the MI355X path

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False] * len(self._indices(indices))

    def render(self, mode=None):
        return None

    def close(self):
        if self.engine is not None:
            self.engine.close()
            self.engine = None

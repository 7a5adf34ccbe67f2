"""SB3-style vectorised env over the batched engine.

The reference trains with ``SubprocVecEnv([make_env]*8)`` / ``DummyVecEnv`` over
``Monitor(CarEnv(...))`` (learn/ppo.py:65-78).  ``VecCarEnv`` replaces the whole stack
with one ``BatchedCarEnv``: E envs step in one launch, auto-reset happens in the same
launch, and the final observation of a finished episode is returned in
``info["terminal_observation"]`` exactly as SB3's VecEnv convention, with
``info["TimeLimit.truncated"]`` and Monitor's ``info["episode"] = {"r", "l", "t"}``.

``track_file=None`` is the reference's random-track mode (``CarEnv(track_file=None)``,
src/car_env.py:243-303, 331-398, as learn/ppo.py:67-72 trains): every env draws a new
track at each reset -- any bundled track but the one it just drove -- keyed by its own
seed, ``seed + env index`` (``seed()``, as SB3 seeds sub-envs).  The draws, the fresh
worlds on the new track and the regrouping of the workgroups by track all happen on the
device, in the auto-reset of the step launch and two small kernels after it
(``BatchedCarEnv.set_random_tracks``): a step makes no host round trip in either mode.

``return_tensors=False`` (default) returns numpy arrays like an SB3 VecEnv;
``return_tensors=True`` keeps obs / rewards / dones on the device and makes no host
synchronisation per step: each step writes fresh output tensors (no copies), SB3
Monitor's episode bookkeeping runs in one device launch, actions are validated on the device
(an invalid action raises AssertionError, as the reference's ``assert
self.action_space.contains(action)``, src/car_env.py:694, at the next point that reads
the host: ``infos``, ``reset``, ``check_actions()``, or at the latest ``check_every``
steps later -- one small host read per ``check_every`` steps), and ``infos`` is a list
built from device copies the first time it is read.  The env state after an invalid
action is undefined (the reference never steps one).
"""
import ctypes
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
        if self.random_tracks:
            files = [self._tracks[0]] * self.num_envs      # replaced by each env's first draw in seed() below
            self._env_tracks = None
        else:
            files = track_file
            self._env_tracks = ([track_path(track_file)] * self.num_envs if isinstance(track_file, str)
                                else [track_path(f) for f in track_file])
        self.engine = BatchedCarEnv(self.num_envs, self.num_cars, files, reset_on_lap=reset_on_lap, device=device)
        self.device = self.engine.device
        self._L, self._h = self.engine.L, self.engine.h
        if self.random_tracks:
            self._ids = np.array([self.engine._add_track(f) for f in self._tracks], np.int32)
        self._actions = None
        self._discrete_actions = 0
        self._t0 = time.time()
        self._ep_ret = torch.zeros(self.num_envs, self.num_cars, dtype=torch.float64, device=self.device)
        self._ep_len = torch.zeros(self.num_envs, dtype=torch.int64, device=self.device)
        self._bad = torch.zeros((), dtype=torch.int32, device=self.device)   # invalid action seen (device flag)
        self.check_every = max(1, int(check_every))   # return_tensors: read the flag at least this often
        self._unchecked = 0
        self._attrs = [dict() for _ in range(self.num_envs)]
        self.seed(seed)

    # ------------------------------------------------------------------ random-track mode (src/car_env.py:243-303)
    @property
    def env_tracks(self) -> List[str]:
        """the .track file each env is on (random-track mode: read from the device)"""
        return self.engine.env_track_files() if self.random_tracks else list(self._env_tracks)

    @property
    def episode_tracks(self) -> List[deque]:
        """random-track mode: per env, the tracks of its last (up to 64) episodes since it was seeded, the current one
        last -- replayed on the host from its seed and the device's draw count (draw k: _lib.track_draw)."""
        out = [deque(maxlen=64) for _ in range(self.num_envs)]
        if not self.random_tracks:
            return out
        ids, draws = self.engine.env_track_ids()
        cur = self._seq_t0.copy()
        for k in range(int(self._seq_k0.min()), int(draws.max()) if draws.size else 0):
            live = (self._seq_k0 <= k) & (k < draws)
            if not live.any():
                continue
            nxt = _lib.track_draw(self._seeds, k, cur, self._ids)
            cur = np.where(live, nxt, cur)
            for e in np.nonzero(live)[0]:
                out[e].append(self.engine._track_files_by_id[int(cur[e])])
        assert np.array_equal(cur, ids), "random-track replay disagrees with the device"
        return out

    # ------------------------------------------------------------------ SB3 VecEnv API
    def reset(self):
        self.check_actions()
        obs = self.engine.reset()     # random-track mode: every env draws its next track on the device first
        self._ep_ret.zero_()
        self._ep_len.zero_()
        return self._out(obs.clone())

    def step_async(self, actions):
        torch = self._torch
        if isinstance(actions, torch.Tensor):
            a = actions if actions.device == self.device else actions.to(self.device)
        else:
            a = torch.as_tensor(np.asarray(actions), device=self.device)
        E, C = self.num_envs, self.num_cars
        if self.discrete_action_space:
            a = a.reshape(E, C)
            if a.dtype != torch.int32:     # checked before the conversion (a float 2.5 or an int64 2**32 + 1 is invalid)
                bad = (a < 0) | (a > 4) | (a != a.trunc()) if a.is_floating_point() else (a < 0) | (a > 4)
                self._bad |= bad.any().to(torch.int32)
                a = a.to(torch.int32)
        else:
            a = a.reshape(E, C, 2)
            if a.dtype != torch.float32:
                a = a.to(torch.float32)
        if not a.is_contiguous():
            a = a.contiguous()
        self._discrete_actions = int(self.discrete_action_space)
        self._on_device(self._launch_check, a)    # range / NaN check on the device (action_check_kernel)
        self._actions = a
        self._unchecked += 1
        if not self.return_tensors or self._unchecked >= self.check_every:
            self.check_actions()

    def check_actions(self):
        """Raise AssertionError (the reference's `assert self.action_space.contains(action)`, src/car_env.py:694)
        if any action handed to step_async since the last check was outside the action space."""
        self._unchecked = 0
        if int(self._bad.item()):
            self._bad.zero_()
            raise AssertionError("Invalid action: continuous actions must be in [-1, 1], discrete in {0..4}")

    def step_wait(self):
        if self._actions is None:
            raise RuntimeError("step_async() must be called before step_wait()")
        torch = self._torch
        E, C, dev = self.num_envs, self.num_cars, self.device
        # fresh output tensors written by the step launch itself (the caller may keep them)
        obs = torch.empty(E, C, 38, dtype=torch.float32, device=dev)
        tobs = torch.empty(E, C, 38, dtype=torch.float32, device=dev)
        rew = torch.empty(E, C, dtype=torch.float32, device=dev)
        ef = torch.empty(E, dtype=torch.uint8, device=dev)
        done = torch.empty(E, dtype=torch.bool, device=dev)
        sret = torch.empty(E, C, dtype=torch.float64, device=dev)
        slen = torch.empty(E, dtype=torch.int64, device=dev)
        self._on_device(self._launch_step, obs, tobs, rew, ef, done, sret, slen)
        self._actions = None
        now = round(time.time() - self._t0, 6)
        snap = (done, tobs, sret, slen, ef)
        if self.return_tensors:    # no host sync: the infos are built from these tensors the first time they are read
            infos = _LazyInfos(lambda: self._infos(self._snapshot(*snap, check=True), now))
            return self._out(obs), (rew if C > 1 else rew[:, 0]), done, infos
        infos = self._infos(self._snapshot(*snap), now)
        r = rew.cpu().numpy()
        return self._out(obs), (r if C > 1 else r[:, 0]), done.cpu().numpy(), infos

    def _on_device(self, fn, *args):
        """fn(stream, *args) with the env's device current (switched, and back, only when another one is)"""
        torch = self._torch
        if torch.cuda.current_device() == self.device.index:
            return fn(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream), *args)
        with torch.cuda.device(self.device):
            return fn(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream), *args)

    def _launch_check(self, st, a):
        _lib.check(self._L.nascar_check_actions(self._h, a.data_ptr(), self._discrete_actions, self._bad.data_ptr(), st))

    def _launch_step(self, st, obs, tobs, rew, ef, done, sret, slen):
        # CarEnv.step with SB3-style auto-reset in the launch (random-track mode: new tracks on the device too)
        _lib.check(self._L.nascar_step(self._h, self._actions.data_ptr(), self._discrete_actions, obs.data_ptr(),
                                       rew.data_ptr(), None, ef.data_ptr(), 1, tobs.data_ptr(), st))
        # Monitor / VecEnv bookkeeping: done, episode return and length (vec_post_kernel)
        _lib.check(self._L.nascar_vec_post(self._h, rew.data_ptr(), ef.data_ptr(), self._ep_ret.data_ptr(),
                                           self._ep_len.data_ptr(), done.data_ptr(), sret.data_ptr(), slen.data_ptr(), st))

    def _snapshot(self, done, tobs, ret, length, ef, check=False):
        if check:
            self.check_actions()
        idx = self._torch.nonzero(done).flatten().tolist()
        if not idx:
            return idx, None, None, None, None, None, None
        f = ef[idx].cpu().numpy()
        return (idx, tobs[idx].cpu().numpy(), ret[idx].cpu().numpy(), length[idx].cpu().numpy(),
                (f & 1) != 0, (f & 2) != 0, (f >> 4) & 7)

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
        """SB3 VecEnv.seed: sub-env i is seeded seed + i -- in random-track mode the key of its track draws (its next
        reset takes draw 0 of the new seed; at construction each env's first track is draw 0, as CarEnv.__init__
        picks one, src/car_env.py:158-163, and the first reset takes draw 1)."""
        if seed is None:
            seed = random.randint(0, 2 ** 31 - 1)
        seeds = [seed + e for e in range(self.num_envs)]
        if self.random_tracks:
            self._set_seeds(np.array(seeds, np.uint64), None)
        return seeds

    def _set_seeds(self, seeds, envs):
        """(re)key the random-track draws: all envs (envs None) or the listed ones restart their draw counters"""
        eng = self.engine
        if eng.random_track_ids is None:    # construction: each env's first track is draw 0 (applied at once)
            first = _lib.track_draw(seeds, 0, -1, self._ids)
            eng.set_env_tracks([eng._track_files_by_id[int(t)] for t in first])
            self._seeds, self._seq_k0, self._seq_t0 = seeds.copy(), np.ones(self.num_envs, np.int64), first.copy()
            eng.set_random_tracks(self._tracks, self._seeds, draws=1)
            return
        ids, draws = eng.env_track_ids()
        sel = np.arange(self.num_envs) if envs is None else np.asarray(envs, np.int64)
        self._seeds[sel] = seeds[sel] if envs is None else seeds
        draws = draws.astype(np.int64)
        draws[sel] = 0
        self._seq_k0[sel] = 0
        self._seq_t0[sel] = ids[sel]
        eng.set_random_tracks(self._tracks, self._seeds, draws=draws.astype(np.int32))

    def _indices(self, indices):
        if indices is None:
            return list(range(self.num_envs))
        return [indices] if isinstance(indices, int) else list(indices)

    def get_attr(self, name, indices=None):
        out = []
        tracks = self.env_tracks if name == "track_file" else None
        for e in self._indices(indices):
            if name in self._attrs[e]:
                out.append(self._attrs[e][name])
            elif name == "track_file":
                out.append(tracks[e])
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
        """CarEnv.seed on sub-env e: re-keys its random-track draws (random.Random(seed_value) in the reference's spirit)"""
        if seed_value is None:
            seed_value = random.randint(0, 2 ** 31 - 1)
        if self.random_tracks:
            self._set_seeds(np.array([seed_value], np.uint64), [e])
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

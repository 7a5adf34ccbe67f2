"""BatchedCarEnv: E independent reference CarEnvs x C cars stepped by one fused
HIP kernel per step (libnascar.so), state resident in HBM.

All buffers are torch tensors on the HIP device; ``step`` launches on torch's
current stream and returns device tensors (no host sync).  This is the engine
under both the Gymnasium ``CarEnv`` (E=1, nascargymnasium_amd/car_env.py) and
the SB3-style ``VecCarEnv`` (nascargymnasium_amd/vec_env.py).
"""
import ctypes
from typing import Optional, Sequence, Union

import numpy as np
import torch

from . import _lib
from .track import build_walls, load_track, track_path


def _ptr(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


class BatchedCarEnv:
    """E envs x C cars of the reference CarEnv on one GPU.

    track_file: one track (name or path) for all envs, or a sequence of E tracks
    (per-env track index; envs are grouped per track into workgroups).
    envs_per_block / beam_cell: scheduling and memory choices with identical results (set_envs_per_block;
    nascar_set_beam_cell: the distance sensors' beam-list cell size in m, default 1).
    """

    def __init__(self, num_envs: int, num_cars: int = 1, track_file: Union[str, Sequence[str]] = "daytona",
                 reset_on_lap: bool = False, device: Union[str, int, torch.device] = "cuda",
                 start_position=None, start_angle: float = 0.0, perf_history: bool = False,
                 envs_per_block: Optional[int] = None, beam_cell: Optional[float] = None):
        if not torch.cuda.is_available():
            raise RuntimeError("BatchedCarEnv needs a HIP device (torch.cuda.is_available() is False); "
                               "the product path has no CPU fallback")
        if num_cars < 1 or num_cars > 64:
            raise ValueError("num_cars must be in [1, 64]")
        self.E, self.C, self.N = int(num_envs), int(num_cars), int(num_envs) * int(num_cars)
        self.device = torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.L = _lib.lib()
        files = [track_file] * self.E if isinstance(track_file, str) else list(track_file)
        if len(files) != self.E:
            raise ValueError("need one track per env")
        uniq = sorted(set(track_path(f) for f in files))
        first = load_track(track_path(files[0]))
        sx, sy = start_position if start_position is not None else first.start_position
        cfg = _lib.NascarConfig(self.E, self.C, int(reset_on_lap), self.device.index, float(sx), float(sy),
                                float(start_angle))
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(self.L.nascar_create(ctypes.byref(cfg), ctypes.byref(h)))
        self.h = h
        if envs_per_block is not None:
            self.set_envs_per_block(envs_per_block)
        if beam_cell is not None:     # before the tracks are added: their beam lists are built at this cell size
            _lib.check(self.L.nascar_set_beam_cell(self.h, float(beam_cell)))
        self.tracks, self._track_id, self._track_files_by_id = [], {}, {}
        self.random_track_ids = None
        for p in uniq:
            self._add_track(p)
        self.set_env_tracks(files)
        dev = self.device
        self.obs = torch.zeros(self.E, self.C, _lib.OBS_DIM, dtype=torch.float32, device=dev)
        self.reward = torch.zeros(self.E, self.C, dtype=torch.float32, device=dev)
        self.car_flags = torch.zeros(self.E, self.C, dtype=torch.uint8, device=dev)
        self.env_flags = torch.zeros(self.E, dtype=torch.uint8, device=dev)
        self.terminal_obs = torch.zeros_like(self.obs)
        self._info = torch.zeros(self.E, self.C, _lib.N_INFO, dtype=torch.float64, device=dev)
        self._actions = torch.zeros(self.E, self.C, 2, dtype=torch.float32, device=dev)
        if perf_history:
            self.set_perf_history(True)

    def set_car_contact(self, enable: bool = True):
        """BUILD-ONLY EXTENSION (no reference counterpart): cars of an env collide with each other (staggered start
        grid, central impulses between overlapping closing car boxes).  Off by default; parity holds only when off."""
        _lib.check(self.L.nascar_set_car_contact(self.h, int(bool(enable))))

    def set_rollout_streams(self, streams: int = 4):
        """How `rollout` schedules its steps (identical results either way): streams >= 1 splits the envs into that
        many shards, each stepped on its own stream (shard 0 on the current one), so one shard's slow cars (Box2D
        TOI chains) overlap the other shards' work (default 4, or GPU_MAX_HW_QUEUES if fewer); 0 runs all steps in
        one fused launch."""
        _lib.check(self.L.nascar_set_rollout_streams(self.h, int(streams)))

    @property
    def rollout_streams(self) -> int:
        return int(self.L.nascar_get_rollout_streams(self.h))

    def set_rollout_pipe(self, sensor_workgroups: int = 0):
        """Pipelined `rollout` (identical results): each workgroup of envs goes on to its next step as soon as its own
        sensors are done, with the sensors in a second persistent kernel of `sensor_workgroups` workgroups fed from a
        device queue, so a slow car delays only its own envs (not the batch's step).  0 turns it off.  Used by
        `rollout` for policies 0 / 1 / 3 without random tracks, car contact or obs trajectories (else the setting of
        set_rollout_streams applies)."""
        _lib.check(self.L.nascar_set_rollout_pipe(self.h, int(sensor_workgroups)))
        self.rollout_pipe = int(sensor_workgroups)

    def rollout_pipe_status(self) -> int:
        """Waits for the current stream and reports whether a pipelined rollout since the last call gave up on a
        clock-bounded wait (1; its results are not valid) or not (0)."""
        import torch
        r = int(self.L.nascar_rollout_pipe_status(self.h, ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)))
        if r < 0:
            _lib.check(r)
        return r

    def set_envs_per_block(self, epb: int = 0):
        """Workgroup layout of the one-lane-per-car step kernels: `epb` whole envs per 128-lane workgroup, in
        [1, 128 // C]; 0 restores the automatic choice.  Results do not depend on it (tests pin every layout the
        bench runs against the oracle); it changes only which cars share a wave."""
        _lib.check(self.L.nascar_set_envs_per_block(self.h, int(epb)))

    @property
    def envs_per_block(self) -> int:
        return int(self.L.nascar_get_envs_per_block(self.h))

    def set_fused_logic(self, enable: bool = True):
        """One launch per step for the vehicle model + Box2D step and the env logic (each workgroup runs its envs'
        logic once its own cars' physics is done; the default) or two (False); identical results."""
        _lib.check(self.L.nascar_set_fused_logic(self.h, int(bool(enable))))

    @property
    def fused_logic(self) -> bool:
        return bool(self.L.nascar_get_fused_logic(self.h))

    def set_sensor_lanes(self, lanes: int = 0):
        """Lanes per car of the distance-sensor kernel: 4 or 16 (one ray per lane), 0 automatic (16).  Identical
        results; a scheduling choice."""
        _lib.check(self.L.nascar_set_sensor_lanes(self.h, int(lanes)))

    def set_sensor_block(self, threads: int = 0):
        """threads per workgroup of the 16-lane sensor kernel: 64 / 128 (walls read from global memory) or 256 / 512 /
        1024 (walls staged in LDS per workgroup); 0: automatic (128); identical results"""
        _lib.check(self.L.nascar_set_sensor_block(self.h, int(threads)))

    def set_perf_history(self, enable: bool = True):
        """Keep Car.velocity_history on the device so the info's `performance` dict is Car.validate_performance
        (src/car.py:1060-1098); a 640-sample float32 ring per car, one 4-byte store per car-step.  Enabled before the
        first reset (as CarEnv does) it covers every episode; enabled mid-episode, an env's window holds steps taken
        before the enable, so its info reports perf_count -1 ("history not kept") until its next reset or until
        600 steps have been recorded since the enable."""
        with torch.cuda.device(self.device):
            _lib.check(self.L.nascar_set_perf_history(self.h, int(bool(enable)), _stream()))

    def _add_track(self, path: str) -> int:
        """Load a .track file into the handle (TrackLoader + _create_track_walls tables); returns its id."""
        path = track_path(path)
        if path in self._track_id:
            return self._track_id[path]
        t = load_track(path)
        seg = np.ascontiguousarray(t.segment_table())
        walls = np.ascontiguousarray(build_walls(t)[:, :4])
        dp = ctypes.POINTER(ctypes.c_double)
        with torch.cuda.device(self.device):   # (the library also brackets its device work with the handle's device)
            tid = _lib.check(self.L.nascar_add_track(self.h, seg.ctypes.data_as(dp), seg.shape[0], float(t.total_length),
                                                     walls.ctypes.data_as(dp), walls.shape[0]))
        self.tracks.append(t)
        self._track_id[path] = tid
        self._track_files_by_id[tid] = path
        return tid

    def set_env_tracks(self, files: Sequence[str]):
        """Per-env track (name or path), applied by the next reset of each env (fresh worlds on the new track, as
        CarEnv.reset rebuilds CarPhysics, src/car_env.py:375-394); until then an env steps on its old track.  New
        tracks are loaded on demand.  The start pose is the handle's (every bundled track starts its GRID at (0, 0),
        heading 0)."""
        if isinstance(files, str):
            files = [files] * self.E
        if len(files) != self.E:
            raise ValueError("need one track per env")
        env_track = np.array([self._add_track(f) for f in files], np.int32)
        _lib.check(self.L.nascar_set_env_tracks(self.h, env_track.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
        self.env_track = env_track
        self.track_files = [track_path(f) for f in files]

    # ------------------------------------------------------------------ random-track mode (src/car_env.py:243-303)
    def set_random_tracks(self, files: Sequence[str], seeds, draws=None):
        """Random-track mode on the device (CarEnv(track_file=None), src/car_env.py:243-303, 331-398; learn/ppo.py:65-78
        trains every env this way): every reset of an env -- `reset(mask)` or the auto-reset inside a step -- first draws
        its next track from `files` (any but its current one, CarEnv._select_random_track) and a changed track gets fresh
        worlds; the block map is rebuilt on the device, so a step makes no host round trip.  Draw k of env e is
        `_lib.track_draw(seeds[e], k, current, ids)`; `draws` (default 0) are the per-env draw counters to continue from.
        Files not loaded yet are loaded here.  While the mode is on, `set_env_tracks` raises; `clear_random_tracks` ends
        it (the envs keep their current tracks)."""
        ids = np.array([self._add_track(f) for f in files], np.int32)
        seeds = np.ascontiguousarray(np.asarray(seeds, dtype=np.uint64).ravel())
        if seeds.size != self.E:
            raise ValueError(f"need one seed per env ({self.E}), got {seeds.size}")
        dr = None
        if draws is not None:
            dr = np.ascontiguousarray(np.broadcast_to(np.asarray(draws, np.int32), (self.E,)))
        i32p, u64p = ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_uint64)
        with torch.cuda.device(self.device):
            _lib.check(self.L.nascar_set_random_tracks(self.h, ids.ctypes.data_as(i32p), int(ids.size),
                                                       seeds.ctypes.data_as(u64p),
                                                       dr.ctypes.data_as(i32p) if dr is not None else None, _stream()))
        self.random_track_ids = ids
        self.random_track_files = [track_path(f) for f in files]

    def clear_random_tracks(self):
        """End random-track mode: the envs keep the tracks they are on, managed by `set_env_tracks` again."""
        with torch.cuda.device(self.device):
            _lib.check(self.L.nascar_set_random_tracks(self.h, None, 0, None, None, _stream()))
        self.random_track_ids = None
        ids, _ = self.env_track_ids()
        self.env_track = ids
        self.track_files = [self._track_files_by_id[i] for i in ids]

    def env_track_ids(self):
        """(track id per env, draws taken per env) as numpy int32 arrays -- the device's in random-track mode (one host
        synchronisation), else the host's assignment and zeros."""
        t = torch.empty(2, self.E, dtype=torch.int32, device=self.device)
        with torch.cuda.device(self.device):
            _lib.check(self.L.nascar_get_env_tracks(self.h, _ptr(t[0]), _ptr(t[1]), _stream()))
        a = t.cpu().numpy()
        return a[0].copy(), a[1].copy()

    def env_track_files(self):
        """the .track path each env is on now"""
        ids, _ = self.env_track_ids()
        return [self._track_files_by_id[i] for i in ids]

    def block_map(self):
        """(blk_track [nb], blk_env [nb, envs_per_block]) numpy int32: the workgroup layout of the next launch (test hook,
        nascar_debug_block_map; one host synchronisation)"""
        cap = self.E + 128
        bt = torch.empty(cap, dtype=torch.int32, device=self.device)
        be = torch.empty(cap * max(1, self.envs_per_block), dtype=torch.int32, device=self.device)
        with torch.cuda.device(self.device):
            nb = _lib.check(self.L.nascar_debug_block_map(self.h, _ptr(bt), _ptr(be), cap, _stream()))
        epb = self.envs_per_block
        return bt[:nb].cpu().numpy(), be[:nb * epb].cpu().numpy().reshape(nb, epb)

    # ------------------------------------------------------------------ core API
    def reset(self, env_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        """CarEnv.reset for all envs (or those with env_mask[e] != 0, uint8[E] on device)."""
        with torch.cuda.device(self.device):
            m = None if env_mask is None else env_mask.to(self.device, torch.uint8).contiguous()
            _lib.check(self.L.nascar_reset(self.h, _ptr(m), _ptr(self.obs), _stream()))
        return self.obs

    def step(self, actions: torch.Tensor, auto_reset: bool = False, terminal_obs: bool = False):
        """CarEnv.step for all envs.  actions: float32 [E, C, 2] (continuous) or int32 [E, C] (discrete)."""
        self.launch_step(actions, auto_reset, terminal_obs)
        terminated = (self.env_flags & _lib.EF_TERMINATED) != 0
        truncated = (self.env_flags & _lib.EF_TRUNCATED) != 0
        return self.obs, self.reward, terminated, truncated

    def launch_step(self, actions: torch.Tensor, auto_reset: bool = False, terminal_obs: bool = False):
        """Enqueue exactly one env step (model, logic and sensor kernels) on the current stream (no other device work when
        `actions` is already a contiguous float32/int32 tensor on this device)."""
        discrete = not actions.is_floating_point()
        a = actions.to(self.device, torch.int32 if discrete else torch.float32).contiguous()
        if a.numel() != self.N * (1 if discrete else 2):
            raise ValueError(f"actions must have {self.N * (1 if discrete else 2)} elements, got {tuple(a.shape)}")
        with torch.cuda.device(self.device):
            _lib.check(self.L.nascar_step(self.h, _ptr(a), int(discrete), _ptr(self.obs), _ptr(self.reward),
                                          _ptr(self.car_flags), _ptr(self.env_flags), int(auto_reset),
                                          _ptr(self.terminal_obs) if terminal_obs else None, _stream()))

    def step_driven(self, policy: int, seed: int = 0, step: int = 0, auto_reset: bool = True, terminal_obs: bool = False):
        """One env step whose actions come from device action source `policy` (0 uniform, 1 rule driver, 3 noisy rule
        driver) on the current obs, computed inside the step launch; equals policy_actions(policy, seed, step) +
        step(...)."""
        with torch.cuda.device(self.device):
            _lib.check(self.L.nascar_step_driven(self.h, int(policy), int(seed), int(step), _ptr(self.obs), _ptr(self.reward),
                                                 _ptr(self.car_flags), _ptr(self.env_flags), int(auto_reset),
                                                 _ptr(self.terminal_obs) if terminal_obs else None, _stream()))
        return self.obs, self.reward

    def rollout(self, policy: int, steps: int, seed: int = 0, step0: int = 0, auto_reset: bool = True,
                trajectory: bool = False, out=None, obs_trajectory: bool = False):
        """`steps` env steps in one call (sharded over streams, or one fused launch: set_rollout_streams), actions
        from device action source `policy` (0 uniform, 1 rule driver, 2 the SAC actor -- sharded only, 3 noisy rule
        driver) on the previous observation; equals `steps` x (policy_actions(policy, seed, step0 + k) +
        step(..., auto_reset)).  Returns (obs, reward, car_flags, env_flags): the last step's, or with
        trajectory=True the per-step records [steps, E, C] / [steps, E] (obs the last step's).  obs_trajectory=True
        (with trajectory=True, sharded rollout only) also records every step's observation: obs [steps + 1, E, C, 38],
        record 0 the observation before the rollout, record k + 1 the one after step k (a learner's rollout buffer,
        written by the kernels in place).  `out`: caller-owned buffers (reward, car_flags, env_flags), preceded by
        obs when obs_trajectory, each with at least the records this call writes."""
        steps = int(steps)
        if out is not None and not trajectory:
            raise ValueError("`out` buffers are written only with trajectory=True")
        if obs_trajectory and not trajectory:
            raise ValueError("obs_trajectory needs trajectory=True")
        if trajectory and out is not None:      # caller-owned per-step buffers (at least `steps` records)
            n_out = 4 if obs_trajectory else 3
            if len(out) != n_out:
                raise ValueError("out must be (" + ("obs, " if obs_trajectory else "") + "reward, car_flags, env_flags)")
            ot = out[0] if obs_trajectory else None
            rew, cf, ef = out[n_out - 3:]
            checks = [("reward", rew, torch.float32, (self.E, self.C), steps),
                      ("car_flags", cf, torch.uint8, (self.E, self.C), steps),
                      ("env_flags", ef, torch.uint8, (self.E,), steps)]
            if obs_trajectory:
                checks.append(("obs", ot, torch.float32, (self.E, self.C, _lib.OBS_DIM), steps + 1))
            for name, t, dt, inner, n in checks:
                self._check_record_buffer(name, t, dt, inner, n)
        elif trajectory:
            rew = torch.empty(steps, self.E, self.C, dtype=torch.float32, device=self.device)
            cf = torch.empty(steps, self.E, self.C, dtype=torch.uint8, device=self.device)
            ef = torch.empty(steps, self.E, dtype=torch.uint8, device=self.device)
            ot = (torch.empty(steps + 1, self.E, self.C, _lib.OBS_DIM, dtype=torch.float32, device=self.device)
                  if obs_trajectory else None)
        else:
            rew, cf, ef, ot = self.reward, self.car_flags, self.env_flags, None
        traj = (_lib.TRAJ_RECORDS if trajectory else 0) | (_lib.TRAJ_OBS if obs_trajectory else 0)
        with torch.cuda.device(self.device):
            if ot is not None:
                ot[0].copy_(self.obs)
            _lib.check(self.L.nascar_rollout(self.h, int(policy), int(seed), int(step0), steps,
                                             _ptr(ot if ot is not None else self.obs), _ptr(rew), _ptr(cf), _ptr(ef),
                                             int(auto_reset), traj, _stream()))
            if trajectory and steps > 0:
                self.reward.copy_(rew[steps - 1]); self.car_flags.copy_(cf[steps - 1]); self.env_flags.copy_(ef[steps - 1])
                if ot is not None:
                    self.obs.copy_(ot[steps])
        return (ot if ot is not None else self.obs), rew, cf, ef

    def _check_record_buffer(self, name, t, dtype, inner, steps):
        """the kernels write record k at data_ptr + k * prod(inner) elements: anything but a contiguous tensor of
        this dtype on this device with shape [>= steps, *inner] would be written out of bounds (steps: the records
        this call writes)"""
        if not isinstance(t, torch.Tensor):
            raise ValueError(f"out {name}: expected a torch.Tensor, got {type(t).__name__}")
        if t.device != self.device:
            raise ValueError(f"out {name}: on {t.device}, the env is on {self.device}")
        if t.dtype != dtype:
            raise ValueError(f"out {name}: dtype {t.dtype}, expected {dtype}")
        if tuple(t.shape[1:]) != inner or t.dim() != len(inner) + 1:
            raise ValueError(f"out {name}: shape {tuple(t.shape)}, expected [>= {steps}, {', '.join(map(str, inner))}]")
        if t.shape[0] < steps:
            raise ValueError(f"out {name}: holds {t.shape[0]} records, fewer than steps = {steps}")
        if not t.is_contiguous():
            raise ValueError(f"out {name}: must be contiguous")

    def set_step_events(self, events=None):
        """Profiling hook (nascar_set_step_events): 4 torch.cuda.Event(enable_timing=True) recorded by every following
        whole-grid step on its stream -- before model_kernel, after model_kernel, after logic_kernel, after the
        sensor launch -- so their elapsed times are the three kernels' durations; None switches it off."""
        if events is None:
            _lib.check(self.L.nascar_set_step_events(self.h, None, 0))
            self._step_events = None
            return
        if len(events) != 4:
            raise ValueError("need 4 events")
        with torch.cuda.device(self.device):
            for e in events:
                if not e.cuda_event:   # torch creates the HIP event at its first record
                    e.record()
            arr = (ctypes.c_void_p * 4)(*[ctypes.c_void_p(e.cuda_event) for e in events])
            _lib.check(self.L.nascar_set_step_events(self.h, arr, 4))
        self._step_events = list(events)    # kept alive while the engine may record them

    def info_tensor(self) -> torch.Tensor:
        """per-car info [E, C, N_INFO] float64 (fields: _lib.INFO_FIELDS)."""
        with torch.cuda.device(self.device):
            _lib.check(self.L.nascar_get_info(self.h, _ptr(self._info), _stream()))
        return self._info

    def termination_reason(self) -> torch.Tensor:
        return (self.env_flags >> 4) & 7

    def set_actor(self, weights, precision: str = "fp32"):
        """Load an SB3 SAC MlpPolicy actor: a dict from nascargymnasium_amd.policy.load_sb3_actor / random_actor.
        precision "fp32" (default): float32 throughout, the reference's model.predict precision (<= 1e-5 on the
        reference's sac_1235 checkpoint); "bf16": the MFMA kernel (bf16 operands, fp32 accumulation), ~8x faster but
        NOT faithful for trained policies (max |delta action| 0.40 on sac_1235)."""
        from .policy import actor_arrays
        if precision not in ("bf16", "fp32"):
            raise ValueError("precision must be 'bf16' or 'fp32'")
        arrs = actor_arrays(weights)
        fp = ctypes.POINTER(ctypes.c_float)
        _lib.check(self.L.nascar_set_actor(self.h, *[a.ctypes.data_as(fp) for a in arrs], 38, 256, 2))
        _lib.check(self.L.nascar_set_actor_precision(self.h, int(precision == "fp32")))
        self._actor_arrays = arrs

    def actor_forward(self, obs: torch.Tensor) -> torch.Tensor:
        """The loaded actor on a device batch of observations [..., 38] -> actions [..., 2]."""
        o = obs.to(self.device, torch.float32).contiguous()
        n = o.numel() // 38
        out = torch.empty(o.shape[:-1] + (2,), dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            _lib.check(self.L.nascar_actor_forward(self.h, _ptr(o), n, _ptr(out), _stream()))
        return out

    def policy_actions(self, policy: int, seed: int = 0, step: int = 0, obs: Optional[torch.Tensor] = None):
        """device-generated actions: 0 uniform U[-1,1]^2, 1 BaseController fallback driver, 2 the SAC actor."""
        o = self.obs if obs is None else obs
        with torch.cuda.device(self.device):
            _lib.check(self.L.nascar_policy_actions(self.h, int(policy), int(seed), int(step), _ptr(o),
                                                    _ptr(self._actions), _stream()))
        return self._actions

    # ------------------------------------------------------------------ checkpointing
    def state_bytes(self) -> int:
        return int(self.L.nascar_state_bytes(self.h))

    def get_state(self) -> torch.Tensor:
        buf = torch.empty(self.state_bytes(), dtype=torch.uint8, device=self.device)
        with torch.cuda.device(self.device):
            _lib.check(self.L.nascar_get_state(self.h, _ptr(buf), _stream()))
        return buf

    def set_state(self, buf: torch.Tensor):
        if buf.numel() != self.state_bytes():
            raise ValueError("state blob size mismatch")
        with torch.cuda.device(self.device):
            _lib.check(self.L.nascar_set_state(self.h, _ptr(buf.to(self.device).contiguous()), _stream()))

    def close(self):
        if getattr(self, "h", None):
            torch.cuda.synchronize(self.device)
            self.L.nascar_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

"""Gymnasium ``CarEnv`` / ``BaseEnv`` with the reference API, stepped by the HIP engine.

Drop-in for ``src.car_env.CarEnv`` (src/car_env.py:75-1470) and ``src.base_env.BaseEnv``
(src/base_env.py:29-257) on the hot path: same constructor arguments, action /
observation spaces, ``reset``/``step`` return shapes, error behaviour and the
attributes callers read (``disabled_cars``, ``cumulative_collision_impacts``,
``termination_reason``, ``simulation_time``, ``track_file``, ``action_space`` ...).
One ``CarEnv`` is one env of a ``BatchedCarEnv`` (E = 1) on the HIP device; the
Box2D/Python per-car loop of the reference runs as libnascar.so's fused kernels.

Not provided (out of scope): pygame rendering (``render_mode="human"``
raises), the observation visualiser, wall-clock FPS statistics.
"""
import random
import time
from typing import Dict, Optional, Tuple

import numpy as np

from . import _lib
from .spaces import Box, Discrete, Env, MultiDiscrete
from .track import available_tracks, load_track, track_path

# src/constants/control.py:26-27, sensors.py:20-64, car_specs.py:9-50, environment.py:10
CAR_ACTION_LOW = np.array([-1.0, -1.0], dtype=np.float32)
CAR_ACTION_HIGH = np.array([1.0, 1.0], dtype=np.float32)
OBS_DIM = 38
CAR_OBSERVATION_LOW = np.array([-1.0, -1.0, -1.0, -1.0, 0.0, -1.0, -1.0] + [0.0] * 12 + [0.0, -1.0, 0.0] + [0.0] * 16,
                               dtype=np.float32)
CAR_OBSERVATION_HIGH = np.ones(OBS_DIM, dtype=np.float32)
MAX_CARS = 10
CAR_MAX_SPEED_MS = 200.0 * 0.44704
CAR_TARGET_100KMH_MS = 100.0 * 0.277778
CAR_ACCELERATION_0_100_KMH = 3.0
DT = 1.0 / 60.0


class BaseEnv(Env):
    """src/base_env.py:29-257: spaces and the action conversions."""
    metadata = {"render_modes": ["human"], "render_fps": 60}

    def __init__(self, discrete_action_space: bool = False, num_cars: int = 1):
        super().__init__()
        self.discrete_action_space = discrete_action_space
        self.num_cars = num_cars
        if discrete_action_space:
            self.action_space = Discrete(5) if num_cars == 1 else MultiDiscrete([5] * num_cars)
        elif num_cars == 1:
            self.action_space = Box(low=CAR_ACTION_LOW, high=CAR_ACTION_HIGH, shape=(2,), dtype=np.float32)
        else:
            self.action_space = Box(low=np.tile(CAR_ACTION_LOW, (num_cars, 1)), high=np.tile(CAR_ACTION_HIGH, (num_cars, 1)),
                                    shape=(num_cars, 2), dtype=np.float32)
        if num_cars == 1:
            self.observation_space = Box(low=CAR_OBSERVATION_LOW, high=CAR_OBSERVATION_HIGH, shape=(OBS_DIM,),
                                         dtype=np.float32)
        else:
            self.observation_space = Box(low=np.tile(CAR_OBSERVATION_LOW, (num_cars, 1)),
                                         high=np.tile(CAR_OBSERVATION_HIGH, (num_cars, 1)),
                                         shape=(num_cars, OBS_DIM), dtype=np.float32)
        self.start_time = None
        self.elapsed_time = 0.0
        self.last_action = np.zeros(3, dtype=np.float32)

    @staticmethod
    def _convert_to_internal_action(action):
        """[throttle_brake, steering] -> [throttle, brake, steering] (src/base_env.py:201-225)."""
        tb, steer = action[0], action[1]
        return [tb, 0.0, steer] if tb >= 0 else [0.0, -tb, steer]

    @staticmethod
    def _discrete_to_continuous(action):
        """{0..4} -> [tb, steering] (src/base_env.py:227-252)."""
        table = {0: [0.0, 0.0], 1: [1.0, 0.0], 2: [-1.0, 0.0], 3: [0.0, -1.0], 4: [0.0, 1.0]}
        try:
            return table[int(action)]
        except (KeyError, TypeError, ValueError):
            raise ValueError(f"Invalid discrete action: {action}") from None


# src/constants/environment.py:19-26
MIN_REALISTIC_FPS, MAX_REALISTIC_FPS = 5.0, 300.0
PERFORMANCE_VALIDATION_MIN_SAMPLES = 10
PERFORMANCE_SPEED_TOLERANCE, PERFORMANCE_TIME_TOLERANCE = 0.95, 1.1

_SIM_T = [0.0]


def _sim_time(k: int) -> float:
    """the float64 time after k steps of 1/60 s, summed one step at a time as CarEnv/CarPhysics/
    validate_performance do (src/car_env.py:573, src/car.py:1085-1086)"""
    while len(_SIM_T) <= k:
        _SIM_T.append(_SIM_T[-1] + DT)
    return _SIM_T[k]


def validate_performance(count: int, max_speed: float, first_fast: int) -> dict:
    """Car.validate_performance (src/car.py:1060-1098) from the device's window summary: count = samples in
    velocity_history (-1: history not kept), max_speed = their maximum, first_fast = index of the first sample
    >= CAR_TARGET_100KMH_MS (-1: none)."""
    res = {"max_speed_ms": CAR_MAX_SPEED_MS, "target_100kmh_ms": CAR_TARGET_100KMH_MS,
           "target_acceleration_time": CAR_ACCELERATION_0_100_KMH, "current_max_speed": 0.0,
           "estimated_0_100_time": 0.0, "performance_valid": False}
    if count > PERFORMANCE_VALIDATION_MIN_SAMPLES:
        res["current_max_speed"] = max_speed
        if first_fast >= 0:
            res["estimated_0_100_time"] = _sim_time(first_fast + 1)
        speed_ok = max_speed >= CAR_MAX_SPEED_MS * PERFORMANCE_SPEED_TOLERANCE
        est = res["estimated_0_100_time"]
        accel_ok = est <= CAR_ACCELERATION_0_100_KMH * PERFORMANCE_TIME_TOLERANCE if est > 0 else False
        res["performance_valid"] = speed_ok and accel_ok
    return res


def physics_stats(k: int, bodies: int) -> dict:
    """CarPhysics.get_performance_stats (src/car_physics.py:573-592) after k steps since the reset: the world's
    simulation_time is the env time before its last step, average_fps is updated every 60 steps
    (src/car_physics.py:374-385) and clamped to [MIN_REALISTIC_FPS, MAX_REALISTIC_FPS]."""
    fps = 60.0
    if k >= 60:
        m = 60 * (k // 60)
        elapsed = _sim_time(m - 1) - (_sim_time(m - 61) if m > 60 else 0.0)
        fps = 60 / elapsed if elapsed > 0 else 60.0
    return {"physics_steps": k, "simulation_time": _sim_time(k - 1) if k > 0 else 0.0,
            "average_fps": max(MIN_REALISTIC_FPS, min(fps, MAX_REALISTIC_FPS)), "bodies_in_world": bodies}


def build_info(info_np, num_cars: int, followed: int, reason, bodies: int) -> dict:
    """CarEnv._get_multi_info (src/car_env.py:1160-1227) as a plain dict from one env's host copy of the device
    info rows ([C, N_INFO] float64, fields _lib.INFO_FIELDS)."""
    F = _lib.INFO_INDEX
    cars = []
    for i in range(num_cars):
        r = info_np[i]
        speed = float(r[F["speed"]])
        last = None if np.isnan(r[F["last_lap_time"]]) else float(r[F["last_lap_time"]])
        best = None if np.isnan(r[F["best_lap_time"]]) else float(r[F["best_lap_time"]])
        timing = bool(r[F["is_timing"]])
        cur = float(r[F["current_lap_time"]])
        cars.append({
            "car_index": i,
            "disabled": bool(r[F["disabled"]]),
            "car_position": (float(r[F["x"]]), float(r[F["y"]])),
            "car_speed_kmh": speed * 3.6,
            "car_speed_ms": speed,
            "on_track": bool(r[F["on_track"]]),
            "performance": validate_performance(int(r[F["perf_count"]]), float(r[F["perf_max_speed"]]),
                                                int(r[F["perf_first_fast"]])),
            "lap_timing": {   # LapTimer.get_timing_info (src/lap_timer.py:354-372)
                "current_lap_time": cur, "last_lap_time": last, "best_lap_time": best,
                "lap_count": int(r[F["lap_count"]]), "is_timing": timing,
                "has_crossed_startline": bool(r[F["has_crossed_startline"]]),
                "total_distance_traveled": float(r[F["total_distance_traveled"]]),
                "formatted_current": _format_time(cur if timing else None),
                "formatted_last": _format_time(last), "formatted_best": _format_time(best)},
            "cumulative_reward": float(r[F["cumulative_reward"]]),
            "cumulative_impact_force": float(r[F["cumulative_impact_force"]]),
        })
    sim = float(info_np[0, F["simulation_time"]])
    k = int(round(sim / DT))
    physics = [{**physics_stats(k, bodies), **c["performance"]} for c in cars]
    return {"simulation_time": sim, "num_cars": num_cars, "followed_car_index": followed,
            "termination_reason": reason, "cars": cars, "physics": physics}


def _format_time(t: Optional[float]) -> str:
    """LapTimer.format_time (src/lap_timer.py:328-352)."""
    if t is None or t < 0:
        return "--:--.---"
    total = int(t)
    ms = int(round((t - total) * 1000))
    return f"{total // 60:2d}:{total % 60:02d}.{ms:03d}"


class CarEnv(BaseEnv):
    """src/car_env.py CarEnv on the MI355X engine (one env, ``num_cars`` cars)."""

    def __init__(self, render_mode: Optional[str] = None, track_file: Optional[str] = None,
                 start_position: Optional[Tuple[float, float]] = None, start_angle: float = 0.0,
                 reset_on_lap: bool = False, discrete_action_space: bool = False, num_cars: int = 1,
                 car_names: Optional[list] = None, device=None):
        super().__init__(discrete_action_space=discrete_action_space, num_cars=num_cars)
        if num_cars < 1 or num_cars > MAX_CARS:
            raise ValueError(f"Number of cars must be between 1 and {MAX_CARS}")
        if render_mode is not None:
            raise NotImplementedError("rendering (pygame) is outside the MI355X hot path; use render_mode=None")
        self.render_mode = render_mode
        if car_names is None:
            self.car_names = [f"Car {i}" for i in range(num_cars)]
        else:
            if len(car_names) != num_cars:
                raise ValueError(f"Number of car names ({len(car_names)}) must match number of cars ({num_cars})")
            self.car_names = list(car_names)
        self.start_angle = start_angle
        self.reset_on_lap = reset_on_lap
        self.followed_car_index = 0
        self._is_random_track_mode = track_file is None
        self.track_file = track_file
        if track_file:
            self._original_track_file = track_file
            self.track = load_track(track_path(track_file))     # FileNotFoundError / ValueError as the loader
        else:
            self.track_file = self._select_random_track()
            self.track = load_track(track_path(self.track_file))
        self.start_position = start_position or (0.0, 0.0)
        if self.start_position == (0.0, 0.0) and self.track.segments:
            for seg in self.track.segments:
                if seg.segment_type in ("GRID", "STARTLINE"):
                    self.start_position = seg.start_position
                    break
        import torch
        from .batched import BatchedCarEnv
        self._torch = torch
        self._engine = BatchedCarEnv(1, num_cars, track_path(self.track_file), reset_on_lap=reset_on_lap,
                                     device=device if device is not None else "cuda",
                                     start_position=self.start_position, start_angle=start_angle, perf_history=True)
        self._ready = False
        self.cars = []
        self.disabled_cars = set()
        self.cumulative_collision_impacts = {i: 0.0 for i in range(num_cars)}
        self.termination_reason = None
        self.simulation_time = 0.0
        self._cumulative_rewards = [0.0] * num_cars
        self._info_cache = None

    # ------------------------------------------------------------------ track selection (src/car_env.py:243-303)
    def _select_random_track(self) -> str:
        tracks = available_tracks()
        prev = getattr(self, "track_file", None)
        if len(tracks) > 1 and prev in tracks:
            tracks = [t for t in tracks if t != prev]
        return random.choice(tracks)

    def switch_to_random(self):
        self.track_file = None
        if hasattr(self, "_original_track_file"):
            delattr(self, "_original_track_file")
        self._is_random_track_mode = True

    def seed(self, seed_value: Optional[int] = None) -> list:
        """src/car_env.py:1414-1436 (seeds Python's and numpy's global RNGs, used for track choice)."""
        if seed_value is None:
            seed_value = random.randint(0, 2 ** 32 - 1)
        random.seed(seed_value)
        np.random.seed(seed_value % 2 ** 32)
        return [seed_value]

    # ------------------------------------------------------------------ Gymnasium API
    def reset(self, seed: Optional[int] = None, options: Optional[Dict] = None):
        super().reset(seed=seed)
        self.seed(seed_value=seed)
        self.start_time = time.time()
        self.elapsed_time = 0.0
        self.last_action = np.zeros(3, dtype=np.float32)
        if self._is_random_track_mode:
            self.track_file = self._select_random_track()
            self.track = load_track(track_path(self.track_file))
            self._engine.set_env_tracks([track_path(self.track_file)])
        obs = self._engine.reset()[0].cpu().numpy()
        self._info_cache = self._engine.info_tensor()[0].cpu().numpy()
        self._ready = True
        self.cars = list(range(self.num_cars))
        self.disabled_cars = set()
        self.cumulative_collision_impacts = {i: 0.0 for i in range(self.num_cars)}
        self.termination_reason = None
        self.simulation_time = 0.0
        self._cumulative_rewards = [0.0] * self.num_cars
        info = self._make_info(self._info_cache)
        return (obs[0], info) if self.num_cars == 1 else (obs, info)

    def step(self, action):
        assert self.action_space.contains(action), f"Invalid action {action}"
        if not self._ready:
            raise RuntimeError("Environment not properly initialized. Call reset() first.")
        torch = self._torch
        C = self.num_cars
        if self.discrete_action_space:
            a = np.asarray(action, dtype=np.int64).reshape(C)
            internal = [self._convert_to_internal_action(self._discrete_to_continuous(x)) for x in a]
            dev_a = torch.from_numpy(a.astype(np.int32)).view(1, C)
        else:
            a = np.asarray(action, dtype=np.float32).reshape(C, 2)
            internal = [self._convert_to_internal_action(x) for x in a]
            dev_a = torch.from_numpy(np.ascontiguousarray(a)).view(1, C, 2)
        self.last_action = np.array(internal[0], dtype=np.float32)
        self.elapsed_time = time.time() - self.start_time
        eng = self._engine
        eng.step(dev_a.to(eng.device))
        # one device->host transfer of everything the caller sees this step: obs, reward (float32, exact in
        # float64), the env flag byte and the info rows, packed on the device
        info_t = eng.info_tensor()
        packed = torch.cat([eng.obs[0].reshape(-1).double(), eng.reward[0].double(), eng.env_flags[:1].double(),
                            info_t[0].reshape(-1)]).cpu().numpy()
        obs = packed[:C * 38].astype(np.float32).reshape(C, 38)
        rew = packed[C * 38:C * 39].astype(np.float32)
        ef = int(packed[C * 39])
        terminated, truncated = bool(ef & _lib.EF_TERMINATED), bool(ef & _lib.EF_TRUNCATED)
        reason = (ef >> 4) & 7
        info_np = packed[C * 39 + 1:].reshape(C, _lib.N_INFO)
        F = _lib.INFO_FIELDS
        self.simulation_time = float(info_np[0, F.index("simulation_time")])
        self.disabled_cars = {i for i in range(C) if info_np[i, F.index("disabled")] != 0}
        self.cumulative_collision_impacts = {i: float(info_np[i, F.index("cumulative_impact_force")]) for i in range(C)}
        self._cumulative_rewards = [float(np.float32(self._cumulative_rewards[i]) + rew[i]) for i in range(C)]
        self.termination_reason = _lib.REASONS.get(reason) if (terminated or truncated) else self.termination_reason
        self._info_cache = info_np
        info = self._make_info(info_np)
        if C == 1:
            return obs[0], rew[0], terminated, truncated, info
        return obs, rew, terminated, truncated, info

    # ------------------------------------------------------------------ race tables (src/car_env.py:1485-1637)
    def _info_rows(self):
        return self._info_cache if self._info_cache is not None else self._engine.info_tensor()[0].cpu().numpy()

    def _calculate_race_positions(self) -> list:
        """CarEnv._calculate_race_positions (src/car_env.py:1485-1542): (car_index, car_name, total_progress,
        virtual_laps, current_progress) of the non-disabled cars, leader first."""
        if not self._ready:
            return []
        F = {f: i for i, f in enumerate(_lib.INFO_FIELDS)}
        rows = self._info_rows()
        L = self.track.get_total_track_length()
        out = []
        for i in range(self.num_cars):
            if i in self.disabled_cars:
                continue
            r = rows[i]
            laps, prog = int(r[F["lap_count"]]), float(r[F["track_progress"]])
            virtual = laps
            if (bool(r[F["is_timing"]]) and bool(r[F["has_crossed_startline"]]) and prog < L * 0.15
                    and float(r[F["total_distance_traveled"]]) > L * 0.8):
                virtual = laps + 1
            out.append((i, self.car_names[i], virtual * L + prog, virtual, prog))
        out.sort(key=lambda x: (x[3], x[4]), reverse=True)
        return out

    def _get_best_lap_times_data(self) -> list:
        """CarEnv._get_best_lap_times_data (src/car_env.py:1613-1638): (car_index, car_name, best_lap_time)
        of the non-disabled cars with a best lap, fastest first."""
        if not self._ready:
            return []
        F = {f: i for i, f in enumerate(_lib.INFO_FIELDS)}
        rows = self._info_rows()
        out = [(i, self.car_names[i], float(rows[i][F["best_lap_time"]])) for i in range(self.num_cars)
               if i not in self.disabled_cars and not np.isnan(rows[i][F["best_lap_time"]])]
        out.sort(key=lambda x: x[2])
        return out

    # ------------------------------------------------------------------ info (src/car_env.py:1160-1227)
    def _make_info(self, info_np) -> dict:
        """the step's / reset's info dict, built eagerly from the host copy fetched with the step (picklable,
        as SubprocVecEnv workers need; later steps do not change it)"""
        return build_info(info_np, self.num_cars, self.followed_car_index, self.termination_reason, 1 + self._nwalls())

    def _nwalls(self) -> int:
        from .track import build_walls
        if getattr(self, "_nwalls_cache", None) is None or self._nwalls_cache[0] != self.track_file:
            self._nwalls_cache = (self.track_file, len(build_walls(self.track)))
        return self._nwalls_cache[1]

    # ------------------------------------------------------------------ misc API
    def render(self):
        return None

    def check_quit_requested(self) -> bool:
        return False

    def get_state(self):
        """Raw device state snapshot (checkpoint / state injection)."""
        return self._engine.get_state()

    def set_state(self, blob):
        self._engine.set_state(blob)

    def close(self):
        eng = getattr(self, "_engine", None)
        if eng is not None:
            eng.close()
            self._engine = None
        self._ready = False

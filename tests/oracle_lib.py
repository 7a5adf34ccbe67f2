"""ctypes binding of the CPU parity oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "build", "liboracle.so")

INFO_FIELDS = [
    "x", "y", "vx", "vy", "angle", "omega", "rpm", "lateral_force", "slip_deg", "banking",
    "load_fl", "load_fr", "load_rl", "load_rr", "temp_fl", "temp_fr", "temp_rl", "temp_rr",
    "wear_fl", "wear_fr", "wear_rl", "wear_rr", "lap_count", "last_lap", "best_lap", "is_timing",
    "current_lap_time", "lap_distance", "disabled", "cum_impact", "cum_reward", "stuck_duration",
    "backward", "progress", "sim_time", "impulse", "sleep_time", "awake", "n_contacts", "overflow",
    "on_track", "n_active_collisions", "info_cum_reward", "speed",
]
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, f32p, f64p = ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_double)
        L.or_create.restype = vp
        L.or_create.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.or_destroy.argtypes = [vp]
        L.or_num_walls.argtypes = [vp]
        L.or_num_segments.argtypes = [vp]
        L.or_total_length.argtypes = [vp]
        L.or_total_length.restype = ctypes.c_double
        L.or_walls.argtypes = [vp, f64p, f32p]
        L.or_segments.argtypes = [vp, f64p]
        L.or_reset.argtypes = [vp, ctypes.c_int]
        L.or_step.argtypes = [vp, f32p]
        L.or_outputs.argtypes = [vp, f32p, f32p, ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_int32)]
        L.or_car_info.argtypes = [vp, ctypes.c_int, f64p]
        L.or_sinf.restype = ctypes.c_float
        L.or_sinf.argtypes = [ctypes.c_float]
        L.or_cosf.restype = ctypes.c_float
        L.or_cosf.argtypes = [ctypes.c_float]
        L.or_raycast.restype = ctypes.c_float
        L.or_raycast.argtypes = [vp, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float]
        L.or_set_body.argtypes = [vp, ctypes.c_int] + [ctypes.c_float] * 6
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


class OracleEnv:
    """E envs x C cars of the restated reference CarEnv on the CPU."""

    def __init__(self, track_path, num_envs=1, num_cars=1, reset_on_lap=False, start_position=None, start_angle=0.0):
        self.L = lib()
        self.E, self.C = num_envs, num_cars
        self.h = self.L.or_create(track_path.encode(), num_envs, num_cars, int(reset_on_lap))
        if not self.h:
            raise FileNotFoundError(track_path)
        if start_position is not None or start_angle != 0.0:
            self.L.or_set_start.argtypes = [ctypes.c_void_p] + [ctypes.c_double] * 3
            sx, sy = start_position if start_position is not None else (np.nan, np.nan)
            if start_position is None:      # keep the track's default start point
                s = self.segments()
                row = next(r for r in s if r[0] in (0.0, 1.0))
                sx, sy = row[2], row[3]
            self.L.or_set_start(self.h, float(sx), float(sy), float(start_angle))

    def close(self):
        if self.h:
            self.L.or_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def walls(self):
        n = self.L.or_num_walls(self.h)
        d = np.zeros((n, 4), np.float64)
        f = np.zeros((n, 12), np.float32)
        self.L.or_walls(self.h, _p(d, ctypes.c_double), _p(f, ctypes.c_float))
        return d, f

    def segments(self):
        n = self.L.or_num_segments(self.h)
        s = np.zeros((n, 13), np.float64)
        self.L.or_segments(self.h, _p(s, ctypes.c_double))
        return s

    def total_length(self):
        return self.L.or_total_length(self.h)

    def reset(self, env=None):
        envs = range(self.E) if env is None else [env]
        for e in envs:
            self.L.or_reset(self.h, e)
        return self.outputs()

    def step(self, actions):
        a = np.ascontiguousarray(actions, dtype=np.float32).reshape(self.E * self.C, 2)
        self.L.or_step(self.h, _p(a, ctypes.c_float))
        return self.outputs()

    def outputs(self):
        obs = np.zeros((self.E, self.C, 38), np.float32)
        rew = np.zeros((self.E, self.C), np.float32)
        cf = np.zeros((self.E, self.C), np.uint8)
        ef = np.zeros((self.E, 3), np.int32)
        self.L.or_outputs(self.h, _p(obs, ctypes.c_float), _p(rew, ctypes.c_float),
                          _p(cf, ctypes.c_uint8), _p(ef, ctypes.c_int32))
        return obs, rew, cf, ef

    def car_info(self, idx):
        o = np.zeros(len(INFO_FIELDS), np.float64)
        self.L.or_car_info(self.h, idx, _p(o, ctypes.c_double))
        return dict(zip(INFO_FIELDS, o.tolist()))


class OracleGroups:
    """E envs of one batched run as several OracleEnv groups (one per track of a mixed batch, or shards of one
    track), stepped in parallel host threads (the C step releases the GIL inside ctypes).  Global env e lives in
    group g at local index j; outputs are gathered back into [E, ...] arrays in global env order."""

    def __init__(self, tracks, num_cars, shards=1, threads=8):
        from concurrent.futures import ThreadPoolExecutor
        tracks = list(tracks)
        self.E, self.C = len(tracks), num_cars
        keys = sorted(set(tracks))
        members = []
        for t in keys:
            envs = [e for e in range(self.E) if tracks[e] == t]
            for s in range(shards):
                part = envs[s::shards]
                if part:
                    members.append((t, np.array(part, np.int64)))
        self.groups = [(OracleEnv(t, len(m), num_cars), m) for t, m in members]
        self.where = {}
        for g, (_, m) in enumerate(self.groups):
            for j, e in enumerate(m.tolist()):
                self.where[e] = (g, j)
        self.pool = ThreadPoolExecutor(max_workers=min(threads, len(self.groups)))

    def _gather(self, outs):
        obs = np.zeros((self.E, self.C, 38), np.float32)
        rew = np.zeros((self.E, self.C), np.float32)
        cf = np.zeros((self.E, self.C), np.uint8)
        ef = np.zeros((self.E, 3), np.int32)
        for (_, m), (o, r, c, f) in zip(self.groups, outs):
            obs[m], rew[m], cf[m], ef[m] = o, r, c, f
        return obs, rew, cf, ef

    def reset(self, envs=None):
        if envs is None:
            for env, _ in self.groups:
                env.reset()
        else:
            for e in envs:
                g, j = self.where[int(e)]
                self.groups[g][0].reset(j)
        return self.outputs()

    def step(self, actions):
        a = np.asarray(actions, np.float32).reshape(self.E, self.C, 2)
        futs = [self.pool.submit(env.step, a[m]) for env, m in self.groups]
        return self._gather([f.result() for f in futs])

    def outputs(self):
        return self._gather([env.outputs() for env, _ in self.groups])

    def close(self):
        self.pool.shutdown()
        for env, _ in self.groups:
            env.close()


def car_state(env, idx, n_fields=71):
    L = lib()
    L.or_car_state.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    o = np.zeros(n_fields, np.float64)
    L.or_car_state(env.h, idx, _p(o, ctypes.c_double))
    return o


# ---------------------------------------------------------------- GPU state -> oracle (state injection)
GPU_MAXC, N_EI32 = 16, 5


def _a256(x):
    return (x + 255) & ~255


def gpu_arena(blob, E, C):
    """Split a nascar_get_state blob (uint8, the arena of nascar_create: nascar_kernels.hip, nascar_layout.h) into its
    blocks: per-car f32 / f64 / i32 fields, acceleration ring, contact records (raw words), listener keys / normals,
    per-env time and words, rule-driver state."""
    from gpu_state import F32, F64, I32
    b = np.ascontiguousarray(blob).view(np.uint8)
    N = E * C
    out, o = {}, 0

    def take(name, nbytes, dtype, shape):
        nonlocal o
        out[name] = b[o:o + nbytes].view(dtype).reshape(shape)
        o = _a256(o + nbytes)
    take("f32", 4 * len(F32) * N, np.float32, (len(F32), N))
    take("f64", 8 * len(F64) * N, np.float64, (len(F64), N))
    take("i32", 4 * len(I32) * N, np.int32, (len(I32), N))
    take("acc", 8 * 20 * N, np.float64, (20, N))
    take("ct", 80 * GPU_MAXC * N, np.int32, (N, GPU_MAXC * 20))
    take("key", 4 * GPU_MAXC * N, np.int32, (N, GPU_MAXC))
    take("n", 8 * GPU_MAXC * N, np.float32, (N, GPU_MAXC * 2))
    take("time", 8 * E, np.float64, (E,))
    take("ei32", 4 * N_EI32 * E, np.int32, (N_EI32, E))
    take("ctl", 8 * 4 * N, np.float64, (N, 4))
    assert o == _a256(len(b)) or o == len(b), (o, len(b))
    return out


def inject_gpu_state(orc, blob, E, C, envs):
    """Continue OracleEnv `orc` (len(envs) envs x C cars) from the GPU state `blob` of an E x C engine: oracle env i
    takes GPU env envs[i].  Returns the driver state rows (throttle_brake, steering, last_forward, speed_limit) of
    the selected cars, to seed the host rule driver (tests/drivers.py) as the device one stands."""
    A = gpu_arena(blob, E, C)
    L = orc.L
    orc.reset()   # every car's world wired to the track (the injected state then overwrites its fields)
    dp, ip, fp = ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_float)
    L.or_set_car_full.argtypes = [ctypes.c_void_p, ctypes.c_int, dp, dp, ip, dp, ip, ip, fp]
    L.or_set_env_full.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_double] + [ctypes.c_int] * 5
    rows = []
    for i, ge in enumerate(envs):
        t = A["ei32"][:, ge]
        L.or_set_env_full(orc.h, i, float(A["time"][ge]), int(t[0]), int(t[1]), int(t[2]), int(t[3]), int(t[4]))
        for car in range(C):
            n = ge * C + car
            f32 = np.ascontiguousarray(A["f32"][:, n].astype(np.float64))
            f64 = np.ascontiguousarray(A["f64"][:, n])
            i32 = np.ascontiguousarray(A["i32"][:, n])
            acc = np.ascontiguousarray(A["acc"][:, n])
            ct = np.ascontiguousarray(A["ct"][n])
            key = np.ascontiguousarray(A["key"][n])
            nn = np.ascontiguousarray(A["n"][n])
            L.or_set_car_full(orc.h, i * C + car, _p(f32, ctypes.c_double), _p(f64, ctypes.c_double),
                              _p(i32, ctypes.c_int32), _p(acc, ctypes.c_double), _p(ct, ctypes.c_int32),
                              _p(key, ctypes.c_int32), _p(nn, ctypes.c_float))
            rows.append(A["ctl"][n])
    return np.array(rows)

"""ctypes binding of libnascar.so (the C ABI declared in include/nascar.h).

The product path has exactly one implementation -- the HIP kernels in
libnascar.so.  There is no CPU fallback: if the library is missing or no HIP
device is visible, the env constructors raise.
"""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NASCAR_LIB") or os.path.join(HERE, "libnascar.so")   # NASCAR_LIB: A/B experiments
CSRC = os.path.join(HERE, "csrc")

INFO_FIELDS = ["x", "y", "vx", "vy", "angle", "omega", "speed", "lap_count", "last_lap_time", "best_lap_time",
               "is_timing", "current_lap_time", "total_distance_traveled", "has_crossed_startline", "disabled",
               "cumulative_reward", "cumulative_impact_force", "on_track", "engine_rpm", "simulation_time",
               "n_contacts", "error", "track_progress", "perf_count", "perf_max_speed", "perf_first_fast"]
N_INFO = len(INFO_FIELDS)
INFO_INDEX = {f: i for i, f in enumerate(INFO_FIELDS)}
OBS_DIM = 38

# car flag bits / env flag bits (csrc/nascar_layout.h)
CF_DISABLED, CF_JUST_DISABLED, CF_COLLISION, CF_LAP, CF_ERROR = 1, 2, 4, 8, 128
EF_TERMINATED, EF_TRUNCATED, EF_RESET = 1, 2, 8
TRAJ_RECORDS, TRAJ_OBS = 1, 2          # nascar_rollout traj flags (include/nascar.h)
REASONS = {0: None, 1: "all_cars_disabled", 2: "all_active_cars_low_reward (threshold: -250.0)",
           3: "time_limit", 4: "truncated"}

# -fno-slp-vectorize: the one-lane-per-car code is long dependent scalar chains (Box2D's solver / GJK / TOI per car), and
# the SLP vectorizer packs pairs of its f32 operations into v_pk_* instructions plus the v_mov shuffles that feed them,
# lengthening the chains a lone wave waits on (driver's command, 3 A/B rounds: 144.0 -> 139.2 us per step; round 5)
HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-fno-fast-math", "-fno-slp-vectorize", "-fPIC",
               "-shared", "-std=c++17", "-Wno-unused-value", "-Wno-unused-result"]


class NascarConfig(ctypes.Structure):
    _fields_ = [("num_envs", ctypes.c_int32), ("num_cars", ctypes.c_int32), ("reset_on_lap", ctypes.c_int32),
                ("device", ctypes.c_int32), ("start_x", ctypes.c_double), ("start_y", ctypes.c_double),
                ("start_angle", ctypes.c_double)]


def build(verbose=False):
    """Compile csrc/nascar_kernels.hip for gfx950 into nascargymnasium_amd/libnascar.so (in-tree)."""
    src = os.path.join(CSRC, "nascar_kernels.hip")
    cmd = ["hipcc"] + HIPCC_FLAGS + ["-o", LIB_PATH, src]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed:\n" + r.stderr[-4000:])
    if verbose:
        print(" ".join(cmd))
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'` "
                           "(there is no CPU fallback for the product path)")
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
    d_p = ctypes.POINTER(ctypes.c_double)
    L.nascar_create.argtypes = [ctypes.POINTER(NascarConfig), ctypes.POINTER(vp)]
    L.nascar_create.restype = ctypes.c_int
    L.nascar_destroy.argtypes = [vp]
    L.nascar_destroy.restype = None
    L.nascar_last_error.restype = ctypes.c_char_p
    L.nascar_add_track.argtypes = [vp, d_p, i32, ctypes.c_double, d_p, i32]
    L.nascar_add_track.restype = ctypes.c_int
    L.nascar_set_env_tracks.argtypes = [vp, ctypes.POINTER(i32)]
    L.nascar_set_env_tracks.restype = ctypes.c_int
    L.nascar_reset.argtypes = [vp, vp, vp, vp]
    L.nascar_reset.restype = ctypes.c_int
    L.nascar_step.argtypes = [vp, vp, i32, vp, vp, vp, vp, i32, vp, vp]
    L.nascar_step.restype = ctypes.c_int
    L.nascar_step_driven.argtypes = [vp, i32, u64, i64, vp, vp, vp, vp, i32, vp, vp]
    L.nascar_step_driven.restype = ctypes.c_int
    L.nascar_rollout.argtypes = [vp, i32, u64, i64, i32, vp, vp, vp, vp, i32, i32, vp]
    L.nascar_rollout.restype = ctypes.c_int
    L.nascar_set_car_contact.argtypes = [vp, i32]
    L.nascar_set_car_contact.restype = ctypes.c_int
    L.nascar_set_rollout_streams.argtypes = [vp, i32]
    L.nascar_set_rollout_streams.restype = ctypes.c_int
    L.nascar_get_rollout_streams.argtypes = [vp]
    L.nascar_get_rollout_streams.restype = ctypes.c_int
    L.nascar_set_rollout_pipe.argtypes = [vp, i32]
    L.nascar_set_rollout_pipe.restype = ctypes.c_int
    L.nascar_rollout_pipe_status.argtypes = [vp, vp]
    L.nascar_rollout_pipe_status.restype = ctypes.c_int
    L.nascar_set_envs_per_block.argtypes = [vp, i32]
    L.nascar_set_envs_per_block.restype = ctypes.c_int
    L.nascar_get_envs_per_block.argtypes = [vp]
    L.nascar_get_envs_per_block.restype = ctypes.c_int
    L.nascar_set_sensor_lanes.argtypes = [vp, i32]
    L.nascar_set_sensor_lanes.restype = ctypes.c_int
    L.nascar_set_sensor_block.argtypes = [vp, i32]
    L.nascar_set_sensor_block.restype = ctypes.c_int
    L.nascar_set_beam_cell.argtypes = [vp, ctypes.c_float]
    L.nascar_set_beam_cell.restype = ctypes.c_int
    L.nascar_set_fused_logic.argtypes = [vp, i32]
    L.nascar_set_fused_logic.restype = ctypes.c_int
    L.nascar_get_fused_logic.argtypes = [vp]
    L.nascar_get_fused_logic.restype = ctypes.c_int
    L.nascar_set_perf_history.argtypes = [vp, i32, vp]
    L.nascar_set_perf_history.restype = ctypes.c_int
    L.nascar_get_info.argtypes = [vp, vp, vp]
    L.nascar_get_info.restype = ctypes.c_int
    L.nascar_state_bytes.argtypes = [vp]
    L.nascar_state_bytes.restype = i64
    L.nascar_get_state.argtypes = [vp, vp, vp]
    L.nascar_get_state.restype = ctypes.c_int
    L.nascar_set_state.argtypes = [vp, vp, vp]
    L.nascar_set_state.restype = ctypes.c_int
    L.nascar_policy_actions.argtypes = [vp, i32, u64, i64, vp, vp, vp]
    L.nascar_policy_actions.restype = ctypes.c_int
    fp = ctypes.POINTER(ctypes.c_float)
    L.nascar_set_actor.argtypes = [vp, fp, fp, fp, fp, fp, fp, i32, i32, i32]
    L.nascar_set_actor.restype = ctypes.c_int
    L.nascar_set_actor_precision.argtypes = [vp, i32]
    L.nascar_set_actor_precision.restype = ctypes.c_int
    L.nascar_actor_forward.argtypes = [vp, vp, i32, vp, vp]
    L.nascar_actor_forward.restype = ctypes.c_int
    L.nascar_set_step_events.argtypes = [vp, ctypes.POINTER(vp), i32]
    L.nascar_set_step_events.restype = ctypes.c_int
    L.nascar_debug_sincosf.argtypes = [vp, vp, vp, i32, vp]
    L.nascar_debug_sincosf.restype = ctypes.c_int
    L.nascar_debug_sensors.argtypes = [vp, vp, vp, i32, vp]
    L.nascar_debug_sensors.restype = ctypes.c_int
    i32p, u64p = ctypes.POINTER(i32), ctypes.POINTER(u64)
    L.nascar_track_draw.argtypes = [i32, u64p, i32p, i32p, i32p, i32, i32p]
    L.nascar_track_draw.restype = ctypes.c_int
    L.nascar_set_random_tracks.argtypes = [vp, i32p, i32, u64p, i32p, vp]
    L.nascar_set_random_tracks.restype = ctypes.c_int
    L.nascar_get_env_tracks.argtypes = [vp, vp, vp, vp]
    L.nascar_get_env_tracks.restype = ctypes.c_int
    L.nascar_vec_post.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.nascar_vec_post.restype = ctypes.c_int
    L.nascar_check_actions.argtypes = [vp, vp, i32, vp, vp]
    L.nascar_check_actions.restype = ctypes.c_int
    L.nascar_set_track_cache.argtypes = [i32, ctypes.c_char_p]
    L.nascar_set_track_cache.restype = ctypes.c_int
    L.nascar_prebuild_track.argtypes = [d_p, i32, ctypes.c_double, d_p, i32, ctypes.c_float]
    L.nascar_prebuild_track.restype = ctypes.c_int
    L.nascar_debug_block_map.argtypes = [vp, vp, vp, i32, vp]
    L.nascar_debug_block_map.restype = ctypes.c_int
    _lib = L
    # track build cache: NASCAR_TRACK_CACHE names an on-disk cache directory (none by default; bench.py sets one for
    # multi-rank runs), NASCAR_TRACK_RETAIN the builds kept alive after their last handle (default 8)
    set_track_cache(int(os.environ.get("NASCAR_TRACK_RETAIN", "8")), os.environ.get("NASCAR_TRACK_CACHE", ""))
    return L


EXPORTED = ["nascar_create", "nascar_destroy", "nascar_last_error", "nascar_add_track", "nascar_set_env_tracks",
            "nascar_reset", "nascar_step", "nascar_step_driven", "nascar_rollout", "nascar_get_info", "nascar_set_perf_history", "nascar_set_car_contact", "nascar_set_rollout_streams", "nascar_get_rollout_streams", "nascar_set_rollout_pipe", "nascar_rollout_pipe_status", "nascar_set_envs_per_block", "nascar_get_envs_per_block", "nascar_set_sensor_lanes", "nascar_set_sensor_block", "nascar_set_beam_cell", "nascar_set_fused_logic", "nascar_get_fused_logic", "nascar_state_bytes", "nascar_get_state",
            "nascar_set_state", "nascar_policy_actions", "nascar_set_step_events", "nascar_set_actor", "nascar_set_actor_precision", "nascar_actor_forward",
            "nascar_debug_sincosf", "nascar_debug_sensors", "nascar_track_draw", "nascar_set_random_tracks",
            "nascar_get_env_tracks", "nascar_vec_post", "nascar_check_actions", "nascar_set_track_cache",
            "nascar_prebuild_track", "nascar_debug_block_map"]


def check(rc):
    if rc < 0:
        raise RuntimeError("libnascar: " + lib().nascar_last_error().decode())
    return rc


def track_draw(seeds, k, current, tracks):
    """nascar_track_draw (host): the random-track mode's draw k of each env -- its next track id given its seed and
    current track (-1: none), uniform over `tracks` minus the current one (CarEnv._select_random_track,
    src/car_env.py:264-287).  Vectorised over the envs; returns an int32 array."""
    import numpy as np
    seeds = np.ascontiguousarray(seeds, np.uint64).ravel()
    n = seeds.size
    k = np.ascontiguousarray(np.broadcast_to(np.asarray(k, np.int32), (n,)))
    cur = np.ascontiguousarray(np.broadcast_to(np.asarray(current, np.int32), (n,)))
    tr = np.ascontiguousarray(tracks, np.int32)
    out = np.empty(n, np.int32)
    i32p, u64p = ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_uint64)
    check(lib().nascar_track_draw(n, seeds.ctypes.data_as(u64p), k.ctypes.data_as(i32p), cur.ctypes.data_as(i32p),
                                  tr.ctypes.data_as(i32p), tr.size, out.ctypes.data_as(i32p)))
    return out


def set_track_cache(retain=8, directory=""):
    """nascar_set_track_cache: `retain` track builds kept alive after their last handle; `directory` the on-disk cache of
    host-built track tables ("" = none)."""
    check(lib().nascar_set_track_cache(int(retain), (directory or "").encode()))


def prebuild_track(path, beam_cell=1.0):
    """nascar_prebuild_track (host only, no GPU): the track's tables into the disk cache.  True if they were there
    already, False if built now."""
    import numpy as np
    from .track import build_walls, load_track, track_path
    t = load_track(track_path(path))
    seg = np.ascontiguousarray(t.segment_table())
    walls = np.ascontiguousarray(build_walls(t)[:, :4])
    dp = ctypes.POINTER(ctypes.c_double)
    return bool(check(lib().nascar_prebuild_track(seg.ctypes.data_as(dp), seg.shape[0], float(t.total_length),
                                                  walls.ctypes.data_as(dp), walls.shape[0], float(beam_cell))))

"""nascargymnasium_amd -- MI355X-native batched CarEnv (heihachi78/NascarGymnasium hot path).

The reference's per-car Python/Box2D step (src/car_env.py CarEnv.step) runs here as
one fused HIP kernel for gfx950 over E envs x C cars (libnascar.so, include/nascar.h).

    from nascargymnasium_amd import CarEnv          # Gymnasium API, drop-in for src.car_env.CarEnv
    from nascargymnasium_amd import BatchedCarEnv   # E x C cars on device tensors
"""
from .track import Track, available_tracks, build_walls, load_track, track_path  # noqa: F401

__all__ = ["Track", "available_tracks", "build_walls", "load_track", "track_path", "BatchedCarEnv", "CarEnv",
           "BaseEnv", "VecCarEnv"]


def __getattr__(name):   # torch-dependent pieces load lazily
    if name == "BatchedCarEnv":
        from .batched import BatchedCarEnv
        return BatchedCarEnv
    if name in ("CarEnv", "BaseEnv"):
        from . import car_env
        return getattr(car_env, name)
    if name == "VecCarEnv":
        from .vec_env import VecCarEnv
        return VecCarEnv
    raise AttributeError(name)

"""Replay a golden env scenario (tests/golden/env_*.npz) through a batched env
implementation and compare step by step.  Used by the CPU oracle tests and the
GPU parity tests.  TEST INFRASTRUCTURE."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TRACKS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "nascargymnasium_amd", "tracks")


def scenarios():
    return sorted(f[4:-4] for f in os.listdir(GOLDEN) if f.startswith("env_") and f.endswith(".npz"))


def load(name):
    d = np.load(os.path.join(GOLDEN, f"env_{name}.npz"))
    return {k: d[k] for k in d.files}


DISCRETE_TO_CONTINUOUS = np.array([[0, 0], [1, 0], [-1, 0], [0, -1], [0, 1]], np.float32)  # src/base_env.py:227-252


def is_discrete(d):
    return bool(d.get("discrete", False))


def continuous_actions(d, k):
    """step k's actions as [C, 2] float32 (discrete fixtures mapped with BaseEnv._discrete_to_continuous)"""
    a = d["actions"][k]
    return DISCRETE_TO_CONTINUOUS[a] if is_discrete(d) else a


def start_kwargs(d):
    """CarEnv(start_position=, start_angle=) of a fixture recorded with a non-default start pose (else {})"""
    if "start_angle" not in d:
        return {}
    sp = d["start_position"]
    return {"start_position": None if np.isnan(sp).any() else (float(sp[0]), float(sp[1])),
            "start_angle": float(d["start_angle"])}


def first_mismatch(a, b):
    """index of the first step whose arrays differ (== semantics, NaN==NaN), or -1"""
    a = np.asarray(a); b = np.asarray(b)
    eq = (a == b) | (np.isnan(a) & np.isnan(b)) if a.dtype.kind == "f" else (a == b)
    eq = eq.reshape(eq.shape[0], -1).all(axis=1)
    bad = np.nonzero(~eq)[0]
    return int(bad[0]) if len(bad) else -1

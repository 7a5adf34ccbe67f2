"""Action / observation spaces of the reference env.

When gymnasium is importable (a user's training environment) its own spaces are used,
so ``isinstance(env.action_space, gymnasium.spaces.Box)`` holds as for the reference.
Otherwise (this image has no gymnasium) the three spaces the reference uses are restated
with gymnasium 0.29.1's ``contains`` semantics (requirements.txt:18 pins 0.29.1):

* ``Box.contains``: non-ndarray input is converted with ``np.asarray(x, dtype)``;
  True iff ``np.can_cast(x.dtype, dtype)`` and the shape matches exactly and every
  element is within [low, high].
* ``Discrete.contains``: python int, or an integer numpy scalar / 0-d array, in [start, start+n).
* ``MultiDiscrete.contains``: sequences become arrays; ndarray of matching shape, non-object
  dtype, ``start <= x < start + nvec`` elementwise.

The space objects are the reference's (src/base_env.py:56-99).
"""
from collections.abc import Sequence

import numpy as np

try:  # pragma: no cover - exercised only where gymnasium is installed
    import gymnasium as _gym
    from gymnasium.spaces import Box, Discrete, MultiDiscrete  # noqa: F401
    Env = _gym.Env
    HAVE_GYMNASIUM = True
except ImportError:
    HAVE_GYMNASIUM = False

    class Space:
        def __init__(self, shape, dtype, seed=None):
            self.shape = None if shape is None else tuple(shape)
            self.dtype = None if dtype is None else np.dtype(dtype)
            self._np_random = np.random.default_rng(seed)

        def seed(self, seed=None):
            self._np_random = np.random.default_rng(seed)
            return [seed]

        @property
        def np_random(self):
            return self._np_random

        def __contains__(self, x):
            return self.contains(x)

    class Box(Space):
        def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
            dtype = np.dtype(dtype)
            if shape is None:
                shape = np.shape(low) if np.ndim(low) else np.shape(high)
            shape = tuple(shape)
            self.low = np.full(shape, low, dtype=dtype) if np.isscalar(low) else np.asarray(low, dtype=dtype)
            self.high = np.full(shape, high, dtype=dtype) if np.isscalar(high) else np.asarray(high, dtype=dtype)
            if self.low.shape != shape or self.high.shape != shape:
                raise ValueError(f"low/high shape {self.low.shape}/{self.high.shape} != {shape}")
            super().__init__(shape, dtype, seed)

        def contains(self, x) -> bool:
            if not isinstance(x, np.ndarray):
                try:
                    x = np.asarray(x, dtype=self.dtype)
                except (ValueError, TypeError):
                    return False
            return bool(np.can_cast(x.dtype, self.dtype) and x.shape == self.shape
                        and np.all(x >= self.low) and np.all(x <= self.high))

        def sample(self):
            return self.np_random.uniform(self.low, self.high, self.shape).astype(self.dtype)

        def __repr__(self):
            return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"

    class Discrete(Space):
        def __init__(self, n, seed=None, start=0):
            self.n = np.int64(n)
            self.start = np.int64(start)
            super().__init__((), np.int64, seed)

        def contains(self, x) -> bool:
            if isinstance(x, int):
                v = np.int64(x)
            elif isinstance(x, (np.generic, np.ndarray)) and (np.issubdtype(x.dtype, np.integer) and x.shape == ()):
                v = np.int64(x)
            else:
                return False
            return bool(self.start <= v < self.start + self.n)

        def sample(self):
            return np.int64(self.start + self.np_random.integers(self.n))

        def __repr__(self):
            return f"Discrete({self.n})"

    class MultiDiscrete(Space):
        def __init__(self, nvec, dtype=np.int64, seed=None, start=None):
            self.nvec = np.array(nvec, dtype=dtype, copy=True)
            self.start = np.zeros_like(self.nvec) if start is None else np.array(start, dtype=dtype)
            super().__init__(self.nvec.shape, dtype, seed)

        def contains(self, x) -> bool:
            if isinstance(x, Sequence):
                x = np.array(x)
            return bool(isinstance(x, np.ndarray) and x.shape == self.shape and x.dtype != object
                        and np.all(self.start <= x) and np.all(x - self.start < self.nvec))

        def sample(self):
            return (self.start + self.np_random.integers(self.nvec)).astype(self.dtype)

        def __repr__(self):
            return f"MultiDiscrete({self.nvec})"

    class Env:
        """Minimal gymnasium.Env stand-in: seeding + the attributes callers read."""
        metadata = {"render_modes": []}
        render_mode = None
        spec = None

        def reset(self, *, seed=None, options=None):
            if seed is not None:
                self._np_random = np.random.default_rng(seed)

        @property
        def np_random(self):
            if getattr(self, "_np_random", None) is None:
                self._np_random = np.random.default_rng()
            return self._np_random

        @property
        def unwrapped(self):
            return self

        def close(self):
            pass

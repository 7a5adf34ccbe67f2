"""Host restatements of the device action sources (nascar_policy_actions, csrc/nascar_kernels.hip
policy_kernel) -- TEST INFRASTRUCTURE ONLY (used by tests/ and bench.py's cpu_baseline leg).

* policy 0: counter-hash uniform U[-1,1]^2, key = (seed, car, step)
* policy 1: BaseController._fallback_control (game/control/base_controller.py:39-103)
* policy 3: policy 1 whose action is replaced by policy 0's draw with probability 0.15 per car-step
  (the "rule_noisy" driver of oracle/gen_golden.py with a counter hash instead of a host RNG)
"""
import numpy as np

M64 = (1 << 64) - 1
NOISE_P16 = 9830          # 0.15 * 65536


def mix32(x):
    """splitmix64 finaliser, upper 32 bits (uint64 numpy arrays, wrapping arithmetic)."""
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(M64)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    x = x ^ (x >> np.uint64(31))
    return (x >> np.uint64(32)).astype(np.uint32)


def hash_keys(N, seed, step, ids=None):
    """per-car counter keys; `ids` (optional, length N): the cars' global indices in the device engine (car n of env e
    is e * C + n there), so a host shard of a few envs draws the same numbers as those cars on the device"""
    n = np.arange(N, dtype=np.uint64) if ids is None else np.asarray(ids, dtype=np.uint64)
    with np.errstate(over="ignore"):
        s = np.uint64((seed * 0x100000001B3) & M64)
        k = np.uint64((step * 0x9E3779B1) & M64)
        return s ^ (n << np.uint64(24)) ^ k


def uniform_actions(N, seed, step, ids=None):
    key = hash_keys(N, seed, step, ids)
    with np.errstate(over="ignore"):
        u0 = (mix32(key) >> np.uint32(8)).astype(np.float32) * np.float32(2.0 / 16777216.0) - np.float32(1.0)
        u1 = (mix32(key ^ np.uint64(0xABCDEF12345)) >> np.uint32(8)).astype(np.float32) * np.float32(2.0 / 16777216.0) \
            - np.float32(1.0)
    return np.stack([u0, u1], 1)


class RuleDriver:
    """Vectorised BaseController._fallback_control over N cars (state as the device keeps it:
    throttle_brake a Python float, steering / last_forward / speed_limit numpy float32 values)."""

    def __init__(self, N):
        self.tb = np.zeros(N, np.float64)
        self.steer = np.zeros(N, np.float32)
        self.last = np.zeros(N, np.float32)
        self.lim = np.zeros(N, np.float32)

    def __call__(self, obs):
        o = obs.reshape(-1, 38)
        fwd, spd = o[:, 22], o[:, 4]
        lim = np.where(self.last >= fwd, fwd, self.lim).astype(np.float32)
        lim = np.where(self.last < fwd, np.float32(1.0), lim).astype(np.float32)
        tb = self.tb.copy()
        tb = np.where(spd < lim * np.float32(0.95), tb + 0.1, tb)
        tb = np.where(spd > lim * np.float32(1.05), tb - 0.1, tb)
        r, l = o[:, 37], o[:, 23]
        with np.errstate(divide="ignore", invalid="ignore"):
            s_r = np.float32(1.0) - (l / r)
            s_l = (np.float32(1.0) - (r / l)) * np.float32(-1.0)
        steer = np.where(r > l, s_r, np.where(l > r, s_l, self.steer * np.float32(0.9))).astype(np.float32)
        tb = np.where(np.abs(steer) > np.float32(0.25), tb * 0.5, tb)
        tb = np.clip(tb, -1.0, 1.0)
        steer = np.clip(steer, np.float32(-1.0), np.float32(1.0)).astype(np.float32)
        self.tb, self.steer, self.last, self.lim = tb, steer, fwd.astype(np.float32), lim
        return np.stack([tb.astype(np.float32), steer], 1)


def noisy_mask(N, seed, step, ids=None):
    key = hash_keys(N, seed, step, ids)
    return (mix32(key ^ np.uint64(0x5DEECE66D)) >> np.uint32(16)) < NOISE_P16


class NoisyRuleDriver(RuleDriver):
    """ids: the cars' global indices on the device (default 0..N-1), which key the noise hash"""

    def __init__(self, N, seed=0, ids=None):
        super().__init__(N)
        self.N, self.seed = N, seed
        self.ids = None if ids is None else np.asarray(ids, dtype=np.uint64)
        if self.ids is not None and self.ids.shape != (N,):
            raise ValueError(f"ids must hold {N} car indices")

    def actions(self, obs, step):
        a = self(obs)
        m = noisy_mask(self.N, self.seed, step, self.ids)
        a[m] = uniform_actions(self.N, self.seed, step, self.ids)[m]
        return a

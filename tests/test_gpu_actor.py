"""Fused SAC actor (csrc/nascar_actor.h, bf16 MFMA) vs the PyTorch fp32 forward of the same
SB3 MlpPolicy actor (SACController.control -> model.predict(deterministic=True),
game/control/sac_control_class.py:80-115).

Stated tolerances (bf16 operands X, W1, relu(H1), W2, relu(H2); b1 and W3 as bf16 hi + lo pairs;
fp32 accumulation):
  * vs a PyTorch fp32 forward: max |delta action| <= 3e-2, mean <= 3e-3;
  * vs the same math with those operands rounded to bf16 (float64 accumulation): <= 2e-4.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _ref_fp32(w, x):
    t = {k: torch.from_numpy(v) for k, v in w.items()}
    xt = torch.from_numpy(x)
    h1 = torch.relu(xt @ t["actor.latent_pi.0.weight"].T + t["actor.latent_pi.0.bias"])
    h2 = torch.relu(h1 @ t["actor.latent_pi.2.weight"].T + t["actor.latent_pi.2.bias"])
    a = torch.tanh(h2 @ t["actor.mu.weight"].T + t["actor.mu.bias"]).numpy()
    lo, hi = np.float32(-1.0), np.float32(1.0)
    return lo + (np.float32(0.5) * (a + np.float32(1.0)) * (hi - lo))        # BasePolicy.unscale_action


def _bf16(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(torch.bfloat16).to(torch.float64).numpy()


def _hi_lo(a):
    a = np.asarray(a, np.float32)
    hi = _bf16(a)
    return hi, _bf16((a - hi).astype(np.float32))


def _ref_bf16(w, x):
    """the kernel's arithmetic in float64: bf16 X, W1, relu(H1), W2, relu(H2); b1 and W3 as bf16 hi + lo"""
    b1_hi, b1_lo = _hi_lo(w["actor.latent_pi.0.bias"])
    h1 = np.maximum(_bf16(x) @ _bf16(w["actor.latent_pi.0.weight"]).T + b1_hi + b1_lo, 0)
    h2 = np.maximum(_bf16(h1) @ _bf16(w["actor.latent_pi.2.weight"]).T + w["actor.latent_pi.2.bias"], 0)
    w3_hi, w3_lo = _hi_lo(w["actor.mu.weight"])
    return np.tanh(_bf16(h2) @ (w3_hi + w3_lo).T + w["actor.mu.bias"])


def _obs_batch(n, seed):
    """realistic observations (env rollouts) mixed with uniform ones over the observation box"""
    from nascargymnasium_amd.batched import BatchedCarEnv
    env = BatchedCarEnv(max(1, n // 4), 4, "daytona", device="cuda:0")
    env.reset()
    g = torch.Generator(device="cuda:0").manual_seed(seed)
    for _ in range(30):
        env.step(torch.rand((env.E, 4, 2), generator=g, device="cuda:0") * 2 - 1)
    real = env.obs.reshape(-1, 38).cpu().numpy()
    env.close()
    rng = np.random.default_rng(seed)
    uni = rng.uniform(-1, 1, (n, 38)).astype(np.float32)
    uni[:, 4:5] = np.abs(uni[:, 4:5]); uni[:, 7:19] = np.abs(uni[:, 7:19]); uni[:, 22:] = np.abs(uni[:, 22:])
    x = np.concatenate([real, uni])[:n]
    return np.ascontiguousarray(x, np.float32)


@pytest.mark.parametrize("n,seed", [(4096, 0), (1000, 1), (37, 2), (1, 3)])
def test_actor_matches_fp32_reference(n, seed):
    from nascargymnasium_amd.batched import BatchedCarEnv
    from nascargymnasium_amd.policy import random_actor
    w = random_actor(seed)
    x = _obs_batch(n, seed)
    env = BatchedCarEnv(1, 1, "daytona", device="cuda:0")
    env.set_actor(w, precision="bf16")
    got = env.actor_forward(torch.from_numpy(x).cuda()).cpu().numpy()
    env.close()
    ref = _ref_fp32(w, x)
    d = np.abs(got - ref)
    assert got.shape == (n, 2) and np.all(np.isfinite(got))
    assert d.max() <= 3e-2 and d.mean() <= 3e-3, (d.max(), d.mean())
    assert np.abs(got - _ref_bf16(w, x)).max() <= 2e-4


def test_policy_2_is_the_actor_on_the_env_obs():
    from nascargymnasium_amd.batched import BatchedCarEnv
    from nascargymnasium_amd.policy import random_actor
    env = BatchedCarEnv(300, 3, "martinsville", device="cuda:0")
    env.set_actor(random_actor(7), precision="bf16")
    env.reset()
    for k in range(20):
        a = env.policy_actions(2).clone()
        assert torch.equal(a, env.actor_forward(env.obs))
        env.step(a, auto_reset=True)
    env.close()


def _sac_1235():
    import os
    from golden_replay import GOLDEN
    d = np.load(os.path.join(GOLDEN, "sac_1235_actor.npz"))
    from nascargymnasium_amd.policy import ACTOR_KEYS
    return {k: d[k.replace(".", "__")] for k in ACTOR_KEYS}, d["obs"], d["actions_fp32"]


def test_sac_1235_fp32_matches_reference():
    """The reference's own SAC checkpoint (game/control/models/sac_1235.zip, via oracle/gen_actor_fixture.py) on
    2236 golden-trace observations: the fp32 actor kernel equals the float32 SB3 predict() restatement to 1e-5
    (summation order only), through nascar_actor_forward and through policy 2 on an env's obs buffer."""
    from nascargymnasium_amd.batched import BatchedCarEnv
    w, x, want = _sac_1235()
    env = BatchedCarEnv(1, 1, "daytona", device="cuda:0")
    env.set_actor(w, precision="fp32")
    got = env.actor_forward(torch.from_numpy(x).cuda()).cpu().numpy()
    env.close()
    d = np.abs(got - want)
    assert d.max() <= 1e-5, d.max()
    n = len(x) // 4 * 4
    env = BatchedCarEnv(n // 4, 4, "daytona", device="cuda:0")
    env.set_actor(w, precision="fp32")
    env.obs.copy_(torch.from_numpy(x[:n].reshape(n // 4, 4, 38)).cuda())
    got2 = env.policy_actions(2).cpu().numpy().reshape(n, 2)
    env.close()
    assert np.array_equal(got2, got[:n])


def test_sac_1235_bf16_error_is_the_documented_one():
    """The opt-in bf16-MFMA actor on the same checkpoint and observations.  Measured: max |delta| 0.40, mean 8.7e-3
    -- the trained policy's pre-tanh means are large and sensitive, so bf16 operands are NOT faithful to the
    reference here (fp32, the default, is); this pins the documented error, and the kernel must
    still agree with a float64 emulation of its own bf16 operand rounding."""
    from nascargymnasium_amd.batched import BatchedCarEnv
    w, x, want = _sac_1235()
    env = BatchedCarEnv(1, 1, "daytona", device="cuda:0")
    env.set_actor(w, precision="bf16")
    got = env.actor_forward(torch.from_numpy(x).cuda()).cpu().numpy()
    env.close()
    d = np.abs(got - want)
    assert d.max() <= 0.45 and d.mean() <= 1e-2, (d.max(), d.mean())
    emu = _ref_bf16(w, x)
    emu = np.float32(-1.0) + (np.float32(0.5) * (emu.astype(np.float32) + np.float32(1.0)) * np.float32(2.0))
    assert np.abs(got - emu).max() <= 1e-2


@pytest.mark.parametrize("n,seed", [(4096, 0), (37, 2), (1, 3)])
def test_actor_fp32_random_weights(n, seed):
    from nascargymnasium_amd.batched import BatchedCarEnv
    from nascargymnasium_amd.policy import random_actor
    w = random_actor(seed)
    x = _obs_batch(n, seed)
    env = BatchedCarEnv(1, 1, "daytona", device="cuda:0")
    env.set_actor(w, precision="fp32")
    got = env.actor_forward(torch.from_numpy(x).cuda()).cpu().numpy()
    env.close()
    assert np.abs(got - _ref_fp32(w, x)).max() <= 1e-5

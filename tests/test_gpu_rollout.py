"""nascar_rollout (sharded over internal streams, the default, the fused multi-step kernel and the pipelined pair of
persistent kernels) against the per-step path: K x (nascar_policy_actions +
nascar_step with auto-reset) from the same state must give the same per-step rewards / car flags / env flags,
the same final observation and the same final engine state, bit for bit."""
import os

import numpy as np
import pytest

from golden_replay import TRACKS

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _engine(tracks, E, C, reset_on_lap=False, envs_per_block=None):
    from nascargymnasium_amd.batched import BatchedCarEnv
    files = [os.path.join(TRACKS, tracks[e % len(tracks)]) for e in range(E)]
    return BatchedCarEnv(E, C, files, reset_on_lap=reset_on_lap, device="cuda:0", envs_per_block=envs_per_block)


def _per_step(env, policy, seed, step0, K):
    R, CF, EF = [], [], []
    for k in range(K):
        a = env.policy_actions(policy, seed=seed, step=step0 + k)
        env.launch_step(a, auto_reset=True)
        R.append(env.reward.clone()); CF.append(env.car_flags.clone()); EF.append(env.env_flags.clone())
    return torch.stack(R), torch.stack(CF), torch.stack(EF)


@pytest.mark.parametrize("streams", [4, 0, -1])    # sharded rollout (default) / fused rollout kernel / pipelined rollout
@pytest.mark.parametrize("tracks,E,C,policy,warm,K,epb", [
    (["daytona.track"], 48, 10, 3, 600, 900, 12),      # the bench workload and layout: noisy driver, contacts
    (["daytona.track"], 16, 2, 1, 0, 400, None),       # rule driver from reset
    (["martinsville.track"], 32, 4, 0, 3500, 300, 8),  # uniform, reset_on_lap: the t > 60 s termination + auto-reset
    (["talladega.track", "michigan.track", "nascar2.track", "trioval.track"], 40, 3, 3, 900, 600, None),   # mixed tracks
    # 12 envs per workgroup: 2 track groups of 250 envs = 2 x 21 workgroups (the last of each with 10 envs), 3 uneven
    # shards of 14 workgroups
    (["daytona.track", "nascar.track"], 500, 10, 3, 1200, 200, 12),
    # cfg5's kind of batch: all 8 tracks, 72 envs each = 6 workgroups of 12 per track, interleaved over 4 shards
    (["daytona.track", "martinsville.track", "michigan.track", "nascar.track", "nascar2.track", "nascar_banked.track",
      "talladega.track", "trioval.track"], 576, 10, 3, 600, 150, 12),
])
def test_rollout_equals_per_step(tracks, E, C, policy, warm, K, epb, streams):
    """the per-step path at the automatic layout (one env per workgroup for these batch sizes) against the
    rollout at `epb` envs per workgroup: the same results whatever the schedule and the layout"""
    rol = policy == 0
    a, b = _engine(tracks, E, C, rol), _engine(tracks, E, C, rol, envs_per_block=epb)
    if streams == -1:
        b.set_rollout_pipe(512)
    else:
        b.set_rollout_streams(streams if E != 500 or streams == 0 else 3)
    a.reset()
    if warm:                                    # leave the reset state first (cars spread, contacts active)
        a.rollout(policy, warm, seed=5, step0=0, auto_reset=True)
    b.set_state(a.get_state())
    b.obs.copy_(a.obs)
    R, CF, EF = _per_step(a, policy, 5, warm, K)
    obs_b, Rb, CFb, EFb = b.rollout(policy, K, seed=5, step0=warm, auto_reset=True, trajectory=True)
    torch.cuda.synchronize()
    if streams == -1:
        assert b.rollout_pipe_status() == 0
    for k in range(K):
        assert torch.equal(R[k], Rb[k]), f"reward differs at step {k}"
        assert torch.equal(CF[k], CFb[k]), f"car flags differ at step {k}"
        assert torch.equal(EF[k], EFb[k]), f"env flags differ at step {k}"
    assert torch.equal(a.obs, obs_b)
    assert torch.equal(a.get_state(), b.get_state())
    n_contact = int(((CF & 4) != 0).sum())
    n_reset = int(((EF & 8) != 0).sum())
    if policy == 0:
        assert n_reset > 0          # reset_on_lap: envs terminate once t > 60 s (step 3601) and auto-reset
    if policy == 3:
        assert n_contact > 0
    a.close(); b.close()


def test_rollout_last_step_outputs_and_errors():
    env = _engine(["daytona.track"], 8, 2)
    env.reset()
    obs, rew, cf, ef = env.rollout(3, 50, seed=1)
    assert rew.shape == (8, 2) and obs.shape == (8, 2, 38) and cf.dtype == torch.uint8
    with pytest.raises(RuntimeError):
        env.rollout(2, 5)                        # policy 2 without an actor
    from nascargymnasium_amd.policy import random_actor
    env.set_actor(random_actor(0))
    env.set_rollout_streams(0)
    with pytest.raises(RuntimeError):
        env.rollout(2, 5)                        # the fused rollout kernel has no actor
    env.close()


@pytest.mark.parametrize("tracks,E,precision", [
    (["daytona.track"], 480, "fp32"),            # 40 workgroups of 12 envs: 4 shards, each its own actor launch
    (["daytona.track"], 480, "bf16"),
    (["daytona.track", "nascar.track"], 96, "fp32"),   # non-identity block map: one shard
])
def test_sharded_rollout_sac_equals_per_step(tracks, E, precision):
    """policy 2 in the sharded rollout (the actor per shard on its own cars) == per step: actor on the whole
    batch (nascar_policy_actions) + nascar_step."""
    from nascargymnasium_amd.policy import random_actor
    C, warm, K = 10, 300, 150
    a, b = _engine(tracks, E, C), _engine(tracks, E, C, envs_per_block=12)
    for e in (a, b):
        e.set_actor(random_actor(3), precision=precision)
    a.reset()
    a.rollout(3, warm, seed=2, step0=0, auto_reset=True)
    b.set_state(a.get_state())
    b.obs.copy_(a.obs)
    R, CF, EF = _per_step(a, 2, 0, 0, K)
    obs_b, Rb, CFb, EFb = b.rollout(2, K, auto_reset=True, trajectory=True)
    torch.cuda.synchronize()
    for k in range(K):
        assert torch.equal(R[k], Rb[k]), f"reward differs at step {k}"
        assert torch.equal(CF[k], CFb[k]) and torch.equal(EF[k], EFb[k]), f"flags differ at step {k}"
    assert torch.equal(a.obs, obs_b)
    assert torch.equal(a.get_state(), b.get_state())
    a.close(); b.close()


@pytest.mark.parametrize("policy", [0, 1, 3])
def test_step_driven_equals_policy_plus_step(policy):
    """nascar_step_driven (device action source inside the step launch) == nascar_policy_actions + nascar_step."""
    a, b = _engine(["daytona.track"], 48, 10), _engine(["daytona.track"], 48, 10)
    a.reset(); b.reset()
    for k in range(300):
        a.launch_step(a.policy_actions(policy, seed=4, step=k).clone(), auto_reset=True)
        b.step_driven(policy, seed=4, step=k, auto_reset=True)
        assert torch.equal(a.obs, b.obs) and torch.equal(a.reward, b.reward), k
        assert torch.equal(a.car_flags, b.car_flags) and torch.equal(a.env_flags, b.env_flags), k
    assert torch.equal(a.get_state(), b.get_state())
    a.close(); b.close()

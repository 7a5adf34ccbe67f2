"""BASELINE configs at their own car counts and horizons (round-3 verdict item 1).

* cfg5 -- mixed batch of all 8 .track files at 10 cars per env: every env equals the oracle on its own track,
  every step, under the bench's closed-loop noisy driver with staggered masked resets and in-launch auto-reset
  (reference: the per-env track of src/car_env.py:243-303 / 375-394).
* the bench workload over a whole episode: 24 x 10 daytona at the bench's 12 envs per workgroup (and at 1), noisy
  driver, >= 10 810 steps, so every env age the bench's steady-state window holds (0 .. 10 800 steps,
  src/car_env.py:1154) is pinned against the oracle at the layout the bench runs.
* cfg2's shape (1 car per env) at cfg2's layout (8 envs per workgroup) and at 128 and 1.
* cfg3's build-only car-car contact extension at its own shape (talladega x 10 cars, >= 256 envs): impulses
  reported, sharded rollout == per-step path, and switched off it equals a reference-behaviour engine from the same
  state.  No reference counterpart exists (src/constants/physics.py:9: every car has its own b2World), so this row
  is property-tested only.

Every oracle comparison runs one GPU engine per workgroup layout (tests/closed_loop.py): the wave-cooperative
SolveTOI / event manifolds, per-lane LDS contact slots and the logic kernel's LDS env passes then run with several
envs' cars sharing a wave, as in the bench.  The GPU runs nascar_step_driven (the device driver inside model_kernel, the bench's per-step path; the sharded
rollout equals it bit for bit, tests/test_gpu_rollout.py); the oracle groups step on host threads.
"""
import os

import numpy as np
import pytest

from closed_loop import closed_loop_vs_oracle, make_envs
from golden_replay import TRACKS

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.mark.timeout(900)
def test_cfg5_mixed_tracks_10_cars_vs_oracle():
    """cfg5 at its car count: 128 envs x 10 cars, env e on track e mod 8 (one launch, per-env track index: 16 envs
    per track), noisy driver closed loop with staggered resets and in-launch auto-reset, 900 steps; each env == the
    oracle on its own track every step (obs, rewards, disabled / done flags, termination reasons), at one env per
    workgroup and at the bench's 12 envs per workgroup (per track: one full 12-env workgroup and one of 4)."""
    from oracle_lib import OracleGroups
    tracks = sorted(f for f in os.listdir(TRACKS) if f.endswith(".track"))
    E, C, S = 128, 10, 900
    files = [os.path.join(TRACKS, tracks[e % 8]) for e in range(E)]
    envs = make_envs(E, C, files, [1, 12, 12], fused=(2,))
    orc = OracleGroups(files, C)
    stagger = {7 * e: e for e in range(8, E)}        # envs 8.. reset at staggered steps (ages spread)
    t = closed_loop_vs_oracle(envs, orc, S, seed=23, stagger=stagger)
    for env in envs:
        env.close()
    orc.close()
    assert t["contact"] > 0 and t["disabled"] > 0, t


@pytest.mark.timeout(1200)
def test_bench_workload_full_episode_vs_oracle():
    """The bench's steady-state workload over a whole episode at the bench's layout: 24 x 10 daytona at 12 envs per
    workgroup (2 full workgroups, 120 live lanes in two waves each, as the bench's 8192 x 10 runs; also through the
    fused model + logic kernel) and at one env per workgroup, noisy driver closed loop inside model_kernel, staggered
    resets (env e reset at step 450 e, so the env ages of every step spread over the episode as in the bench's
    settled window), in-launch auto-reset, 10 830 steps.
    Env 0 is never reset by the schedule, so unless an earlier termination ends it, it runs to the 10 800-step time
    limit (src/car_env.py:1154): every env age the bench's window holds is compared with the oracle every step."""
    from oracle_lib import OracleGroups
    E, C, S = 24, 10, 10830
    path = os.path.join(TRACKS, "daytona.track")
    envs = make_envs(E, C, path, [12, 1, 12], fused=(2,))
    orc = OracleGroups([path] * E, C, shards=8)
    stagger = {450 * e: e for e in range(1, E)}
    t = closed_loop_vs_oracle(envs, orc, S, seed=31, stagger=stagger)
    for env in envs:
        env.close()
    orc.close()
    assert t["contact"] > 0 and t["disabled"] > 0 and t["laps"] > 0, t
    assert 4 in t["reasons"] and t["max_age"] >= 10800, t      # an episode ran to the 10 800-step truncation


@pytest.mark.timeout(600)
def test_cfg2_one_car_layouts_vs_oracle():
    """cfg2's shape (1 car per env) at cfg2's own layout: 256 envs x 1 car daytona at 8 envs per workgroup (what the
    engine picks for 4096 x 1: 512 workgroups of 8 cars), at 128 envs per workgroup (two full waves per workgroup)
    and at one env per workgroup (there with 4 distance-sensor lanes per car instead of the small batch's 16); noisy
    driver closed loop, staggered resets, auto-reset, 2500 steps, == the oracle every step."""
    from oracle_lib import OracleGroups
    E, C, S = 256, 1, 2500
    path = os.path.join(TRACKS, "daytona.track")
    envs = make_envs(E, C, path, [8, 128, 1, 8], fused=(3,))
    envs[2].set_sensor_lanes(4)          # the small batch's default is 16 sensor lanes per car; pin 4 too
    orc = OracleGroups([path] * E, C, shards=4)
    stagger = {9 * e: e for e in range(1, E)}
    t = closed_loop_vs_oracle(envs, orc, S, seed=41, stagger=stagger)
    for env in envs:
        env.close()
    orc.close()
    assert t["contact"] > 0, t


@pytest.mark.timeout(600)
@pytest.mark.parametrize("E", [256, 8192])
def test_cfg3_car_contact_at_talladega_10_cars(E):
    """cfg3's extension (talladega, 10 cars per env -- a 5-row start grid), at 256 envs and at cfg3's own 8192: impulses
    are reported, the sharded rollout (4 shards at 8192) equals the per-step path bit for bit with contact on, and with
    contact off again the engine equals a reference-behaviour engine started from the same state."""
    from nascargymnasium_amd.batched import BatchedCarEnv
    from nascargymnasium_amd import _lib
    C = 10
    path = os.path.join(TRACKS, "talladega.track")
    F = _lib.INFO_INDEX
    env = BatchedCarEnv(E, C, path, device="cuda:0")
    env.set_car_contact(True)
    env.reset()
    inf = env.info_tensor().cpu().numpy()
    xy = inf[0, :, [F["x"], F["y"]]].T
    assert len({tuple(p) for p in xy.round(3).tolist()}) == C, "start grid not staggered"
    hits = 0
    for k in range(300):
        env.step_driven(3, seed=5, step=k, auto_reset=True)
        hits += int(((env.car_flags & 4) != 0).sum())
    assert hits > 0, "no car-car impulse reported"
    twin = BatchedCarEnv(E, C, path, device="cuda:0")
    twin.set_car_contact(True)
    twin.set_state(env.get_state()); twin.obs.copy_(env.obs)
    assert twin.rollout_streams > 1
    rew = torch.empty(100, E, C, device=env.device)
    for k in range(100):
        env.step_driven(3, seed=5, step=300 + k, auto_reset=True)
        rew[k] = env.reward
    _, trew, _, _ = twin.rollout(3, 100, seed=5, step0=300, auto_reset=True, trajectory=True)
    assert torch.equal(env.obs, twin.obs) and torch.equal(env.get_state(), twin.get_state())
    assert torch.equal(rew, trew)
    env.set_car_contact(False)
    ref = BatchedCarEnv(E, C, path, device="cuda:0")
    ref.set_state(env.get_state()); ref.obs.copy_(env.obs)
    for k in range(200):
        env.step_driven(3, seed=6, step=k, auto_reset=True)
        ref.step_driven(3, seed=6, step=k, auto_reset=True)
        assert torch.equal(env.obs, ref.obs) and torch.equal(env.reward, ref.reward), k
    assert torch.equal(env.get_state(), ref.get_state())
    for x in (env, twin, ref):
        x.close()


@pytest.mark.timeout(600)
def test_bench_steady_state_full_size_vs_oracle():
    """The bench's own workload at its full size, layout and schedule: daytona 8192 x 10 at 12 envs per workgroup,
    settled once by bench.settle (10 800 noisy-driver steps, env ages staggered over the episode).  Three engines then
    hold that state and run the same 150 steps:
      A -- one whole-batch launch per step through nascar_step_driven (the noisy driver inside the step kernel, the
           bench's per-step path); 64 of its envs (spread over the batch) are loaded into the CPU oracle
           (oracle_lib.inject_gpu_state, driver state included) and stepped by the host driver keyed by the device's
           global car ids: the 64 envs' obs, rewards, disabled / collision flags, done flags and termination reasons
           equal the oracle's every step;
      B -- the schedule bench.py TIMES (nascar_rollout on the default 4 shards / 4 streams, each shard's
           launches offset by its workgroups) in one 150-step call recording every step (trajectory + obs trajectory);
      C -- the same schedule exactly as bench.py's timed loop issues it (bench.Stepper: 3 calls of 50 steps, no
           records).
    Every step's observation, reward, car flags and env flags of all 81 920 cars of A equal B's records, and A, B and
    C end with byte-identical state arenas and observations.  The reference steps these cars one by one in Python
    (src/car_env.py:567-570, 678-803); the shards, streams and workgroup offsets must not change any result."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from drivers import NoisyRuleDriver
    from nascargymnasium_amd.batched import BatchedCarEnv
    from oracle_lib import OracleEnv, inject_gpu_state
    E, C, K, seed = 8192, 10, 150, 0
    path = os.path.join(TRACKS, "daytona.track")
    env = BatchedCarEnv(E, C, path, device="cuda:0")
    assert env.envs_per_block == 12 and env.fused_logic
    env.reset()
    bench.settle(env, bench.Stepper(env, "noisy", seed, None, None, 0), bench.EPISODE_STEPS, True, env.device)
    state0, obs0 = env.get_state(), env.obs.clone()
    k0 = bench.EPISODE_STEPS
    twins = []
    for _ in range(2):
        t = BatchedCarEnv(E, C, path, device="cuda:0")
        assert t.envs_per_block == 12 and t.fused_logic and t.rollout_streams == 4, (t.envs_per_block, t.rollout_streams)
        t.set_state(state0)
        t.obs.copy_(obs0)
        twins.append(t)
    ot, rt, cft, eft = twins[0].rollout(3, K, seed=seed, step0=k0, auto_reset=True, trajectory=True,
                                         obs_trajectory=True)
    stc = bench.Stepper(twins[1], "noisy", seed, None, None, 50)
    assert stc.R == 50
    stc.run(k0, K)
    assert torch.equal(ot[0], obs0)
    # A and the oracle
    blob = state0.cpu().numpy()
    gobs = obs0.cpu().numpy().reshape(E, C, 38)
    pick = [int(x) for x in np.linspace(0, E - 1, 64)]
    orc = OracleEnv(path, len(pick), C)
    rows = inject_gpu_state(orc, blob, E, C, pick)
    drv = NoisyRuleDriver(len(pick) * C, seed, ids=[e * C + c for e in pick for c in range(C)])
    drv.tb = rows[:, 0].copy()
    drv.steer, drv.last, drv.lim = (rows[:, j].astype(np.float32) for j in (1, 2, 3))
    pk = torch.tensor(pick, device=env.device)
    oo = np.ascontiguousarray(gobs[pick])
    contact = resets = 0
    for i, k in enumerate(range(k0, k0 + K)):
        ha = drv.actions(oo, k)
        env.step_driven(3, seed=seed, step=k, auto_reset=True)
        # the whole batch: per-step path == the timed schedule's records of this step
        assert torch.equal(env.obs, ot[i + 1]), f"step {k}: per-step obs != sharded rollout's record " \
            f"{torch.nonzero(env.obs != ot[i + 1])[:5].tolist()}"
        assert torch.equal(env.reward, rt[i]), f"step {k}: reward != sharded rollout's"
        assert torch.equal(env.car_flags, cft[i]), f"step {k}: car flags != sharded rollout's"
        assert torch.equal(env.env_flags, eft[i]), f"step {k}: env flags != sharded rollout's"
        # the 64 envs: per-step path == oracle
        oo, orw, ocf, oef = orc.step(ha.reshape(len(pick), C, 2))
        done = (oef[:, 0] != 0) | (oef[:, 1] != 0)
        if done.any():
            for e in np.nonzero(done)[0]:
                orc.reset(int(e))
            oo = orc.outputs()[0]
            resets += int(done.sum())
        gr = env.reward.view(E, C)[pk].cpu().numpy()
        gcf = env.car_flags.view(E, C)[pk].cpu().numpy()
        gef = env.env_flags[pk].cpu().numpy()
        go = env.obs.view(E, C, 38)[pk].cpu().numpy()
        assert np.array_equal(gr, orw), f"step {k}: reward mismatch at {np.argwhere(gr != orw)[:5].tolist()}"
        assert np.array_equal(gcf & 5, ocf & 5), f"step {k}: disabled / collision flags"
        assert np.array_equal((gef & 3) != 0, done), f"step {k}: done flags"
        assert np.array_equal(((gef >> 4) & 7)[done], oef[done, 2]), f"step {k}: termination reasons"
        bad = np.argwhere(go != oo)
        assert len(bad) == 0, f"step {k}: obs mismatch at {bad[:5].tolist()}"
        contact += int(((gcf & 4) != 0).sum())
    sa = env.get_state()
    for name, t in (("rollout, one 150-step call with records", twins[0]), ("rollout, bench.Stepper's 3 x 50", twins[1])):
        assert torch.equal(t.get_state(), sa), f"final state arena differs: {name}"
        assert torch.equal(t.obs, env.obs), f"final obs differ: {name}"
    assert int(((eft & 8) != 0).sum()) > 0, "no auto-reset inside the window"
    orc.close()
    for x in [env] + twins:
        x.close()
    assert contact > 0

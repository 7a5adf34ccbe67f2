"""BASELINE configs at their own car counts and horizons (round-3 verdict item 1).

* cfg5 -- mixed batch of all 8 .track files at 10 cars per env: every env equals the oracle on its own track,
  every step, under the bench's closed-loop noisy driver with staggered masked resets and in-launch auto-reset
  (reference: the per-env track of src/car_env.py:243-303 / 375-394).
* the bench workload over a whole episode: 16 x 10 daytona, noisy driver, >= 10 810 steps, so every env age the
  bench's steady-state window holds (0 .. 10 800 steps, src/car_env.py:1154) is pinned against the oracle.
* cfg3's build-only car-car contact extension at its own shape (talladega x 10 cars, >= 256 envs): impulses
  reported, sharded rollout == per-step path, and switched off it equals a reference-behaviour engine from the same
  state.  No reference counterpart exists (src/constants/physics.py:9: every car has its own b2World), so this row
  is property-tested only.

The GPU runs nascar_step_driven (the device driver inside model_kernel, the bench's per-step path; the sharded
rollout equals it bit for bit, tests/test_gpu_rollout.py); the oracle groups step on host threads.
"""
import os

import numpy as np
import pytest

from golden_replay import TRACKS

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _closed_loop_vs_oracle(env, orc, steps, seed, stagger):
    """Drive `env` (BatchedCarEnv) with device policy 3 and `orc` (OracleGroups) with the host restatement of the
    same driver; compare every step.  stagger: {step: env} masked resets.  Returns event tallies."""
    from drivers import NoisyRuleDriver
    E, C = env.E, env.C
    drv = NoisyRuleDriver(E * C, seed=seed)
    g = env.reset().cpu().numpy()
    oo = orc.reset()[0]
    assert np.array_equal(g, oo), "reset obs"
    t = dict(contact=0, disabled=0, resets=0, laps=0, reasons=set(), max_age=0)
    age = np.zeros(E, np.int64)
    for k in range(steps):
        if k in stagger:
            e = stagger[k]
            m = torch.zeros(E, dtype=torch.uint8, device=env.device)
            m[e] = 1
            env.reset(m)
            orc.reset([e])
            oo = orc.outputs()[0]
            age[e] = 0
        env.step_driven(3, seed=seed, step=k, auto_reset=True)
        oo, orw, ocf, oef = orc.step(drv.actions(oo, k))
        gr, gcf, gef = env.reward.cpu().numpy(), env.car_flags.cpu().numpy(), env.env_flags.cpu().numpy()
        assert np.array_equal(gr, orw), f"step {k}: reward mismatch at {np.argwhere(gr != orw)[:5].tolist()}"
        assert np.array_equal(gcf & 1, ocf & 1), f"step {k}: disabled flags"
        done = (oef[:, 0] != 0) | (oef[:, 1] != 0)
        assert np.array_equal((gef & 3) != 0, done), f"step {k}: done flags"
        assert np.array_equal(((gef >> 4) & 7)[done], oef[done, 2]), f"step {k}: termination reasons"
        age += 1
        if done.any():
            t["reasons"] |= set(oef[done, 2].tolist())
            t["max_age"] = max(t["max_age"], int(age[done].max()))
            orc.reset(np.nonzero(done)[0])
            oo = orc.outputs()[0]
            t["resets"] += int(done.sum())
            age[done] = 0
        go = env.obs.cpu().numpy()
        bad = np.argwhere(go != oo)
        assert len(bad) == 0, f"step {k}: obs mismatch at {bad[:5].tolist()} gpu {go[tuple(bad[0])]} oracle {oo[tuple(bad[0])]}"
        t["contact"] += int(((gcf & 4) != 0).sum())
        t["disabled"] += int(((gcf & 2) != 0).sum())
        t["laps"] += int(((gcf & 8) != 0).sum())
    t["max_age"] = max(t["max_age"], int(age.max()))
    assert not (env.car_flags.cpu().numpy() & 128).any(), "contact buffer overflow"
    return t


@pytest.mark.timeout(900)
def test_cfg5_mixed_tracks_10_cars_vs_oracle():
    """cfg5 at its car count: 64 envs x 10 cars, env e on track e mod 8 (one launch, per-env track index), noisy
    driver closed loop with staggered resets and in-launch auto-reset, 900 steps; each env == the oracle on its own
    track every step (obs, rewards, disabled / done flags, termination reasons)."""
    from nascargymnasium_amd.batched import BatchedCarEnv
    from oracle_lib import OracleGroups
    tracks = sorted(f for f in os.listdir(TRACKS) if f.endswith(".track"))
    E, C, S = 64, 10, 900
    files = [os.path.join(TRACKS, tracks[e % 8]) for e in range(E)]
    env = BatchedCarEnv(E, C, files, device="cuda:0")
    orc = OracleGroups(files, C)
    stagger = {11 * e: e for e in range(8, E)}        # envs 8.. reset at staggered steps (ages spread)
    t = _closed_loop_vs_oracle(env, orc, S, seed=23, stagger=stagger)
    env.close(); orc.close()
    assert t["contact"] > 0 and t["disabled"] > 0, t


@pytest.mark.timeout(1200)
def test_bench_workload_full_episode_vs_oracle():
    """The bench's steady-state workload over a whole episode: 16 x 10 daytona, noisy driver closed loop, staggered
    resets (env e reset at step 600 e), in-launch auto-reset, 10 830 steps.  Env 0 is never reset by the schedule,
    so unless an earlier termination ends it, it runs to the 10 800-step time limit (src/car_env.py:1154): every
    env age the bench's window holds is compared with the oracle every step."""
    from nascargymnasium_amd.batched import BatchedCarEnv
    from oracle_lib import OracleGroups
    E, C, S = 16, 10, 10830
    path = os.path.join(TRACKS, "daytona.track")
    env = BatchedCarEnv(E, C, path, device="cuda:0")
    orc = OracleGroups([path] * E, C, shards=8)
    stagger = {600 * e: e for e in range(1, E)}
    t = _closed_loop_vs_oracle(env, orc, S, seed=31, stagger=stagger)
    env.close(); orc.close()
    assert t["contact"] > 0 and t["disabled"] > 0 and t["laps"] > 0, t
    assert 4 in t["reasons"] and t["max_age"] >= 10800, t      # an episode ran to the 10 800-step truncation


@pytest.mark.timeout(600)
def test_cfg3_car_contact_at_talladega_10_cars():
    """cfg3's extension at its shape (talladega, 10 cars per env -- a 5-row start grid -- 256 envs): impulses are
    reported, the sharded rollout equals the per-step path bit for bit with contact on, and with contact off again
    the engine equals a reference-behaviour engine started from the same state."""
    from nascargymnasium_amd.batched import BatchedCarEnv
    from nascargymnasium_amd import _lib
    E, C = 256, 10
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

"""GPU tests for the boundary's less common paths: the RCCL obs gather (cfg4 single-learner layout), a
mixed-track launch against the oracle per env (cfg5 shape), and track changes that wait for the env's reset."""
import os
import socket

import numpy as np
import pytest

from golden_replay import TRACKS

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _actions(rng, E, C, k):
    a = rng.uniform(-1, 1, (E, C, 2)).astype(np.float32)
    a[: E // 2, :, 0] = np.abs(a[: E // 2, :, 0])          # half the envs mostly throttle -> wall impacts
    a[:, :, 1] *= 0.5 if k % 50 < 25 else 1.0
    return a


def test_obs_gather_rccl_world1():
    """ObsGather over RCCL (torch.distributed "nccl", world size 1, side stream): per-step records after every
    step, then K-step trajectory records of the sharded rollout (obs_trajectory), bit for bit equal to the env's own
    outputs -- received() read without an explicit wait(), and the previous record's views still intact after the
    next push (double-buffered receive)."""
    import torch.distributed as dist
    from nascargymnasium_amd.batched import BatchedCarEnv
    from nascargymnasium_amd.gather import ObsGather
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        E, C, K = 64, 4, 25
        env = BatchedCarEnv(E, C, os.path.join(TRACKS, "daytona.track"), device="cuda:0")
        g = ObsGather(E, C, env.device)
        env.reset()
        for k in range(40):
            env.launch_step(env.policy_actions(3, seed=1, step=k).clone(), auto_reset=True)
            g.push(env.obs, env.reward, env.car_flags, env.env_flags)
            r = g.received()
            assert torch.equal(r["obs"][0], env.obs) and torch.equal(r["reward"][0], env.reward)
            assert torch.equal(r["car_flags"][0], env.car_flags) and torch.equal(r["env_flags"][0], env.env_flags)
        gt = ObsGather(E, C, env.device, steps=K)
        twin = BatchedCarEnv(E, C, os.path.join(TRACKS, "daytona.track"), device="cuda:0")
        twin.set_state(env.get_state()); twin.obs.copy_(env.obs)
        held, want = None, None
        for j in range(4):
            ot, rew, cf, ef = env.rollout(3, K, seed=1, step0=40 + j * K, trajectory=True, obs_trajectory=True)
            # the obs records equal the per-step path's observations step by step
            for k in range(K):
                twin.step_driven(3, seed=1, step=40 + j * K + k, auto_reset=True)
                assert torch.equal(ot[k + 1], twin.obs) and torch.equal(rew[k], twin.reward), (j, k)
            gt.push(ot[1:], rew, cf, ef)
            if held is not None:
                assert torch.equal(held["obs"][0], want[0]) and torch.equal(held["reward"][0], want[1]), j
            r = gt.received()
            assert torch.equal(r["obs"][0], ot[1:]) and torch.equal(r["reward"][0], rew)
            assert torch.equal(r["car_flags"][0], cf) and torch.equal(r["env_flags"][0], ef)
            held, want = r, (ot[1:].clone(), rew.clone())
        for x in (env, twin):
            x.close()
    finally:
        dist.destroy_process_group()


def test_mixed_tracks_vs_oracle():
    """cfg5 shape: 256 envs, env e on track e mod 8, one launch; every env equals the oracle on its own track
    (obs, rewards, disabled flags, done flags) every step."""
    from nascargymnasium_amd.batched import BatchedCarEnv
    from oracle_lib import OracleEnv
    tracks = sorted(f for f in os.listdir(TRACKS) if f.endswith(".track"))
    E, C, S = 256, 2, 400
    env = BatchedCarEnv(E, C, [os.path.join(TRACKS, tracks[e % 8]) for e in range(E)], device="cuda:0")
    groups = [[e for e in range(E) if e % 8 == t] for t in range(8)]
    orcs = [OracleEnv(os.path.join(TRACKS, tracks[t]), len(groups[t]), C) for t in range(8)]
    g = env.reset().cpu().numpy()
    for t in range(8):
        assert np.array_equal(g[groups[t]], orcs[t].reset()[0]), tracks[t]
    rng = np.random.default_rng(11)
    contacts = 0
    for k in range(S):
        a = _actions(rng, E, C, k)
        env.step(torch.from_numpy(a).cuda(), auto_reset=False)
        go, gr = env.obs.cpu().numpy(), env.reward.cpu().numpy()
        gcf, gef = env.car_flags.cpu().numpy(), env.env_flags.cpu().numpy()
        contacts += int((gcf & 4).astype(bool).sum())
        for t in range(8):
            oo, orw, ocf, oef = orcs[t].step(a[groups[t]])
            assert np.array_equal(go[groups[t]], oo), (k, tracks[t])
            assert np.array_equal(gr[groups[t]], orw), (k, tracks[t])
            assert np.array_equal(gcf[groups[t]] & 1, ocf & 1), (k, tracks[t])
            assert np.array_equal(gef[groups[t]] & 3 != 0, (oef[:, 0] != 0) | (oef[:, 1] != 0)), (k, tracks[t])
    assert contacts > 0
    env.close()


def test_track_change_waits_for_reset():
    """nascar_set_env_tracks takes effect at the env's next reset: until then the env keeps stepping on its old
    track (its contacts hold that track's wall indices), the reset builds fresh worlds on the new one, and
    auto-reset afterwards stays on it.  talladega (732 walls) -> martinsville (fewer walls)."""
    from nascargymnasium_amd.batched import BatchedCarEnv
    E, C = 12, 3
    tal, mar = os.path.join(TRACKS, "talladega.track"), os.path.join(TRACKS, "martinsville.track")
    env = BatchedCarEnv(E, C, tal, device="cuda:0")
    twin = BatchedCarEnv(E, C, tal, device="cuda:0")
    fresh = BatchedCarEnv(E, C, mar, device="cuda:0")
    env.reset(); twin.reset()
    rng = np.random.default_rng(3)
    for k in range(400):    # drive into the walls: contact lists fill up
        a = torch.from_numpy(_actions(rng, E, C, k)).cuda()
        env.step(a); twin.step(a)
    assert int(env.info_tensor()[..., env_field("n_contacts")].sum()) > 0
    env.set_env_tracks([mar] * E)
    for k in range(100):    # no reset yet: still talladega
        a = torch.from_numpy(_actions(rng, E, C, k)).cuda()
        assert torch.equal(env.step(a, auto_reset=True)[0], twin.step(a, auto_reset=True)[0]), k
    o = env.reset().clone()
    assert torch.equal(o, fresh.reset())
    for k in range(700):    # idle half the time -> stuck disables -> auto-resets on the new track
        a = torch.from_numpy(_actions(rng, E, C, k) * (k % 200 < 100)).cuda()
        assert torch.equal(env.step(a, auto_reset=True)[0], fresh.step(a, auto_reset=True)[0]), k
    for x in (env, twin, fresh):
        x.close()


def env_field(name):
    from nascargymnasium_amd import _lib
    return _lib.INFO_FIELDS.index(name)


def test_car_contact_extension():
    """Build-only extension (no reference counterpart): with car-car contact on, cars start on a staggered grid,
    closing overlapping cars exchange impulses (total momentum of the pair conserved, impulse reported), the
    rollout path equals the per-step path, and switching it off restores reference behaviour exactly."""
    from nascargymnasium_amd import _lib
    from nascargymnasium_amd.batched import BatchedCarEnv
    E, C = 64, 4
    F = _lib.INFO_INDEX
    env = BatchedCarEnv(E, C, os.path.join(TRACKS, "daytona.track"), device="cuda:0")
    env.set_car_contact(True)
    env.reset()
    inf = env.info_tensor().cpu().numpy()
    xy = inf[0, :, [F["x"], F["y"]]].T
    assert len({tuple(p) for p in xy.round(3).tolist()}) == C          # staggered, not stacked
    # the second row (cars 2, 3) drives into the rear of the first (cars 0, 1, idle): full throttle
    a = torch.zeros(E, C, 2, device="cuda")
    a[:, 2:, 0] = 1.0
    hits = 0
    for k in range(400):
        env.step(a)
        hits += int(((env.car_flags & 4) != 0).sum())
    assert hits > 0, "no car-car impulse reported"
    # rollout == per-step with the extension on
    b = BatchedCarEnv(E, C, os.path.join(TRACKS, "daytona.track"), device="cuda:0")
    b.set_car_contact(True)
    b.set_state(env.get_state()); b.obs.copy_(env.obs)
    for k in range(60):
        env.launch_step(env.policy_actions(3, seed=2, step=k).clone(), auto_reset=True)
    b.rollout(3, 60, seed=2, step0=0, auto_reset=True)
    assert torch.equal(env.obs, b.obs) and torch.equal(env.get_state(), b.get_state())
    # off again: identical to a reference-behaviour engine from the same state
    env.set_car_contact(False); b.set_car_contact(False)
    ref = BatchedCarEnv(E, C, os.path.join(TRACKS, "daytona.track"), device="cuda:0")
    ref.set_state(env.get_state()); ref.obs.copy_(env.obs)
    for k in range(50):
        x = torch.rand(E, C, 2, device="cuda") * 2 - 1
        assert torch.equal(env.step(x)[0], ref.step(x)[0])
    for x in (env, b, ref):
        x.close()


def test_car_contact_rear_end():
    """Car 2 (second row) rams idle car 0 ahead of it: the impulse is reported on both and pushes car 0 forward."""
    from nascargymnasium_amd.batched import BatchedCarEnv
    from nascargymnasium_amd import _lib
    env = BatchedCarEnv(1, 3, os.path.join(TRACKS, "daytona.track"), device="cuda:0")
    env.set_car_contact(True)
    env.reset()
    F = _lib.INFO_INDEX
    a = torch.tensor([[[0.0, 0.0], [0.0, 0.0], [1.0, 0.0]]], device="cuda")
    seen = False
    for k in range(300):
        env.step(a)
        if int(env.car_flags[0, 0]) & 4 and int(env.car_flags[0, 2]) & 4:
            seen = True
            break
    assert seen, "car 2 never reached car 0"
    inf = env.info_tensor().cpu().numpy()[0]
    assert inf[0, F["vx"]] > 0.5 and abs(inf[1, F["vx"]]) < 1e-3      # car 0 pushed, car 1 untouched
    env.close()


def test_car_contact_impulses_conserve_momentum():
    """The car-car extension's solver (b2CollidePolygons manifolds, b2ContactSolver sequential impulses with friction
    and angular terms, restitution 0.1 / friction 0.7 mixed as Box2D mixes two car fixtures): from the state just before
    car 2 (steering slightly) first runs into car 0, one step with the extension on and one with it off differ only by
    the car-car impulses, so the velocity changes must conserve linear momentum and angular momentum about the origin
    (equal and opposite impulses at one contact point), spin the cars (an off-centre hit: angular response), and the
    impulse is reported on both cars."""
    from gpu_state import decode
    from nascargymnasium_amd.batched import BatchedCarEnv
    E, C = 1, 3
    path = os.path.join(TRACKS, "daytona.track")
    env = BatchedCarEnv(E, C, path, device="cuda:0")
    env.set_car_contact(True)
    env.reset()
    a = torch.tensor([[[0.0, 0.0], [0.0, 0.0], [1.0, 0.08]]], device="cuda")
    prev = None
    for k in range(300):
        prev = (env.get_state().clone(), env.obs.clone())
        env.step(a)
        if int(env.car_flags[0, 0]) & 4 and int(env.car_flags[0, 2]) & 4:
            break
    else:
        raise AssertionError("car 2 never reached car 0")
    outs = []
    for on in (True, False):
        t = BatchedCarEnv(E, C, path, device="cuda:0")
        t.set_car_contact(on)
        t.set_state(prev[0]); t.obs.copy_(prev[1])
        t.step(a)
        outs.append((decode(t.get_state().cpu().numpy(), E * C), t.car_flags.cpu().numpy()[0].copy()))
        t.close()
    (on, flags_on), (off, flags_off) = outs
    m, I = 1500.0, 1500.0 * (5.042 ** 2 + 1.996 ** 2) * 0.5 / 12.0     # the car body's mass and inertia (CAR_I_F)
    dvx, dvy, dw = (on[f].astype(np.float64) - off[f] for f in ("vx", "vy", "w"))
    cx, cy = off["xpx"].astype(np.float64), off["xpy"].astype(np.float64)
    p = m * np.hypot(dvx, dvy).max()
    assert p > 100.0, "no car-car impulse"
    assert abs(m * dvx.sum()) < 1e-3 * p and abs(m * dvy.sum()) < 1e-3 * p       # linear momentum
    L = (I * dw + m * (cx * dvy - cy * dvx)).sum()                                 # angular momentum about (0, 0)
    assert abs(L) < 1e-3 * p * (1.0 + np.hypot(cx, cy).max())
    assert np.abs(dw).max() > 1e-4, "an off-centre hit must spin the cars (angular response)"
    assert abs(dvx[1]) == 0.0 and abs(dvy[1]) == 0.0                               # car 1 untouched
    assert flags_on[0] & 4 and flags_on[2] & 4 and not flags_off[0] & 4   # the impulse reported on both cars
    env.close()


def test_full_size_batch_independence_and_determinism():
    """BASELINE's full single-GPU shape (8192 envs x 10 cars, daytona) through size-independent properties:
    (1) every env of the full batch evolves exactly as the same env in a 16-env batch fed the same actions
    (no cross-env interference, block map / grouping correct at full size); (2) the full batch is
    deterministic: the same 300 steps from the same state give the same state bit for bit."""
    from nascargymnasium_amd.batched import BatchedCarEnv
    E, C, K = 8192, 10, 300
    g = torch.Generator(device="cuda:0").manual_seed(2024)
    acts = torch.rand((K, E, C, 2), generator=g, device="cuda:0") * 2 - 1
    acts[:, :, :, 0] = acts[:, :, :, 0].abs()       # mostly throttle: cars reach the walls
    full = BatchedCarEnv(E, C, os.path.join(TRACKS, "daytona.track"), device="cuda:0")
    full.reset()
    snap = full.get_state().clone()
    sub_idx = torch.tensor([0, 1, 11, 12, 13, 127, 1000, 2047, 2048, 4095, 4096, 5000, 6143, 8000, 8190, 8191],
                           device="cuda:0")
    sub = BatchedCarEnv(len(sub_idx), C, os.path.join(TRACKS, "daytona.track"), device="cuda:0")
    sub.reset()
    contacts = 0
    for k in range(K):
        full.step(acts[k], auto_reset=True)
        sub.step(acts[k, sub_idx].contiguous(), auto_reset=True)
        assert torch.equal(full.obs[sub_idx], sub.obs), k
        assert torch.equal(full.reward[sub_idx], sub.reward) and torch.equal(full.env_flags[sub_idx], sub.env_flags), k
        contacts += int(((full.car_flags & 4) != 0).sum())
    end = full.get_state().clone()
    full.set_state(snap)
    full.reset()
    full.set_state(snap)
    for k in range(K):
        full.step(acts[k], auto_reset=True)
    assert torch.equal(full.get_state(), end)
    assert contacts > 0
    full.close(); sub.close()


def test_envs_per_block_switch_mid_run():
    """nascar_set_envs_per_block may change the workgroup layout between launches: an engine whose layout changes
    every 100 steps (12 -> 5 -> 1 -> automatic) stays bit-identical to one at a fixed layout, per step and in its
    final state; out-of-range layouts are rejected."""
    from nascargymnasium_amd.batched import BatchedCarEnv
    E, C = 60, 10
    path = os.path.join(TRACKS, "daytona.track")
    a = BatchedCarEnv(E, C, path, device="cuda:0", envs_per_block=12)
    b = BatchedCarEnv(E, C, path, device="cuda:0", envs_per_block=3)
    with pytest.raises(RuntimeError):
        a.set_envs_per_block(13)          # 13 x 10 cars > 128 lanes
    with pytest.raises(RuntimeError):
        a.set_envs_per_block(-1)
    assert a.envs_per_block == 12
    a.reset(); b.reset()
    for k in range(400):
        if k % 100 == 0 and k:
            a.set_envs_per_block({1: 5, 2: 1, 3: 0}[k // 100])
        a.step_driven(3, seed=9, step=k, auto_reset=True)
        b.step_driven(3, seed=9, step=k, auto_reset=True)
        assert torch.equal(a.obs, b.obs) and torch.equal(a.reward, b.reward), k
        assert torch.equal(a.env_flags, b.env_flags), k
    assert a.envs_per_block == 1     # automatic for 60 envs: spread to one env per workgroup
    a.rollout(3, 100, seed=9, step0=400); b.rollout(3, 100, seed=9, step0=400)
    assert torch.equal(a.obs, b.obs) and torch.equal(a.get_state(), b.get_state())
    a.close(); b.close()


def test_fused_model_logic_kernel_identical():
    """nascar_set_fused_logic: the model + logic step as one launch (each workgroup runs its envs' logic when its own
    cars' physics is done) gives the two-launch path's results bit for bit -- per step with terminal observations,
    through the sharded rollout, and with the car-contact extension on (its pass sits between the two phases)."""
    from nascargymnasium_amd.batched import BatchedCarEnv
    E, C = 48, 10
    path = os.path.join(TRACKS, "daytona.track")
    a = BatchedCarEnv(E, C, path, device="cuda:0", envs_per_block=12)
    b = BatchedCarEnv(E, C, path, device="cuda:0", envs_per_block=12)
    assert b.fused_logic       # the default
    a.set_fused_logic(False)   # model_kernel + logic_kernel
    b.set_fused_logic(True)
    a.reset(); b.reset()
    for k in range(600):
        if k == 400:
            a.set_car_contact(True); b.set_car_contact(True)
        a.step_driven(3, seed=3, step=k, auto_reset=True, terminal_obs=True)
        b.step_driven(3, seed=3, step=k, auto_reset=True, terminal_obs=True)
        assert torch.equal(a.obs, b.obs) and torch.equal(a.reward, b.reward), k
        assert torch.equal(a.car_flags, b.car_flags) and torch.equal(a.env_flags, b.env_flags), k
        assert torch.equal(a.terminal_obs, b.terminal_obs), k
    ra = a.rollout(3, 100, seed=3, step0=600, trajectory=True)
    rb = b.rollout(3, 100, seed=3, step0=600, trajectory=True)
    for x, y in zip(ra, rb):
        assert torch.equal(x, y)
    assert torch.equal(a.get_state(), b.get_state())
    a.close(); b.close()


def test_oracle_continues_from_gpu_mid_episode_state():
    """State injection: 48 x 10 daytona cars driven by the device noisy rule driver for 2 000 steps on the GPU alone
    (bench layout, 12 envs per workgroup; env e reset at step 40 e, so the envs are at different points of their
    episodes), then the GPU state -- every per-car field, contact record, listener entry, acceleration ring, env
    word and the driver's own state -- is loaded into the CPU oracle (oracle_lib.inject_gpu_state), and the two
    continue together for 400 steps: obs, rewards, flags and terminations equal every step.  Parity from a state
    the oracle did not produce itself (the bench's CPU baseline starts from such a state too)."""
    from nascargymnasium_amd.batched import BatchedCarEnv
    from drivers import NoisyRuleDriver
    from oracle_lib import OracleEnv, inject_gpu_state
    E, C, S, K, seed = 48, 10, 2000, 400, 11
    path = os.path.join(TRACKS, "daytona.track")
    env = BatchedCarEnv(E, C, path, device="cuda:0", envs_per_block=12)
    env.reset()
    for k in range(S):
        if k % 40 == 0 and 0 < k // 40 < E:
            m = torch.zeros(E, dtype=torch.uint8, device=env.device)
            m[k // 40] = 1
            env.reset(m)
        env.step_driven(3, seed=seed, step=k, auto_reset=True)
    blob = env.get_state().cpu().numpy()
    oo = env.obs.cpu().numpy().reshape(E, C, 38).copy()
    orc = OracleEnv(path, E, C)
    rows = inject_gpu_state(orc, blob, E, C, list(range(E)))
    drv = NoisyRuleDriver(E * C, seed=seed)
    drv.tb = rows[:, 0].copy()
    drv.steer, drv.last, drv.lim = (rows[:, j].astype(np.float32) for j in (1, 2, 3))
    contact = 0
    for k in range(S, S + K):
        ha = drv.actions(oo, k)
        env.step_driven(3, seed=seed, step=k, auto_reset=True)
        oo, orw, ocf, oef = orc.step(ha)
        done = (oef[:, 0] != 0) | (oef[:, 1] != 0)
        if done.any():
            for e in np.nonzero(done)[0]:
                orc.reset(int(e))
            oo = orc.outputs()[0]
        gr, gcf, gef = env.reward.cpu().numpy(), env.car_flags.cpu().numpy(), env.env_flags.cpu().numpy()
        assert np.array_equal(gr, orw), f"step {k}: reward mismatch at {np.argwhere(gr != orw)[:5].tolist()}"
        assert np.array_equal(gcf & 5, ocf & 5), f"step {k}: disabled / collision flags"
        assert np.array_equal((gef & 3) != 0, done), f"step {k}: done flags"
        go = env.obs.cpu().numpy()
        bad = np.argwhere(go != oo)
        assert len(bad) == 0, f"step {k}: obs mismatch at {bad[:5].tolist()} gpu {go[tuple(bad[0])]} oracle {oo[tuple(bad[0])]}"
        contact += int(((gcf & 4) != 0).sum())
    orc.close(); env.close()
    assert contact > 0

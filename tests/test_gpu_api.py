"""The Gymnasium CarEnv / SB3-style VecCarEnv host API over the HIP engine, checked
against the reference's golden traces (tests/golden) and the engine itself."""
import os

import numpy as np
import pytest

from golden_replay import TRACKS, load, start_kwargs

pytestmark = pytest.mark.gpu


def _replay_carenv(name, steps=None):
    from nascargymnasium_amd import CarEnv
    d = load(name)
    C = int(d["C"])
    disc = bool(d.get("discrete", False))
    env = CarEnv(track_file=os.path.join(TRACKS, str(d["track"])), num_cars=C, reset_on_lap=bool(d["reset_on_lap"]),
                 discrete_action_space=disc, **start_kwargs(d))
    obs, info = env.reset(seed=0)
    want0 = d["obs0"][0] if C == 1 else d["obs0"]
    assert obs.shape == ((38,) if C == 1 else (C, 38)) and obs.dtype == np.float32
    assert np.array_equal(obs, want0)
    assert info["simulation_time"] == 0.0 and len(info["cars"]) == C
    keep = set(d["obs_steps"].tolist()) if "obs_steps" in d else None
    n = len(d["actions"]) if steps is None else steps
    j = 0
    for k in range(n):
        if d["reset"][k]:
            obs, info = env.reset()
            if keep is None or k in keep:
                j += 1
            continue
        a = d["actions"][k]
        if disc:
            a = a.astype(np.int64)          # what MultiDiscrete.sample() / a policy hands over
            obs, rew, term, trunc, info = env.step(int(a[0]) if C == 1 else a)
        else:
            obs, rew, term, trunc, info = env.step(a[0] if C == 1 else a)
        if C == 1:
            assert isinstance(rew, np.float32) and obs.shape == (38,)
        assert bool(term) == bool(d["terminated"][k]) and bool(trunc) == bool(d["truncated"][k]), k
        assert np.array_equal(np.atleast_1d(rew), d["rewards"][k]), k
        if keep is None or k in keep:
            assert np.array_equal(obs.reshape(C, 38), d["obs"][j]), k
            if "perf" in d:   # Car.validate_performance and CarPhysics.get_performance_stats, exact
                for i, c in enumerate(info["cars"]):
                    p = c["performance"]
                    got = [p["current_max_speed"], p["estimated_0_100_time"], float(p["performance_valid"])]
                    assert got == d["perf"][j, i].tolist(), (k, i, got, d["perf"][j, i])
                    ph = info["physics"][i]
                    got = [float(ph["physics_steps"]), ph["simulation_time"], ph["average_fps"], float(ph["bodies_in_world"])]
                    assert got == d["physics"][j, i].tolist(), (k, i, got, d["physics"][j, i])
            j += 1
        lap = [c["lap_timing"]["lap_count"] for c in info["cars"]]
        assert lap == d["info"][k, :, 0].astype(int).tolist(), k
        assert [c["disabled"] for c in info["cars"]] == (d["info"][k, :, 8] != 0).tolist(), k
        assert env.disabled_cars == {i for i in range(C) if d["info"][k, i, 8] != 0}
        if k == 5:   # SubprocVecEnv workers pickle every step's info
            import pickle
            assert pickle.loads(pickle.dumps(info)) == info
    env.close()


@pytest.mark.parametrize("name", ["daytona_mixed", "daytona_crash", "martinsville_lap", "nascar2_seam",
                                  "nascar_banked_discrete", "michigan_discrete1", "talladega_10car",
                                  "daytona_low_reward", "nascar_start_pose", "daytona_start_reversed"])
def test_carenv_golden(name):
    _replay_carenv(name)


def test_carenv_errors_and_discrete():
    from nascargymnasium_amd import CarEnv
    env = CarEnv(track_file="daytona", discrete_action_space=True, num_cars=2)
    with pytest.raises(RuntimeError):
        env.step(np.array([1, 1]))
    env.reset()
    with pytest.raises(AssertionError):
        env.step(np.array([1, 7]))
    for k in range(30):
        obs, rew, term, trunc, info = env.step(np.array([1, 4]))
    assert obs.shape == (2, 38) and rew.shape == (2,)
    assert info["cars"][0]["car_speed_ms"] > 0
    env.close()
    env = CarEnv(track_file="daytona")
    env.reset()
    with pytest.raises(AssertionError):
        env.step(np.array([0.5, 0.5], np.float64))     # gymnasium Box: float64 is not castable to float32
    env.close()


def test_random_track_mode_recreates_worlds():
    from nascargymnasium_amd import CarEnv
    from nascargymnasium_amd.batched import BatchedCarEnv
    env = CarEnv(track_file=None, num_cars=1)
    seen = set()
    for s in range(4):
        obs, info = env.reset(seed=s)
        seen.add(os.path.basename(env.track_file))
        fresh = BatchedCarEnv(1, 1, env.track_file, device="cuda:0")
        fo = fresh.reset()[0, 0].cpu().numpy()
        assert np.array_equal(obs, fo), env.track_file      # reset after a track change == a fresh env
        for k in range(40):
            o, r, t, tr, _ = env.step(np.array([0.8, 0.1], np.float32))
            fo = fresh.step(__import__("torch").tensor([[[0.8, 0.1]]], device="cuda:0"))[0][0, 0].cpu().numpy()
            assert np.array_equal(o, fo)
        fresh.close()
    assert len(seen) >= 2
    env.close()


def test_vec_env_auto_reset_matches_engine():
    import torch
    from nascargymnasium_amd import VecCarEnv
    from nascargymnasium_amd.batched import BatchedCarEnv
    E = 16
    venv = VecCarEnv(E, "martinsville", num_cars=1)
    ref = BatchedCarEnv(E, 1, "martinsville", device="cuda:0")
    o = venv.reset()
    assert o.shape == (E, 38) and np.array_equal(o, ref.reset()[:, 0].cpu().numpy())
    rng = np.random.default_rng(3)
    episodes = 0
    for k in range(800):
        a = rng.uniform(-1, 1, (E, 2)).astype(np.float32)
        a[:, 0] = np.where(np.arange(E) % 2 == 0, 0.0, a[:, 0])     # idle half -> stuck -> episode ends
        obs, rew, done, infos = venv.step(a)
        robs, rrew, rterm, rtrunc = ref.step(torch.from_numpy(a).view(E, 1, 2).cuda(), auto_reset=True, terminal_obs=True)
        assert np.array_equal(obs, robs[:, 0].cpu().numpy()) and np.array_equal(rew, rrew[:, 0].cpu().numpy())
        rdone = (rterm | rtrunc).cpu().numpy()
        assert np.array_equal(done, rdone)
        for e in np.nonzero(done)[0]:
            episodes += 1
            assert np.array_equal(infos[e]["terminal_observation"], ref.terminal_obs[e, 0].cpu().numpy())
            assert infos[e]["episode"]["l"] > 0
    assert episodes > 0
    venv.close(); ref.close()


def test_race_tables_match_oracle():
    """CarEnv._calculate_race_positions / _get_best_lap_times_data (src/car_env.py:1485-1638) from the device
    info vector equal the reference formulas evaluated on the CPU oracle's per-car state."""
    import numpy as np
    from nascargymnasium_amd import CarEnv
    from oracle_lib import OracleEnv
    C = 4
    path = os.path.join(TRACKS, "martinsville.track")
    env = CarEnv(track_file=path, num_cars=C)
    orc = OracleEnv(path, 1, C)
    env.reset(seed=0)
    orc.reset()
    L = env.track.get_total_track_length()
    rng = np.random.default_rng(3)
    checked = 0
    for k in range(900):
        a = rng.uniform(-1, 1, (C, 2)).astype(np.float32)
        a[:, 0] = np.abs(a[:, 0]) * 0.8 + 0.2
        a[:, 1] *= 0.3
        env.step(a)
        orc.step(a[None])
        if k % 60 != 59:
            continue
        rows = [orc.car_info(i) for i in range(C)]
        exp = []
        for i, r in enumerate(rows):
            if r["disabled"]:
                continue
            laps, prog = int(r["lap_count"]), r["progress"]
            virt = laps + 1 if (r["is_timing"] and prog < L * 0.15 and r["lap_distance"] > L * 0.8) else laps
            exp.append((i, f"Car {i}", virt * L + prog, virt, prog))
        exp.sort(key=lambda x: (x[3], x[4]), reverse=True)
        assert env._calculate_race_positions() == exp, f"step {k}"
        best = sorted([(i, f"Car {i}", r["best_lap"]) for i, r in enumerate(rows)
                       if not r["disabled"] and r["best_lap"] == r["best_lap"] and r["best_lap"] >= 0], key=lambda x: x[2])
        got = env._get_best_lap_times_data()
        assert [g[:2] for g in got] == [b[:2] for b in best]
        checked += 1
    assert checked == 15
    env.close()


def test_vec_env_random_tracks_vs_oracle():
    """VecCarEnv(track_file=None): every env draws a new track per episode from its own seeded generator (never
    the one it just drove, src/car_env.py:243-303); each episode equals the oracle run fresh on that env's track
    with the same actions -- obs, rewards, dones and terminal observations."""
    from nascargymnasium_amd import VecCarEnv
    from oracle_lib import OracleEnv
    E = 6
    venv = VecCarEnv(E, None, num_cars=1, seed=123)
    obs = venv.reset()
    orcs = [OracleEnv(venv.env_tracks[e], 1, 1) for e in range(E)]
    for e in range(E):
        assert np.array_equal(obs[e], orcs[e].reset()[0][0, 0])
    rng = np.random.default_rng(8)
    n_done = 0
    for k in range(1400):
        a = rng.uniform(-1, 1, (E, 2)).astype(np.float32)
        a[:, 0] = np.where(np.arange(E) % 3 == 0, np.abs(a[:, 0]), 0.0)   # most envs idle -> stuck -> episode ends
        obs, rew, done, infos = venv.step(a)
        for e in range(E):
            oo, orw, ocf, oef = orcs[e].step(a[e].reshape(1, 1, 2))
            assert np.array_equal(rew[e], orw[0, 0]), (k, e)
            odone = bool(oef[0, 0] or oef[0, 1])
            assert bool(done[e]) == odone, (k, e)
            if odone:
                n_done += 1
                assert np.array_equal(infos[e]["terminal_observation"], oo[0, 0]), (k, e)
                assert venv.episode_tracks[e][-1] != venv.episode_tracks[e][-2]
                orcs[e] = OracleEnv(venv.env_tracks[e], 1, 1)          # fresh worlds on the new track
                oo = orcs[e].reset()
            assert np.array_equal(obs[e], oo[0, 0] if not odone else oo[0][0, 0]), (k, e)
    assert n_done >= E
    assert sum(len(set(t)) for t in venv.episode_tracks) > E
    venv.close()


def test_vec_env_tensor_path_has_lazy_infos_and_device_validation():
    import torch
    from nascargymnasium_amd import VecCarEnv
    E = 8
    venv = VecCarEnv(E, "martinsville", num_cars=2, return_tensors=True)
    venv.reset()
    ended = 0
    for k in range(700):
        obs, rew, done, infos = venv.step(torch.zeros(E, 2, 2, device="cuda"))    # idle -> all disabled at ~600
        assert obs.is_cuda and rew.is_cuda and done.is_cuda
        if k % 100 == 99 or bool(done.any()):
            for e in range(E):
                if bool(done[e]):
                    ended += 1
                    assert infos[e]["terminal_observation"].shape == (2, 38)
                    assert infos[e]["episode"]["l"] == k + 1 and infos[e]["termination_reason"] == "all_cars_disabled"
                else:
                    assert infos[e] == {}
    assert ended == E
    venv.step(torch.full((E, 2, 2), 2.0, device="cuda"))       # invalid: reported at the next host read
    with pytest.raises(AssertionError):
        venv.check_actions()
    # bounded: a loop that never reads infos still sees the error within check_every steps (or at reset)
    venv.step(torch.full((E, 2, 2), -3.0, device="cuda"))
    with pytest.raises(AssertionError):
        for _ in range(venv.check_every):
            venv.step(torch.zeros(E, 2, 2, device="cuda"))
    venv.step(torch.full((E, 2, 2), float("nan"), device="cuda"))
    with pytest.raises(AssertionError):
        venv.reset()
    assert venv.get_attr("track_file")[0].endswith("martinsville.track")
    venv.set_attr("foo", 3, indices=[1])
    assert venv.get_attr("foo", indices=[1]) == [3]
    assert venv.env_method("check_quit_requested") == [False] * E
    assert venv.get_images() == [None] * E
    venv.close()

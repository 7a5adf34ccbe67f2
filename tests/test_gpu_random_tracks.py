"""Random-track mode on the device (CarEnv(track_file=None), src/car_env.py:243-303, 331-398; learn/ppo.py:65-78):
each env's track draws, the fresh worlds on the new track and the regrouping of the workgroups by track all happen on
the device (BatchedCarEnv.set_random_tracks).  Every env is compared with an oracle env run fresh on each track the env
is sent to, every step; the device's draws are replayed on the host (_lib.track_draw); the rollout equals the per-step
path with the mode on."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _actions(rng, E, C):
    """a third of the envs drive (throttle >= 0, random steering: wall crashes, impact disables), the rest idle (stuck
    disables after ~10 s): episodes of ~600-1000 steps, so every env switches track a few times"""
    a = rng.uniform(-1, 1, (E, C, 2)).astype(np.float32)
    drive = (np.arange(E) % 3 == 0)[:, None]
    a[..., 0] = np.where(drive, np.abs(a[..., 0]), 0.0)
    return a


def _replay_tracks(seeds, k0, t0, draws, ids):
    """the track sequence the device must have drawn: draw k of env e from its seed and current track"""
    from nascargymnasium_amd import _lib
    cur = np.array(t0, np.int32)
    for k in range(int(np.min(k0)), int(np.max(draws))):
        live = (k0 <= k) & (k < draws)
        cur = np.where(live, _lib.track_draw(seeds, k, cur, ids), cur)
    return cur


@pytest.mark.parametrize("E,C,epb", [(40, 2, 3), (24, 1, 8)])
def test_random_tracks_vs_oracle_every_step(E, C, epb):
    from nascargymnasium_amd import _lib
    from nascargymnasium_amd.batched import BatchedCarEnv
    from nascargymnasium_amd.track import available_tracks
    from oracle_lib import OracleEnv
    tracks = available_tracks()
    eng = BatchedCarEnv(E, C, [tracks[e % len(tracks)] for e in range(E)], device="cuda:0", envs_per_block=epb)
    seeds = np.arange(E, dtype=np.uint64) * 7919 + 11
    eng.set_random_tracks(tracks, seeds)
    ids = eng.random_track_ids
    t_start = np.array([eng._track_id[tracks[e % len(tracks)]] for e in range(E)], np.int32)
    obs = eng.reset().cpu().numpy()                   # every env draws (draw 0) and gets fresh worlds there
    files = eng.env_track_files()
    orcs = [OracleEnv(files[e], 1, C) for e in range(E)]
    for e in range(E):
        assert np.array_equal(obs[e], orcs[e].reset()[0][0]), e
    rng = np.random.default_rng(21)
    switches, seen = 0, set(files)
    for k in range(1500):
        a = _actions(rng, E, C)
        go, gr, term, trunc = eng.step(torch.from_numpy(a).cuda(), auto_reset=True, terminal_obs=True)
        go, gr = go.cpu().numpy(), gr.cpu().numpy()
        ef = eng.env_flags.cpu().numpy()
        tobs = eng.terminal_obs.cpu().numpy()
        done = np.nonzero(ef & 8)[0]
        files_now = eng.env_track_files() if done.size else files
        for e in range(E):
            oo, orw, _, oef = orcs[e].step(a[e][None])
            assert np.array_equal(gr[e], orw[0]), (k, e)
            odone = bool(oef[0, 0] or oef[0, 1])
            assert odone == bool(ef[e] & 8), (k, e)
            if odone:
                assert np.array_equal(tobs[e], oo[0]), (k, e)          # the old track's final observation
                assert files_now[e] != files[e], (k, e)                # never the track it just drove
                switches += 1
                seen.add(files_now[e])
                orcs[e].close()
                orcs[e] = OracleEnv(files_now[e], 1, C)                 # fresh worlds on the new track
                oo = orcs[e].reset()[0]
            assert np.array_equal(go[e], oo[0]), (k, e)
        files = files_now
    assert switches >= E, switches
    assert len(seen) >= 6, seen
    got, draws = eng.env_track_ids()
    assert np.array_equal(got, _replay_tracks(seeds, np.zeros(E, np.int64), t_start, draws, ids))
    for o in orcs:
        o.close()
    eng.close()


def test_random_tracks_rollout_equals_per_step():
    """nascar_rollout with random tracks on (one shard, the switch and the block map after every step) == per-step
    nascar_step_driven with it on, from the same state: per-step records, final obs, state and track assignment"""
    from nascargymnasium_amd.batched import BatchedCarEnv
    from nascargymnasium_amd.track import available_tracks
    tracks = available_tracks()
    E, C, W, K = 96, 4, 3550, 200
    # reset_on_lap: every env terminates at t > 60 s (step 3601) -- all 96 switch track in one step -- and auto-resets
    engs = [BatchedCarEnv(E, C, [tracks[e % 8] for e in range(E)], reset_on_lap=True, device="cuda:0") for _ in range(2)]
    seeds = np.arange(E, dtype=np.uint64) + 5
    for g in engs:
        g.set_random_tracks(tracks, seeds)
        g.reset()
    a, b = engs
    for k in range(W):
        for g in engs:
            g.step_driven(0, seed=9, step=k, auto_reset=True)
    assert torch.equal(a.get_state(), b.get_state())
    R, EF = [], []
    for k in range(K):
        a.step_driven(0, seed=9, step=W + k, auto_reset=True)
        R.append(a.reward.clone()); EF.append(a.env_flags.clone())
    obs_b, Rb, CFb, EFb = b.rollout(0, K, seed=9, step0=W, auto_reset=True, trajectory=True)
    torch.cuda.synchronize()
    n_reset = 0
    for k in range(K):
        assert torch.equal(R[k], Rb[k]) and torch.equal(EF[k], EFb[k]), k
        n_reset += int(((EF[k] & 8) != 0).sum())
    assert n_reset >= E
    assert torch.equal(a.obs, obs_b)
    assert torch.equal(a.get_state(), b.get_state())
    assert np.array_equal(a.env_track_ids()[0], b.env_track_ids()[0])
    for g in engs:
        g.close()


def _expected_map(ids, ntracks, epb):
    """the layout block_map_kernel must build: tracks in id order, each track's envs in ascending order in whole
    workgroups of epb envs (the last one padded with -1)"""
    bt, be = [], []
    for t in range(ntracks):
        envs = np.nonzero(ids == t)[0].tolist()
        for i in range(0, len(envs), epb):
            bt.append(t)
            chunk = envs[i:i + epb]
            be.append(chunk + [-1] * (epb - len(chunk)))
    return np.array(bt, np.int32), np.array(be, np.int32).reshape(-1, epb)


@pytest.mark.parametrize("extra_tracks", [0, 2])     # 8 tracks: the packed-count fast path; 10: the generic path
def test_device_block_map_matches_host_layout(tmp_path, extra_tracks):
    """block_map_kernel (random-track mode's workgroup layout, rebuilt on the device) against the layout computed here
    from the device's env -> track map, after the initial build, after masked resets (draws) and after steps whose
    auto-resets switch tracks: the used workgroups exactly as expected, the rest empty (track -1)."""
    from nascargymnasium_amd.batched import BatchedCarEnv
    from nascargymnasium_amd.track import available_tracks
    tracks = available_tracks()
    for k in range(extra_tracks):     # copies of bundled tracks under other names: more tracks than the fast path takes
        p = tmp_path / f"extra{k}.track"
        p.write_text(open(tracks[k]).read())
        tracks.append(str(p))
    E, C, epb = 301, 1, 5
    eng = BatchedCarEnv(E, C, [tracks[e % len(tracks)] for e in range(E)], device="cuda:0", envs_per_block=epb)
    eng.set_random_tracks(tracks, np.arange(E, dtype=np.uint64) * 31 + 7)
    rng = np.random.default_rng(3)
    checks = 0

    def check():
        ids, _ = eng.env_track_ids()
        bt, be = eng.block_map()
        want_t, want_e = _expected_map(ids, len(tracks), epb)
        assert len(bt) == (E + epb - 1) // epb + len(tracks)
        n = len(want_t)
        assert np.array_equal(bt[:n], want_t) and (bt[n:] == -1).all()
        assert np.array_equal(be[:n], want_e)
        return 1
    checks += check()
    eng.reset()
    checks += check()
    for k in range(6):
        mask = torch.from_numpy((rng.random(E) < 0.3).astype(np.uint8)).cuda()
        eng.reset(mask)
        checks += check()
    a = torch.zeros(E, C, 2, device="cuda")          # idle: every env stuck-disabled at ~600 steps, auto-resets, switches
    for k in range(700):
        eng.step(a, auto_reset=True)
    checks += check()
    assert checks == 9
    eng.close()

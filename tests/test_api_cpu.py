"""Host-side API semantics on CPU (no GPU needed): the restated gymnasium 0.29.1 spaces,
BaseEnv action conversions (src/base_env.py:201-252) and CarEnv constructor errors
(src/car_env.py:103-129, src/track_generator.py:318-319)."""
import numpy as np
import pytest

from nascargymnasium_amd.car_env import BaseEnv, CarEnv, _format_time
from nascargymnasium_amd.spaces import Box, Discrete, MultiDiscrete


def test_box_contains_semantics():
    sp = BaseEnv(num_cars=1).action_space
    assert isinstance(sp, Box) and sp.shape == (2,)
    assert sp.contains(np.array([0.5, -1.0], np.float32))
    assert sp.contains([0.5, -1.0])                              # list -> asarray(float32)
    assert not sp.contains(np.array([0.5, -1.0], np.float64))    # np.can_cast(float64, float32) is False
    assert not sp.contains(np.array([1.5, 0.0], np.float32))     # out of bounds
    assert not sp.contains(np.array([[0.5, 0.0]], np.float32))   # shape must match exactly
    assert not sp.contains("abc")
    multi = BaseEnv(num_cars=3).action_space
    assert multi.shape == (3, 2) and multi.contains(np.zeros((3, 2), np.float32))
    assert not multi.contains(np.zeros((2,), np.float32))
    obs = BaseEnv(num_cars=1).observation_space
    assert obs.shape == (38,) and obs.low[4] == 0.0 and obs.low[5] == -1.0 and obs.low[20] == -1.0


def test_discrete_contains_semantics():
    sp = BaseEnv(discrete_action_space=True, num_cars=1).action_space
    assert isinstance(sp, Discrete)
    assert sp.contains(0) and sp.contains(4) and sp.contains(np.int64(3)) and sp.contains(np.array(2))
    assert not sp.contains(5) and not sp.contains(-1) and not sp.contains(1.0) and not sp.contains(np.array([1]))
    md = BaseEnv(discrete_action_space=True, num_cars=4).action_space
    assert isinstance(md, MultiDiscrete)
    assert md.contains([0, 1, 2, 4]) and md.contains(np.array([4, 4, 4, 4]))
    assert not md.contains([0, 1, 2, 5]) and not md.contains([0, 1, 2])


def test_action_conversions():
    conv = BaseEnv._convert_to_internal_action
    assert conv([0.7, -0.2]) == [0.7, 0.0, -0.2]
    assert conv([-0.4, 0.3]) == [0.0, 0.4, 0.3]
    d2c = BaseEnv._discrete_to_continuous
    assert [d2c(a) for a in range(5)] == [[0.0, 0.0], [1.0, 0.0], [-1.0, 0.0], [0.0, -1.0], [0.0, 1.0]]
    with pytest.raises(ValueError):
        d2c(7)


def test_carenv_constructor_errors():
    with pytest.raises(ValueError):
        CarEnv(track_file="daytona", num_cars=0)
    with pytest.raises(ValueError):
        CarEnv(track_file="daytona", num_cars=11)
    with pytest.raises(ValueError):
        CarEnv(track_file="daytona", num_cars=2, car_names=["a"])
    with pytest.raises(FileNotFoundError):
        CarEnv(track_file="/nonexistent/track.track")
    with pytest.raises(NotImplementedError):
        CarEnv(track_file="daytona", render_mode="human")


def test_carenv_needs_device():
    """The product path fails loudly without a HIP device (no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        CarEnv(track_file="daytona")


def test_format_time():
    assert _format_time(None) == "--:--.---" and _format_time(-1.0) == "--:--.---"
    assert _format_time(83.4567) == " 1:23.457"


def test_sb3_actor_loader(tmp_path):
    """policy.load_sb3_actor reads an SB3 zip with zipfile + torch.load(weights_only=True)."""
    import io
    import zipfile
    import torch
    from nascargymnasium_amd.policy import ACTOR_KEYS, load_sb3_actor, random_actor
    w = random_actor(3)
    sd = {k: torch.from_numpy(v) for k, v in w.items()}
    sd["critic.qf0.0.weight"] = torch.zeros(4, 4)
    buf = io.BytesIO()
    torch.save(sd, buf)
    p = tmp_path / "sac.zip"
    with zipfile.ZipFile(p, "w") as z:
        z.writestr("policy.pth", buf.getvalue())
        z.writestr("data", "{}")
    got = load_sb3_actor(str(p))
    assert set(got) == set(ACTOR_KEYS)
    for k in ACTOR_KEYS:
        assert np.array_equal(got[k], w[k])
    bad = tmp_path / "bad.zip"
    with zipfile.ZipFile(bad, "w") as z:
        buf2 = io.BytesIO(); torch.save({"x": torch.zeros(1)}, buf2); z.writestr("policy.pth", buf2.getvalue())
    with pytest.raises(ValueError):
        load_sb3_actor(str(bad))


def test_sac_fixture_consistent():
    """tests/golden/sac_1235_actor.npz: its actions are the float32 SB3 predict() restatement of its weights,
    and (where the reference is present) its weights are sac_1235.zip's actor tensors."""
    import os
    import sys
    import numpy as np
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "oracle"))
    from gen_actor_fixture import sb3_predict_fp32
    from nascargymnasium_amd.policy import ACTOR_KEYS, load_sb3_actor
    d = np.load(os.path.join(root, "tests", "golden", "sac_1235_actor.npz"))
    w = {k: d[k.replace(".", "__")] for k in ACTOR_KEYS}
    assert np.array_equal(sb3_predict_fp32(w, d["obs"]), d["actions_fp32"])
    z = "/root/reference/game/control/models/sac_1235.zip"
    if os.path.exists(z):
        ref = load_sb3_actor(z)
        assert all(np.array_equal(ref[k], w[k]) for k in ACTOR_KEYS)


def _shell_env(E=4, C=2):
    """a BatchedCarEnv shell (no device handle) to exercise host-side argument checks on CPU"""
    import torch
    from nascargymnasium_amd.batched import BatchedCarEnv
    env = BatchedCarEnv.__new__(BatchedCarEnv)
    env.E, env.C, env.N, env.device = E, C, E * C, torch.device("cpu")
    return env


def test_rollout_out_buffers_rejected():
    """rollout(trajectory=True, out=...) hands raw pointers to the kernels, which write record k at
    ptr + k * E * C (or k * E): every malformed buffer is refused before any launch."""
    import torch
    env = _shell_env()
    E, C, K = env.E, env.C, 5
    good = (torch.zeros(K, E, C), torch.zeros(K, E, C, dtype=torch.uint8), torch.zeros(K, E, dtype=torch.uint8))
    bad = {
        "dtype": (torch.zeros(K, E, C, dtype=torch.float64), good[1], good[2]),
        "flags dtype": (good[0], torch.zeros(K, E, C, dtype=torch.int32), good[2]),
        "inner shape": (torch.zeros(K, E, C + 1), good[1], good[2]),
        "env shape": (good[0], good[1], torch.zeros(K, E, C, dtype=torch.uint8)),
        "rank": (torch.zeros(K, E * C), good[1], good[2]),
        "too few": (torch.zeros(K - 1, E, C), good[1], good[2]),
        "strided": (torch.zeros(K, C, E).transpose(1, 2), good[1], good[2]),
        "not a tensor": (np.zeros((K, E, C), np.float32), good[1], good[2]),
        "arity": good[:2],
    }
    for what, out in bad.items():
        with pytest.raises(ValueError):
            env.rollout(3, K, trajectory=True, out=out)
        assert what
    with pytest.raises(ValueError, match="trajectory=True"):
        env.rollout(3, K, trajectory=False, out=good)
    with pytest.raises(ValueError, match="trajectory=True"):
        env.rollout(3, K, obs_trajectory=True)
    obs_ok = torch.zeros(K + 1, E, C, 38)
    with pytest.raises(ValueError, match="fewer than"):      # obs records: steps + 1 (record 0 = the entry obs)
        env.rollout(3, K, trajectory=True, obs_trajectory=True, out=(torch.zeros(K, E, C, 38),) + good)
    with pytest.raises(ValueError):                          # obs missing from out
        env.rollout(3, K, trajectory=True, obs_trajectory=True, out=good)
    with pytest.raises(ValueError):
        env.rollout(3, K, trajectory=True, obs_trajectory=True, out=(obs_ok[..., :37],) + good)
    if torch.cuda.is_available():
        return
    env.device = torch.device("cuda", 0)          # right shapes, wrong device
    with pytest.raises(ValueError, match="on cpu"):
        env.rollout(3, K, trajectory=True, out=good)


def test_lazy_infos_fill_on_any_access():
    """VecCarEnv's lazy info list (return_tensors=True) behaves as the eager list for every list operation."""
    import pickle
    from nascargymnasium_amd.vec_env import _LazyInfos
    want = [{"a": 1}, {}, {"episode": {"r": 1.0}}]
    mk = lambda: _LazyInfos(lambda: [dict(x) for x in want])   # noqa: E731
    assert repr(mk()) == repr(want) and str(mk()) == str(want)
    assert mk() == want and not (mk() != want)
    assert mk().copy() == want and {"a": 1} in mk()
    assert mk().index({}) == 1 and mk().count({}) == 1
    assert list(reversed(mk())) == want[::-1] and mk() + [] == want and [] + list(mk()) == want
    assert len(mk()) == 3 and mk()[2] == want[2] and list(mk()) == want
    x = mk(); x.append({"b": 2}); assert len(x) == 4 and x[3] == {"b": 2}
    assert pickle.loads(pickle.dumps(mk())) == want
    assert bool(mk()) and mk() * 2 == want * 2
    # two lazy operands: the other one is filled too (list's C methods read its storage directly)
    assert mk() == mk() and not (mk() != mk()) and want == mk()
    assert mk() + mk() == want * 2
    y = mk(); y.extend(mk()); assert y == want * 2
    z = mk(); z += mk(); assert z == want * 2

"""GPU parity of the 16 distance sensors on arbitrary car poses (nascar_debug_sensors).

The step kernels only ever see poses the physics produces; here the sensor hand-off is set directly to
random poses -- on the track, in the walls' band, far outside every beam-list cell (fallback path), with
wound-up angles and exact multiples of pi/8 -- on all 8 tracks, and both device sensor implementations (beam
lists, the step's default, and wall groups) must agree bit-exactly with each other and, for EVERY pose (~31 k
poses, ~500 k rays), with the CPU oracle's brute-force b2PolygonShape::RayCast over every wall
(oracle/b2_oracle.c ob_raycast), evaluated as DistanceSensor.get_sensor_distances does
(src/distance_sensor.py:95-103, src/car_env.py:946).
"""
import ctypes
import math
import os
import subprocess
import sys
import zlib

import numpy as np
import pytest

from golden_replay import TRACKS

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _poses(rng, walls, n):
    """n poses: 60 % within 12 m of a wall, 25 % uniform over the walls' extent +- 60 m, 15 % far away."""
    cx, cy = walls[:, 0], walls[:, 1]
    lo, hi = np.array([cx.min(), cy.min()]) - 60, np.array([cx.max(), cy.max()]) + 60
    k1, k2 = int(n * 0.6), int(n * 0.25)
    j = rng.integers(0, len(walls), k1)
    near = np.stack([cx[j], cy[j]], 1) + rng.normal(0, 6.0, (k1, 2))
    box = rng.uniform(lo, hi, (k2, 2))
    far = rng.uniform(lo - 400, hi + 400, (n - k1 - k2, 2))
    xy = np.concatenate([near, box, far]).astype(np.float32)
    ang = rng.uniform(-3.2, 3.2, n)
    ang[::7] = rng.uniform(-60, 60, len(ang[::7]))                       # wound-up body angles
    ang[::11] = rng.integers(-16, 16, len(ang[::11])) * (math.pi / 8)    # rays exactly axis-aligned
    return np.concatenate([xy, ang.astype(np.float32)[:, None]], 1)


def _device_sensors(env, poses, impl):
    from nascargymnasium_amd import _lib
    p = torch.from_numpy(np.ascontiguousarray(poses)).cuda()
    obs = torch.full((env.N, 38), -7.0, dtype=torch.float32, device="cuda")
    _lib.check(env.L.nascar_debug_sensors(env.h, ctypes.c_void_p(p.data_ptr()), ctypes.c_void_p(obs.data_ptr()),
                                          impl, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    torch.cuda.synchronize()
    return obs.cpu().numpy()


def _oracle_sensors_all(path, poses, threads=8):
    """DistanceSensor values of every pose with the oracle's brute-force ray cast over all walls (or_sensors:
    Python-float ray ends as the reference computes them), host threads over pose chunks"""
    from concurrent.futures import ThreadPoolExecutor
    from oracle_lib import OracleEnv
    out = np.zeros((len(poses), 16), np.float32)
    fp = ctypes.POINTER(ctypes.c_float)

    def run(lo, hi):
        orc = OracleEnv(path, 1, 1)
        orc.L.or_sensors.argtypes = [ctypes.c_void_p, fp, ctypes.c_int, fp]
        p = np.ascontiguousarray(poses[lo:hi], np.float32)
        o = np.zeros((hi - lo, 16), np.float32)
        orc.L.or_sensors(orc.h, p.ctypes.data_as(fp), hi - lo, o.ctypes.data_as(fp))
        out[lo:hi] = o
        orc.close()
    bounds = np.linspace(0, len(poses), threads + 1).astype(int)
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(lambda k: run(bounds[k], bounds[k + 1]), range(threads)))
    return out


def _oracle_sensors(orc, pose):
    """one pose, ray by ray through or_raycast, as DistanceSensor.get_sensor_distances (Python floats)"""
    x, y, a = (float(v) for v in pose)
    out = np.zeros(16, np.float32)
    for i in range(16):
        sa = -math.radians(i * 22.5) + a
        x2, y2 = np.float32(x + math.cos(sa) * 250.0), np.float32(y + math.sin(sa) * 250.0)
        fr = orc.L.or_raycast(orc.h, x, y, float(x2), float(y2))
        d32 = np.float32(float(fr) * 250.0 if fr >= 0.0 else 250.0)
        out[i] = min(max(np.float32(d32 / np.float32(250.0)), np.float32(0.0)), np.float32(1.0))
    return out


@pytest.mark.parametrize("track,E,C", [("daytona.track", 2048, 10), ("martinsville.track", 1024, 8),
                                       ("talladega.track", 512, 4), ("nascar_banked.track", 512, 3),
                                       ("michigan.track", 512, 4), ("nascar.track", 512, 4),
                                       ("nascar2.track", 512, 4), ("trioval.track", 512, 4)])
def test_sensors_on_random_poses(track, E, C):
    """every pose: beam-list kernel (4 and 16 lanes per car) == wall-group kernel == the oracle's brute-force
    cast, bit for bit"""
    _check_sensors(os.path.join(TRACKS, track), E, C, zlib.crc32(track.encode()))


def _check_sensors(path, E, C, seed):
    from nascargymnasium_amd.batched import BatchedCarEnv
    from nascargymnasium_amd.track import build_walls, load_track
    from oracle_lib import OracleEnv
    rng = np.random.default_rng(seed)
    walls = build_walls(load_track(path))
    env = BatchedCarEnv(E, C, path, device="cuda:0")
    poses = _poses(rng, walls, E * C)
    env.set_sensor_lanes(4)
    beams = _device_sensors(env, poses, 1)
    env.set_sensor_lanes(16)
    beams16 = _device_sensors(env, poses, 1)
    groups = _device_sensors(env, poses, 0)
    env.close()
    bad = np.argwhere(beams16.view(np.uint32) != beams.view(np.uint32))
    assert len(bad) == 0, f"16 vs 4 lanes per car differ at {bad[:5].tolist()}"
    assert (beams[:, :22] == -7.0).all(), "sensor launch wrote outside obs[22:38]"
    bad = np.argwhere(beams[:, 22:].view(np.uint32) != groups[:, 22:].view(np.uint32))
    assert len(bad) == 0, f"beam vs group sensors differ at {bad[:5].tolist()}"
    assert (beams[:, 22:] < 1.0).any() and (beams[:, 22:] == 1.0).any()
    ref = _oracle_sensors_all(path, poses)
    bad = np.argwhere(beams[:, 22:].view(np.uint32) != ref.view(np.uint32))
    assert len(bad) == 0, f"{len(bad)} rays differ from the oracle, first at car {bad[0, 0]} pose {poses[bad[0, 0]].tolist()}: " \
                          f"gpu {beams[bad[0, 0], 22:]} oracle {ref[bad[0, 0]]}"
    orc = OracleEnv(path, 1, 1)      # the batched oracle equals the per-ray Python path on a sample
    for n in rng.integers(0, E * C, 40):
        assert np.array_equal(_oracle_sensors(orc, poses[n]).view(np.uint32), ref[n].view(np.uint32)), n
    orc.close()


def test_beam_cell_size_changes_nothing():
    """nascar_set_beam_cell: beam lists built at 2 m and 4 m cells give the 1 m default's sensor values on every pose
    (the lists are conservative at any cell size); a 2 m build takes a quarter of the 1 m build's list memory."""
    from nascargymnasium_amd.batched import BatchedCarEnv
    from nascargymnasium_amd.track import build_walls, load_track
    path = os.path.join(TRACKS, "daytona.track")
    rng = np.random.default_rng(77)
    poses = _poses(rng, build_walls(load_track(path)), 4096)
    out = {}
    for cell in (None, 2.0, 4.0):
        env = BatchedCarEnv(1024, 4, path, device="cuda:0", beam_cell=cell)
        out[cell] = _device_sensors(env, poses, 1)
        env.close()
    for cell in (2.0, 4.0):
        bad = np.argwhere(out[cell].view(np.uint32) != out[None].view(np.uint32))
        assert len(bad) == 0, f"{cell} m cells differ from 1 m at {bad[:5].tolist()}"
    with pytest.raises(RuntimeError):
        BatchedCarEnv(4, 1, path, device="cuda:0", beam_cell=0.1)


# six 180-degree curves of 180 chords per side: 2 160 + walls, a sensor wall image of ~70 KB (beyond 64 KiB of LDS)
MANY_WALLS_TRACK = """WIDTH 16
GRID
STARTLINE
STRAIGHT 15
LEFT 180 400
LEFT 180 400
RIGHT 180 250
RIGHT 180 250
LEFT 180 300
LEFT 180 300
STRAIGHT 40
"""


def test_track_with_many_walls(tmp_path):
    """A custom track with more walls than the bundled ones (2 000+, whose sensor wall image exceeds 64 KiB of LDS)
    loads; its sensors equal the oracle's brute-force cast on random poses, and 300 closed-loop steps equal the
    oracle every step (per-step path), with the sharded and the fused rollout equal to the per-step path."""
    from nascargymnasium_amd.batched import BatchedCarEnv
    from nascargymnasium_amd.track import build_walls, load_track
    from closed_loop import closed_loop_vs_oracle
    from oracle_lib import OracleGroups
    path = str(tmp_path / "many_walls.track")
    with open(path, "w") as f:
        f.write(MANY_WALLS_TRACK)
    nwall = len(build_walls(load_track(path)))
    assert nwall > 2048, nwall
    _check_sensors(path, 256, 4, 1234)
    E, C, S = 8, 3, 300
    env = BatchedCarEnv(E, C, path, device="cuda:0")
    orc = OracleGroups([path] * E, C, shards=4)
    t = closed_loop_vs_oracle([env], orc, S, seed=5, stagger={})
    orc.close()
    assert t["contact"] >= 0
    outs = []
    for streams in (4, 0):   # sharded rollout / fused rollout kernel (its LDS holds the wall image too)
        b = BatchedCarEnv(E, C, path, device="cuda:0")
        b.set_rollout_streams(streams)
        b.reset()
        b.rollout(3, seed=5, step0=0, steps=S)
        outs.append(b.obs.cpu().numpy().copy())
        b.close()
    ref = BatchedCarEnv(E, C, path, device="cuda:0")
    ref.reset()
    for k in range(S):
        ref.step_driven(3, seed=5, step=k, auto_reset=True)
    ro = ref.obs.cpu().numpy()
    ref.close()
    env.close()
    for o in outs:
        assert np.array_equal(o.view(np.uint32), ro.view(np.uint32))


def test_sensor_workgroup_sizes_identical():
    """ray_sensor_kernel at 16 lanes per car in 64- and 128-thread workgroups (the default; walls read from the global
    image) and 256-, 512- and 1024-thread workgroups (walls staged in LDS; nascar_set_sensor_block), and at 4 lanes
    per car: the same sensor values on every pose, bit for bit."""
    from nascargymnasium_amd.batched import BatchedCarEnv
    from nascargymnasium_amd.track import build_walls, load_track
    path = os.path.join(TRACKS, "martinsville.track")
    rng = np.random.default_rng(4242)
    poses = _poses(rng, build_walls(load_track(path)), 480 * 10)
    out = {}
    for rb in ("64", "128", "256", "512", "1024"):
        env = BatchedCarEnv(480, 10, path, device="cuda:0", envs_per_block=12)   # 120 cars per step workgroup
        env.set_sensor_block(int(rb))
        out[rb] = _device_sensors(env, poses, 1)
        if rb == "128":
            env.set_sensor_lanes(4)
            out["lpc4"] = _device_sensors(env, poses, 1)
        env.close()
    for k in ("64", "256", "512", "1024", "lpc4"):
        bad = np.argwhere(out[k].view(np.uint32) != out["128"].view(np.uint32))
        assert len(bad) == 0, f"{k} differs from 128-thread workgroups at {bad[:5].tolist()}"


def test_coop_walk_round_cap_fallback(tmp_path):
    """ray_walk_coop hands a ray still walking after RAY_COOP_ROUNDS rounds to its own lane (ray_walk_rest); no bundled
    list gets there in the product build (1024 rounds).  The tools build with a cap of 1 round
    (tools/build/libnascar_coop1.so, __graft_entry__.build) sends every walk longer than the heads plus one round down
    that branch; on martinsville (the tightest track: the longest walks) and on the many-walls track its sensor values
    equal the product build's and the wall-group kernel's on every pose, bit for bit (16 lanes per car)."""
    from nascargymnasium_amd.batched import BatchedCarEnv
    from nascargymnasium_amd.track import build_walls, load_track
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    variant = os.path.join(root, "tools", "build", "libnascar_coop1.so")
    assert os.path.exists(variant), "build() builds the RAY_COOP_ROUNDS=1 test variant"
    many = str(tmp_path / "many_walls.track")
    with open(many, "w") as f:
        f.write(MANY_WALLS_TRACK)
    for path, E, C in ((os.path.join(TRACKS, "martinsville.track"), 512, 8), (many, 256, 4)):
        rng = np.random.default_rng(99)
        poses = _poses(rng, build_walls(load_track(path)), E * C)
        env = BatchedCarEnv(E, C, path, device="cuda:0")
        product = _device_sensors(env, poses, 1)
        groups = _device_sensors(env, poses, 0)
        env.close()
        pf, of = str(tmp_path / "poses.npy"), str(tmp_path / "out.npy")
        np.save(pf, poses)
        child = os.path.join(root, "tests", "sensor_child.py")
        r = subprocess.run([sys.executable, child, path, str(E), str(C), pf, of], capture_output=True, text=True,
                           timeout=300, env=dict(os.environ, NASCAR_LIB=variant))
        assert r.returncode == 0, r.stderr[-2000:]
        capped = np.load(of)
        bad = np.argwhere(capped.view(np.uint32) != product.view(np.uint32))
        assert len(bad) == 0, f"{os.path.basename(path)}: capped walk differs at {bad[:5].tolist()}"
        assert np.array_equal(capped[:, 22:].view(np.uint32), groups[:, 22:].view(np.uint32))

"""Host logic of bench.py and the host restatement of the device action sources (no GPU)."""
import os

import numpy as np
import pytest

import bench
from drivers import M64, mix32, noisy_mask, uniform_actions, RuleDriver


def _mix32_py(x):
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return (x ^ (x >> 31)) >> 32


def test_mix32_matches_python_ints():
    xs = np.array([0, 1, 2**63 + 5, M64, 0x123456789ABCDEF], np.uint64)
    assert [int(v) for v in mix32(xs)] == [_mix32_py(int(v)) for v in xs]


def test_uniform_and_noise_rates():
    u = uniform_actions(200000, 3, 17)
    assert u.dtype == np.float32 and u.min() >= -1 and u.max() < 1
    assert abs(u.mean()) < 0.01
    m = noisy_mask(200000, 3, 17)
    assert abs(m.mean() - 0.15) < 0.005


def test_rule_driver_steers_toward_open_side():
    d = RuleDriver(2)
    obs = np.zeros((2, 38), np.float32)
    obs[:, 22] = 1.0
    obs[0, 23], obs[0, 37] = 0.2, 0.8     # left close, right open -> steer right (+)
    obs[1, 23], obs[1, 37] = 0.8, 0.2
    a = d(obs)
    assert a[0, 1] > 0 and a[1, 1] < 0
    assert np.isclose(a[0, 1], np.float32(1) - np.float32(0.2) / np.float32(0.8))


def test_stagger_schedule_spreads_env_ages():
    at = bench.stagger_schedule(8192, 10800)
    age = 10800 - at
    assert at.min() >= 1 and at.max() <= 10800
    assert age.min() == 0 and age.max() < 10800
    h = np.histogram(age, bins=10, range=(0, 10800))[0]
    assert h.min() > 0.9 * h.mean()
    assert np.abs(np.diff(age[:120])).mean() > 1000    # a workgroup's envs are not at the same point of their lap
    short = bench.stagger_schedule(100, 600)          # settle shorter than an episode: old envs never reset
    assert (short == -1).sum() == 100 - ((600 * 100 + 10799) // 10800)


def test_throughput_is_whole_job():
    assert bench.throughput(8, 8192, 10, 200, 0.02) == 8 * 8192 * 10 * 200 / 0.02


def _bench(args, env=None, timeout=240):
    import os
    import subprocess
    import sys
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(bench.ROOT, "bench.py")] + args, cwd=bench.ROOT, env=e,
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("gather", [False, True])
def test_gpus_n_runs_main_on_n_ranks(gather):
    """`bench.py --gpus 2 --plumbing` outside torchrun starts 2 ranks itself (torch.distributed.run child) and runs
    bench.main() unchanged on the CPU stand-in engine (PlumbingEngine) over gloo: the settle, the warm-up, the
    barrier-bracketed timed window, the statistics and kernel passes, the per-step pass, the secondary pass and every
    collective main() issues (gather_all, the reduce_max / reduce_sum calls, the barriers), with and without the
    --gather path (ObsGather of the rollout's trajectory records to rank 0).  Rank 0's line has n_gpus = world = 2,
    the MAX over the ranks' timings, the whole-job value from it, and both ranks issued the same collectives in the
    same order."""
    import json
    K, E, C = 6, 16, 10
    args = ["--gpus", "2", "--plumbing", "--steps", str(K), "--warmup", "2", "--envs", str(E), "--cars", str(C),
            "--settle", "12"] + (["--gather"] if gather else [])
    r = _bench(args)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 only
    d = json.loads(lines[0])
    assert d["metric"].startswith("plumbing")
    assert d["n_gpus"] == 2 and d["ranks"]["world_size"] == 2 and d["ranks"]["backend"] == "gloo"
    el = d["ranks"]["elapsed_s"]
    assert len(el) == 2 and max(el) >= K * 2e-3          # rank 1 sleeps 2 ms per step
    assert np.isclose(d["ms_per_step"], max(el) / K * 1e3)
    assert np.isclose(d["value"], 2 * E * C * K / max(el))
    col = d["collectives"]
    assert col["ranks"] == 2 and col["all_ranks_equal"], col
    seq = col["rank0"]
    # timed window (2 barriers) + per-step window (2 barriers), the per-rank gather, the reductions of main()
    assert seq[:4] == ["barrier"] * 4
    assert seq[4:9] == ["all_gather[1]", "all_reduce_max[2]", "all_reduce_max[2]", "all_reduce_max[1]",
                        "all_reduce_sum[7]"], seq
    cache = ["all_gather[1]"] * 3      # the per-rank track-cache statistics (multi-rank runs), after every window
    if gather:
        assert seq[9:] == cache and "uniform_from_reset" not in d
        assert "RCCL gather" in d["config"]["parallelism"]
    else:   # the secondary pass: its own barrier-bracketed window and MAX
        assert seq[9:] == ["barrier", "barrier", "all_reduce_max[1]"] + cache, seq
        assert d["uniform_from_reset"]["ms_per_step"] >= 2.0
    assert set(d["roofline"]["kernel_times_ms"]) == {"model_logic_kernel", "ray_sensor_kernel"}
    assert d["per_step"]["ms_per_step"] >= 2.0
    ws = d["workload_stats"]
    assert ws["window_car_steps"] > 0 and 0 < ws["contact_frac"] < 1


def test_world_size_mismatch_is_an_error():
    """launched as 2 ranks but told --gpus 1 (or the reverse): exit non-zero before any process group forms"""
    r = _bench(["--gpus", "1", "--plumbing", "--steps", "1"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"},
               timeout=60)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def test_host_cores_reports_the_cpu(monkeypatch):
    n, txt = bench.host_cores()
    assert n >= 1 and "affinity" in txt and f"{n} threads used" in txt
    # an OMP_NUM_THREADS set for another reason binds the thread count: the description says so, and
    # NASCAR_CPU_SHARE overrides it
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    monkeypatch.delenv("NASCAR_CPU_SHARE", raising=False)
    n1, txt1 = bench.host_cores()
    aff = len(__import__("os").sched_getaffinity(0))
    assert n1 == 1 and ("binding limit" in txt1) == (aff > 1)
    monkeypatch.setenv("NASCAR_CPU_SHARE", "2")
    n2, txt2 = bench.host_cores()
    assert n2 == min(2, aff) and "NASCAR_CPU_SHARE=2" in txt2


def test_host_driver_global_ids_match_the_device_keys():
    """the host driver of a few picked envs, keyed by the cars' global ids, draws the same noise as those cars in
    the full batch (the device's key uses the global car index n = e * C + c)"""
    from drivers import NoisyRuleDriver
    E, C, step = 300, 10, 12345
    full = uniform_actions(E * C, 5, step)
    fm = noisy_mask(E * C, 5, step)
    pick = [3, 77, 299]
    ids = [e * C + c for e in pick for c in range(C)]
    assert np.array_equal(uniform_actions(len(ids), 5, step, ids), full[ids])
    assert np.array_equal(noisy_mask(len(ids), 5, step, ids), fm[ids])
    d = NoisyRuleDriver(len(ids), 5, ids=ids)
    obs = np.zeros((len(ids), 38), np.float32)
    obs[:, 22] = 1.0
    a = d.actions(obs, step)
    assert np.array_equal(a[fm[ids]], full[ids][fm[ids]])


def test_mixed_multi_rank_track_cache(tmp_path):
    """Multi-rank startup over all 8 tracks (cfg5's batch; verdict r05 item 5): `bench.py --gpus 2 --plumbing --mixed`
    on gloo, both ranks prebuilding the 8 tracks into one on-disk track cache (rotated orders, a lock file per track):
    every track is built exactly once across the ranks and loaded by the other; a second job on the same cache builds
    nothing and each rank's tracks load in a fraction of the build time.  (Coarse 8 m beam cells keep the CPU test
    small; the file format and the locking do not depend on it.)"""
    import json
    cache = str(tmp_path / "tracks")
    args = ["--gpus", "2", "--plumbing", "--mixed", "--beam-cell", "8", "--steps", "2", "--warmup", "1", "--envs", "16",
            "--cars", "2", "--settle", "2", "--no-secondary"]
    runs = []
    for _ in range(2):
        r = _bench(args, env={"NASCAR_TRACK_CACHE": cache})
        assert r.returncode == 0, r.stderr[-3000:]
        runs.append(json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])["track_cache"])
    first, second = runs
    assert first["dir"] == cache
    assert sum(first["built"]) == 8 and sum(first["loaded"]) == 8, first      # each track built once, loaded once
    assert sum(second["built"]) == 0 and second["loaded"] == [8, 8], second
    assert max(second["prebuild_s"]) < 3.0 and max(second["prebuild_s"]) < max(first["prebuild_s"]), (first, second)
    assert len([f for f in os.listdir(cache) if f.endswith(".nbt")]) == 8

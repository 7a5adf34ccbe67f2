"""Per-phase cycle profile of step_kernel (profile build, -DNASCAR_PROFILE).

    python tools/phase_profile.py [--envs E] [--cars C] [--track daytona] [--steps S]

Builds tools/libnascar_prof.so, runs S steps of uniform random driving after a warm-up and prints, per
phase, the mean/max s_memtime cycles per wave, plus the wave start/end spread (s_memrealtime, 100 MHz).
"""
import argparse
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from nascargymnasium_amd import _lib  # noqa: E402

PHASES = ["stage_track+sync", "car_load", "update_physics", "b2_step", "bank/disable/lap+sync_pre",
          "sync1+envpass1+stuck", "car_obs(sensors)", "rewards+sync_pre", "sync2+term+sync3", "obs+state store"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=8192)
    ap.add_argument("--cars", type=int, default=10)
    ap.add_argument("--track", default="daytona")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--no-build", action="store_true")
    ap.add_argument("--lib", default="libnascar_prof.so")
    ap.add_argument("--up", action="store_true", help="library built with -DNASCAR_PROFILE_UP")
    a = ap.parse_args()
    so = os.path.join(ROOT, "tools", a.lib)
    if not a.no_build:
        subprocess.run(["hipcc"] + _lib.HIPCC_FLAGS + ["-DNASCAR_PROFILE", "-o", so,
                        os.path.join(_lib.CSRC, "nascar_kernels.hip")], check=True)
    _lib.LIB_PATH = so
    import torch
    from nascargymnasium_amd.batched import BatchedCarEnv
    from nascargymnasium_amd.track import track_path
    L = _lib.lib()
    L.nascar_debug_profile.argtypes = [ctypes.c_void_p]
    env = BatchedCarEnv(a.envs, a.cars, track_path(a.track), device="cuda:0")
    env.reset()
    g = torch.Generator(device="cuda:0"); g.manual_seed(7)
    for _ in range(a.warmup):
        env.step(torch.rand((a.envs, a.cars, 2), generator=g, device="cuda:0") * 2 - 1, auto_reset=True)
    nwaves = 65536
    buf = torch.zeros(2 * nwaves * 16 + 16, dtype=torch.int64, device="cuda:0")
    L.nascar_debug_profile(ctypes.c_void_p(buf.data_ptr()))
    acc = []
    for _ in range(a.steps):
        acts = torch.rand((a.envs, a.cars, 2), generator=g, device="cuda:0") * 2 - 1
        buf.zero_()
        torch.cuda.synchronize()
        env.launch_step(acts, auto_reset=True)
        torch.cuda.synchronize()
        acc.append(buf[:2 * nwaves * 16].view(2 * nwaves, 16).cpu().numpy().copy())
        cnt = buf[2 * nwaves * 16:].cpu().numpy()
        if cnt[6]:
            print("sensor workgroups %d: per WG items %.1f q1 %.1f q2 %.1f | rays with a hit (any lane) %.1f | active cars %.1f"
                  % (cnt[6], cnt[0] / cnt[6], cnt[1] / cnt[6], cnt[2] / cnt[6], cnt[3] / cnt[6], cnt[5] / cnt[6]))
    L.nascar_debug_profile(ctypes.c_void_p(0))
    sens = []
    for b in acc:
        sb = b[nwaves:]
        sb = sb[(sb[:, 0] != 0) & (sb[:, 6] != 0)].astype(np.float64)
        sens.append(np.diff(sb[:, :7], axis=1))
    acc = [b[:nwaves] for b in acc]
    res = []
    for b in acc:
        b = b[b[:, 10] != 0]
        d = np.diff(b[:, :11].astype(np.float64), axis=1)
        res.append((d, b[:, 14], b[:, 15]))
    d = np.concatenate([r[0] for r in res])
    tot = d.sum(1)
    # b2_step sub-phases: 3 -> 11 collide, 11 -> 12 solve, 12 -> 13 broadphase update, 13 -> 4 solve_toi
    sub = []
    for b in acc:
        b = b[(b[:, 10] != 0) & (b[:, 11] != 0) & (b[:, 12] != 0) & (b[:, 13] != 0)].astype(np.float64)
        sub.append(np.stack([b[:, 11] - b[:, 3], b[:, 12] - b[:, 11], b[:, 13] - b[:, 12], b[:, 4] - b[:, 13]], 1))
    sub = np.concatenate(sub)
    print(f"waves/launch {len(res[0][0])}, mean wave cycles {tot.mean():.0f} (max {tot.max():.0f})")
    for k, name in enumerate(PHASES):
        print(f"  {name:28s} mean {d[:, k].mean():10.0f}  max {d[:, k].max():10.0f}  {100 * d[:, k].mean() / tot.mean():5.1f}%")
    if len(sub):
        names = (["engine force", "brake/drag/rolling + acc history", "weight transfer + tyres", "lateral..end"]
                 if a.up else ["collide", "solve", "sync_fixtures+find_new_contacts", "solve_toi"])
        pre = "update_physics" if a.up else "b2_step"
        if a.up:   # slots: 2 -> 11 -> 12 -> 13 -> 3
            sub = []
            for b in acc:
                b = b[(b[:, 10] != 0) & (b[:, 11] != 0) & (b[:, 12] != 0) & (b[:, 13] != 0)].astype(np.float64)
                sub.append(np.stack([b[:, 11] - b[:, 2], b[:, 12] - b[:, 11], b[:, 13] - b[:, 12], b[:, 3] - b[:, 13]], 1))
            sub = np.concatenate(sub)
        for k, name in enumerate(names):
            print(f"    {pre}/{name:34s} mean {sub[:, k].mean():10.0f}  max {sub[:, k].max():10.0f}")
    sd = np.concatenate(sens)
    if len(sd):
        print(f"sensor_kernel: waves/launch {len(sens[0])}, mean wave cycles {sd.sum(1).mean():.0f}")
        for k, name in enumerate(["setup (walls/groups/pose)", "ray end points (f64 cos/sin)", "barrier", "group/wall cull",
                                  "barrier", "write obs"]):
            print(f"  {name:30s} mean {sd[:, k].mean():10.0f}  max {sd[:, k].max():10.0f}")
    for _, st, en in res[:3]:
        t0 = st.min()
        print(f"  realtime (us): first start 0, last start {(st.max() - t0) / 100:.1f}, "
              f"median end {(np.median(en) - t0) / 100:.1f}, last end {(en.max() - t0) / 100:.1f}")
    env.close()


if __name__ == "__main__":
    main()

"""Replay chosen envs of a saved steady state on their own (profile build), to time one car's Box2D chain without
the wave divergence of its 60-odd neighbours.

    python tools/env_replay.py --load-state /tmp/nascar_ss.pt --lib libprof_x.so [--envs 5,17] [--auto 4]
                               [--steps 3] [--copies 1]

The saved state (bench.py --save-state: arena + obs + step of an E x C engine) is cut down to the chosen envs
(--auto k: the k envs whose cars had the most Box2D contacts at save time), each repeated --copies times, and
loaded into a small engine; the full engine's device driver (policy 3, keyed by the ORIGINAL car indices) gives
the actions, which the small engine steps through nascar_step -- the same car trajectories.  Per step it prints,
for every wave of the small engine, the model_kernel phase cycles (s_memtime stamps of the -DNASCAR_PROFILE build)
and the per-car counters of the Box2D step (TOI events, island sizes and cycles).
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from nascargymnasium_amd import _lib  # noqa: E402

MAXC, N_EI32 = 16, 5
NW = 65536
APROF_BASE = 2 * NW * 16 + 64
LPROF_BASE = APROF_BASE + 4096 * 16
CPROF_BASE = LPROF_BASE + NW * 16


def _a256(x):
    return (x + 255) & ~255


def layout(E, C):
    """byte offsets and sizes of the state arena blocks (nascar_create), per-car or per-env, in order"""
    from gpu_state import F32, F64, I32
    N = E * C
    blocks = [("f32", 4 * len(F32), "field", len(F32), 4), ("f64", 8 * len(F64), "field", len(F64), 8),
              ("i32", 4 * len(I32), "field", len(I32), 4), ("acc", 8 * 20, "field", 20, 8),
              ("ct", 80 * MAXC, "car", 1, 80 * MAXC), ("key", 4 * MAXC, "car", 1, 4 * MAXC),
              ("act_n", 8 * MAXC, "car", 1, 8 * MAXC), ("time", 8, "env", 1, 8), ("ei32", 4 * N_EI32, "envfield", N_EI32, 4),
              ("ctl", 32, "car", 1, 32)]
    out, o = [], 0
    for name, per, kind, nf, item in blocks:
        cnt = E if kind in ("env", "envfield") else N
        out.append((name, o, kind, nf, item, cnt))
        o = _a256(o + per * cnt)
    return out, o


def subset_state(blob, E, C, envs):
    """the arena of an engine holding only `envs` (in that order) of an E x C arena"""
    envs = np.asarray(envs, np.int64)
    cars = (envs[:, None] * C + np.arange(C)[None, :]).reshape(-1)
    src, _ = layout(E, C)
    dst, total = layout(len(envs), C)
    out = np.zeros(total, np.uint8)
    for (name, so, kind, nf, item, scnt), (_, do, _, _, _, dcnt) in zip(src, dst):
        idx = envs if kind in ("env", "envfield") else cars
        if kind in ("field", "envfield"):
            a = blob[so:so + nf * item * scnt].view(np.uint8).reshape(nf, scnt, item)
            out[do:do + nf * item * dcnt] = a[:, idx, :].reshape(-1)
        else:
            a = blob[so:so + item * scnt].reshape(scnt, item)
            out[do:do + item * dcnt] = a[idx].reshape(-1)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--load-state", required=True)
    ap.add_argument("--lib", default="libnascar_prof.so", help="profile build under tools/")
    ap.add_argument("--envs", default=None, help="comma-separated env indices of the saved engine")
    ap.add_argument("--auto", type=int, default=4, help="else: the envs with the most contacts at save time")
    ap.add_argument("--copies", type=int, default=1, help="each chosen env repeated this many times")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--cars", type=int, default=10)
    ap.add_argument("--track", default="daytona")
    a = ap.parse_args()
    _lib.LIB_PATH = os.path.join(ROOT, "tools", a.lib)
    import torch
    from gpu_state import decode
    from nascargymnasium_amd.batched import BatchedCarEnv
    from nascargymnasium_amd.track import track_path
    L = _lib.lib()
    L.nascar_debug_profile.argtypes = [ctypes.c_void_p]
    blobd = torch.load(a.load_state, map_location="cpu", weights_only=True)
    blob, obs0, step0 = blobd["state"].numpy(), blobd["obs"], int(blobd["step"])
    C = a.cars
    E = obs0.shape[0]
    st = decode(blob, E * C)
    if a.envs:
        envs = [int(x) for x in a.envs.split(",")]
    else:
        nct = st["nct"].reshape(E, C).sum(1)
        envs = np.argsort(-nct)[:a.auto].tolist()
    envs = [e for e in envs for _ in range(a.copies)]
    print(f"envs {envs} (contacts per env at save time: {[int(st['nct'].reshape(E, C)[e].sum()) for e in envs]})")
    full = BatchedCarEnv(E, C, track_path(a.track), device="cuda:0")
    full.set_state(blobd["state"].cuda())
    full.obs.copy_(obs0.cuda())
    small = BatchedCarEnv(len(envs), C, track_path(a.track), device="cuda:0", envs_per_block=1)
    small.set_state(torch.from_numpy(subset_state(blob, E, C, envs)).cuda())
    small.obs.copy_(obs0[envs].cuda())
    N = len(envs) * C
    buf = torch.zeros(CPROF_BASE + (1 << 20) * 32 + 65536 * 5, dtype=torch.int64, device="cuda:0")
    idx = torch.tensor(envs, device="cuda:0")
    for s in range(a.steps):
        act = full.policy_actions(3, seed=0, step=step0 + s).clone()
        full.launch_step(act, auto_reset=True)
        buf.zero_()
        L.nascar_debug_profile(ctypes.c_void_p(buf.data_ptr()))
        small.launch_step(act[idx].contiguous(), auto_reset=True)
        torch.cuda.synchronize()
        L.nascar_debug_profile(ctypes.c_void_p(0))
        same = torch.equal(small.obs, full.obs[idx])
        b = buf.cpu().numpy()
        model = b[:NW * 16].reshape(NW, 16)
        cp = b[CPROF_BASE:CPROF_BASE + N * 32].reshape(N, 32)
        print(f"--- step {s}: small engine == full engine on these envs: {same}")
        for w in np.nonzero(model[:, 0])[0]:
            r = model[w].astype(np.int64)
            if not r[5]:
                continue
            print(f"  wave {w}: total {r[5] - r[0]}: stage {r[1] - r[0]}, update_physics {r[3] - r[2]}, b2_step {r[4] - r[3]} "
                  f"(collide {r[11] - r[3]}, solve {r[12] - r[11]}, sync+find {r[13] - r[12]}, toi {r[4] - r[13]}), "
                  f"store {r[5] - r[4]}")
        for i in range(N):
            if cp[i, 1] or cp[i, 26] or cp[i, 4]:
                print(f"    car {i} (env {envs[i // C]} car {i % C}): contacts {cp[i, 1]}, island {cp[i, 26]} solve {cp[i, 25]} "
                      f"cyc; TOI computed {cp[i, 2]} culled {cp[i, 3]} events {cp[i, 4]}; event island solve {cp[i, 11]}, "
                      f"event contact updates {cp[i, 12]}; TOI scans {cp[i, 14]} job rounds {cp[i, 13]} events {cp[i, 15]}")
    full.close(); small.close()


if __name__ == "__main__":
    main()

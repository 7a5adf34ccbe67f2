"""CPU analysis of the ray sensor's beam-list walks on steady-state poses (diagnostic tooling; uses the oracle).

Runs the bench's workload on the oracle (noisy rule driver, staggered resets, auto-reset), samples car poses, and
for every ray rebuilds the (cell, direction bin) list of build_beams (nascar_kernels.hip) with numpy: membership by
the capsule's angular arc seen from the cell disk (+ 2e-3 rad guard), entries sorted by the distance lower bound.
Reports how many list entries each ray walks (entries whose bound lies within the true best hit, from the oracle's
brute-force cast) and how many rays would be settled by sub-bin free-space certificates.

    python tools/beam_walks.py [--track daytona] [--steps 3000] [--every 25] [--sub 8]
"""
import argparse
import ctypes
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
from drivers import NoisyRuleDriver  # noqa: E402
from oracle_lib import OracleGroups, OracleEnv  # noqa: E402

NB, CELL, GUARD = int(os.environ.get("BW_NB", 256)), float(os.environ.get("BW_CELL", 4.0)), 2e-3


def sample_poses(path, E, C, steps, every, seed=3):
    orc = OracleGroups([path] * E, C, shards=8)
    drv = NoisyRuleDriver(E * C, seed=seed)
    oo = orc.reset()[0]
    stagger = {int(steps * e / E): e for e in range(1, E)}
    poses = []
    for k in range(steps):
        if k in stagger:
            orc.reset([stagger[k]]); oo = orc.outputs()[0]
        oo, _, _, ef = orc.step(drv.actions(oo, k))
        done = (ef[:, 0] != 0) | (ef[:, 1] != 0)
        if done.any():
            orc.reset(np.nonzero(done)[0]); oo = orc.outputs()[0]
        if k % every == every - 1 and k > steps // 4:
            for g, (env, m) in enumerate(orc.groups):
                for j in range(len(m)):
                    for c in range(C):
                        inf = env.car_info(j * C + c)
                        poses.append((inf["x"], inf["y"], inf["angle"]))
    orc.close()
    return np.array(poses, np.float64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--track", default="daytona")
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--every", type=int, default=25)
    ap.add_argument("--envs", type=int, default=16)
    ap.add_argument("--sub", type=int, default=8)
    ap.add_argument("--heads", action="store_true", help="head-format study (continuation reads, quantised bounds)")
    a = ap.parse_args()
    from nascargymnasium_amd.track import build_walls, load_track, track_path
    path = track_path(a.track)
    t = load_track(path)
    walls = build_walls(t)
    poses = sample_poses(path, a.envs, 10, a.steps, a.every)
    print(f"{len(poses)} poses")
    # wall segments as build_beams sees them (f32 body values widened)
    orc = OracleEnv(path, 1, 1)
    _, wf = orc.walls()
    px, py, qs, qc, hx, hy = (wf[:, k].astype(np.float64) for k in (0, 1, 5, 6, 3, 4))
    ax, ay, bx, by = px - hx * qc, py - hx * qs, px + hx * qc, py + hx * qs
    rr = hy + 0.1
    rc = CELL * 0.70710678 + 0.05
    hw = max(s.width for s in t.segments) / 2
    ox = min(ax.min(), bx.min()) - (hw + 8 + 2 * CELL)
    oy = min(ay.min(), by.min()) - (hw + 8 + 2 * CELL)
    fp = ctypes.POINTER(ctypes.c_float)
    orc.L.or_sensors.argtypes = [ctypes.c_void_p, fp, ctypes.c_int, fp]
    pf = np.ascontiguousarray(poses, np.float32)
    sens = np.zeros((len(pf), 16), np.float32)
    orc.L.or_sensors(orc.h, pf.ctypes.data_as(fp), len(pf), sens.ctypes.data_as(fp))
    walked, listlen, free_sub, hit = [], [], [], []
    headst = {}
    cache = {}
    for n, (x, y, ang) in enumerate(poses):
        cx, cy = int((np.float32(x) - np.float32(ox)) / CELL), int((np.float32(y) - np.float32(oy)) / CELL)
        xc, yc = ox + (cx + 0.5) * CELL, oy + (cy + 0.5) * CELL
        key = (cx, cy)
        if key not in cache:
            sx, sy = bx - ax, by - ay
            ll = sx * sx + sy * sy
            tt = np.clip(((xc - ax) * sx + (yc - ay) * sy) / ll, 0, 1)
            d = np.hypot(xc - (ax + tt * sx), yc - (ay + tt * sy))
            R = rr + rc
            lb = np.maximum(d - R, 0)
            inside = d <= R * 1.0001 + 1e-3
            aA, aB = np.arctan2(ay - yc, ax - xc), np.arctan2(by - yc, bx - xc)
            dl = (aB - aA + np.pi) % (2 * np.pi) - np.pi
            a0 = np.where(dl >= 0, aA, aB)
            wid = np.arcsin(np.minimum(1, R / np.maximum(d, 1e-9))) + GUARD
            cache[key] = (lb, inside, a0 - wid, np.abs(dl) + 2 * wid, d - R <= 251)
        lb, inside, lo, span, near = cache[key]
        for i in range(16):
            sa = -math.radians(22.5 * i) + ang
            u = (sa / (2 * np.pi)) % 1.0
            binw = 2 * np.pi / NB
            b = int(u * NB)
            # bin membership: the wall's arc [lo, lo + span] intersects bin b
            blo = b * binw
            rel = (blo - lo) % (2 * np.pi)
            member = near & (inside | (span >= 2 * np.pi - binw) | (rel <= span) | ((lo - blo) % (2 * np.pi) < binw))
            best = sens[n, i] * 250.0 if sens[n, i] < 1.0 else 500.0
            L = np.sort(lb[member])
            walked.append(int(np.searchsorted(L, best, side="right")) + (1 if (L > best).any() else 0))
            listlen.append(len(L))
            if a.heads:    # head-format study: continuation reads and casts with exact / quantised bounds
                for qn, Lq in (("cm", np.floor(L * 100) / 100), ("q6", (np.floor(np.minimum(4 * np.sqrt(L), 62)) / 4) ** 2),
                               ("q8", (np.floor(np.minimum(16 * np.sqrt(L), 254)) / 16) ** 2)):
                    k = int(np.searchsorted(Lq, best, side="right"))
                    casts = k + (1 if k < len(Lq) else 0)
                    for H in (2, 3):
                        headst.setdefault((qn, H), []).append((k >= H and len(Lq) > H, casts, max(0, len(Lq) - H)))
            hit.append(sens[n, i] < 1.0)
            # sub-bin certificate: no member's arc intersects the ray's sub-bin (with guard)
            sub = int((u * NB - b) * a.sub)
            slo = blo + sub * binw / a.sub - GUARD
            rel2 = (slo - lo) % (2 * np.pi)
            w = binw / a.sub + 2 * GUARD
            any_sub = (member & (inside | (rel2 <= span) | ((lo - slo) % (2 * np.pi) < w))).any()
            free_sub.append(not any_sub)
    walked, listlen, free_sub, hit = map(np.array, (walked, listlen, free_sub, hit))
    for (qn, H), v in sorted(headst.items()):
        v = np.array(v)
        print(f"heads {qn} H={H}: rays reading a continuation {v[:, 0].mean():.4f}, casts per ray {v[:, 1].mean():.3f}, "
              f"p99 {np.percentile(v[:, 1], 99):.0f}")
    print(f"rays {len(walked)}: hit {hit.mean():.3f}; list length mean {listlen.mean():.1f} p99 {np.percentile(listlen, 99):.0f}")
    print(f"walked entries: mean {walked.mean():.2f}, p50 {np.percentile(walked, 50):.0f}, p90 {np.percentile(walked, 90):.0f}, "
          f"p99 {np.percentile(walked, 99):.0f}, max {walked.max()}")
    for name, m in (("hit", hit), ("no hit", ~hit)):
        print(f"  {name}: rays {m.mean():.3f}, walked mean {walked[m].mean():.2f} p99 {np.percentile(walked[m], 99):.0f}; "
              f"> 7 entries {np.mean(walked[m] > 7):.3f}")
    print(f"no-hit rays settled by a free sub-bin ({a.sub} per bin): {free_sub[~hit].mean():.3f}; hit rays wrongly free: "
          f"{free_sub[hit].sum()}")
    # one ray per lane (16 lanes per car): a wave is 4 consecutive cars' 64 rays and runs as long as its longest walk;
    # a wave-cooperative continuation would cost the longest head walk (<= 3 entries) plus rounds of the wave's
    # continuation entries (4 per continuing ray per round, spread over the 64 lanes)
    nw = len(walked) // 64
    wv = walked[:nw * 64].reshape(nw, 64)
    head = np.minimum(wv, 3).max(1)
    cont = np.maximum(wv - 3, 0)
    rounds = np.zeros(nw)
    left = cont.copy()
    while (left > 0).any():
        jobs = np.minimum(left, 4).sum(1)
        rounds += np.where(jobs > 0, np.ceil(jobs / 64), 0)
        left = np.maximum(left - 4, 0)
    print(f"waves {nw}: longest walk per wave mean {wv.max(1).mean():.2f} p90 {np.percentile(wv.max(1), 90):.0f}; "
          f"cooperative continuation: head {head.mean():.2f} + rounds {rounds.mean():.2f} = {(head + rounds).mean():.2f}")
    lane = walked.reshape(-1, 4, 4).sum(1)    # lane r: rays r, r+4, r+8, r+12 -> per-lane sequential walk total
    print(f"per-lane walk totals: mean {lane.mean():.1f} p99 {np.percentile(lane, 99):.0f} max {lane.max()}")
    w2 = np.where(free_sub & ~hit, 0, walked).reshape(-1, 4, 4).sum(1)
    print(f"  with free sub-bins: mean {w2.mean():.1f} p99 {np.percentile(w2, 99):.0f} max {w2.max()}")


if __name__ == "__main__":
    main()

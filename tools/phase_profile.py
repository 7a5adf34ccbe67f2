"""Per-phase cycle profile of one env step (profile build, -DNASCAR_PROFILE).

    python tools/phase_profile.py [--envs E] [--cars C] [--track daytona] [--steps S] [--up]

Builds tools/libnascar_prof.so (or --lib), runs S steps of uniform random driving after a warm-up and
prints, per kernel and phase, the mean/max s_memtime cycles per wave, plus the realtime spread of
model_kernel waves (s_memrealtime, 100 MHz).  Stamp regions (nascar_device.h): model_kernel PROF
slots 0-5 (+ sub-phases 11-13, realtime 14/15), sensor_kernel PROFS slots 0-6, logic_kernel LPROF
slots 0-8, counters after the sensor region.
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

NW = 65536
APROF_BASE = 2 * NW * 16 + 64
LPROF_BASE = APROF_BASE + 4096 * 16
MODEL = ["stage segments", "car_load_phys", "update_physics", "b2_step", "store body"]
LOGIC = ["stage + load body/logic", "bank/disable/lap + sync", "env pass 1 + stuck", "car_obs",
         "rewards + sync", "env pass 2 (termination) + sync", "reset / pose / state store", "obs rows"]
SENSOR = ["setup (walls/groups/pose)", "ray end points (f64 sincos)", "barrier", "group/wall cull", "barrier",
          "write obs"]


def phases(rows, names, first, title, extra=""):
    rows = rows[(rows[:, first] != 0) & (rows[:, first + len(names)] != 0)].astype(np.float64)
    if not len(rows):
        print(f"{title}: no stamped waves")
        return rows
    d = np.diff(rows[:, first:first + len(names) + 1], axis=1)
    tot = d.sum(1)
    print(f"{title}: waves {len(rows)}, mean wave cycles {tot.mean():.0f} (max {tot.max():.0f}){extra}")
    for k, name in enumerate(names):
        print(f"  {name:34s} mean {d[:, k].mean():9.0f}  max {d[:, k].max():9.0f}  {100 * d[:, k].mean() / tot.mean():5.1f}%")
    return rows


def shard_timeline(model, sens, env, a):
    """per shard of the sharded rollout (workgroups [nb*s/S, nb*(s+1)/S)): realtime of its model_logic_kernel (start,
    model half end, logic end) and ray_sensor_kernel waves, from the first stamp of any shard (us), and the sensor
    waves' phase cycles"""
    S = env.rollout_streams
    cpb = (128 // a.cars) * a.cars                    # cars per step workgroup
    nb = -(-a.envs * a.cars // cpb)
    sub = 15 if cpb == 120 else None                  # 128-thread sensor workgroups: 8 cars each
    if sub is None:
        print("shard timeline: only for 120 cars per step workgroup")
        return
    t0 = min(model[model[:, 14] != 0, 14].min(), sens[sens[:, 14] != 0, 14].min())
    us = lambda v: (v - t0) / 100
    names = ["(staging)", "pose load", "beam cell lookup", "ray end point (f64)", "list head load", "walk", "store"]
    print(f"sharded rollout timeline (last step of the call; us from the first stamp; {S} shards of ~{nb // S} workgroups):")
    for s in range(S):
        b0, b1 = nb * s // S, nb * (s + 1) // S
        m = model[4 * b0:4 * b1]
        m = m[(m[:, 14] != 0) & (m[:, 9] != 0)].astype(np.float64)
        r = sens[2 * b0 * sub:2 * b1 * sub]
        r = r[(r[:, 14] != 0) & (r[:, 15] != 0)].astype(np.float64)
        if not len(m) or not len(r):
            print(f"  shard {s}: no stamps")
            continue
        d = np.diff(r[:, 0:8], axis=1)
        print(f"  shard {s}: model_logic start {us(m[:, 14].min()):7.1f} model-half end p50 {us(np.median(m[:, 15])):7.1f} "
              f"last {us(m[:, 15].max()):7.1f}, logic end last {us(m[:, 9].max()):7.1f} | sensor waves {len(r)}: first start "
              f"{us(r[:, 14].min()):7.1f} p50 start {us(np.median(r[:, 14])):7.1f} last start {us(r[:, 14].max()):7.1f} "
              f"p50 end {us(np.median(r[:, 15])):7.1f} last end {us(r[:, 15].max()):7.1f}; wave us p50 "
              f"{np.median(r[:, 15] - r[:, 14]) / 100:.1f}")
        print("    sensor wave cycles (mean): " + ", ".join(f"{nm} {d[:, k].mean():.0f}" for k, nm in enumerate(names)))
        # XCD placement (profile slot 10 of the model rows, 8 of the sensor rows: HW_REG_XCC_ID + 1): the rotation
        # (xcc - launch-local block) mod 8 of each dispatch, and how many sensor waves run on their cars' model XCD
        mx = model[4 * b0:4 * b1, 10].reshape(-1, 4)[:, 0].astype(np.int64)
        rx = sens[2 * b0 * sub:2 * b1 * sub, 8].reshape(-1, 2)[:, 0].astype(np.int64)
        if (mx > 0).all() and (rx > 0).all():
            mo = np.bincount((mx - 1 - np.arange(len(mx))) % 8, minlength=8)
            ro = np.bincount((rx - 1 - np.arange(len(rx))) % 8, minlength=8)
            same = (rx - 1 == np.repeat(mx - 1, sub)[:len(rx)]).mean()
            print(f"    XCD rotation (xcc - block) mod 8: model {mo.tolist()}, sensor {ro.tolist()}; sensor workgroups on "
                  f"their cars' model XCD {100 * same:.0f} %")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=8192)
    ap.add_argument("--cars", type=int, default=10)
    ap.add_argument("--track", default="daytona")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--no-build", action="store_true")
    ap.add_argument("--lib", default="libnascar_prof.so")
    ap.add_argument("--up", action="store_true", help="library built with -DNASCAR_PROFILE_UP")
    ap.add_argument("--raw", type=int, default=0, help="print this many raw sensor stamp rows")
    ap.add_argument("--load-state", default=None, help="start from a bench.py --save-state file (steady state); "
                    "actions then come from the device noisy rule driver (policy 3) instead of uniform draws")
    ap.add_argument("--define", action="append", default=[], help="extra -D for the profile build")
    ap.add_argument("--rollout", type=int, default=0, help="also profile one fused rollout launch of this many steps "
                    "(per-wave phase cycles per step: model, logic, sensors, each up to its block barrier)")
    ap.add_argument("--capture", default=None, help="library built with -DNASCAR_TOI_CAPTURE: save every computed TOI job's "
                    "inputs (float32 [n, 16]: car sweep c0.xy c.xy, a0 a alpha0 -, wall px py qs qc hx hy ang key) to this .npy")
    ap.add_argument("--sharded", type=int, default=0, help="step through the sharded rollout (nascar_rollout, R steps per "
                    "profiled call, policy 3) instead of launch_step; the stamps are the last step's, and a per-shard "
                    "timeline (model / logic / sensor realtime) is printed")
    ap.add_argument("--two-kernel", action="store_true", help="step through model_kernel + logic_kernel (the logic "
                    "kernel's own stamps) instead of the fused model_logic_kernel")
    ap.add_argument("--count", action="store_true", help="library built with -DNASCAR_PROFILE_COUNT (sensor event "
                    "counters; the atomics distort that build's sensor timings)")
    a = ap.parse_args()
    so = os.path.join(ROOT, "tools", a.lib)
    if not a.no_build:
        subprocess.run(["hipcc"] + _lib.HIPCC_FLAGS + ["-DNASCAR_PROFILE", "-DNASCAR_AB_KNOBS"] + (["-DNASCAR_PROFILE_UP"] if a.up else [])
                       + (["-DNASCAR_PROFILE_COUNT"] if a.count else []) + ["-D" + d for d in a.define]
                       + ["-o", so, os.path.join(_lib.CSRC, "nascar_kernels.hip")], check=True)
    _lib.LIB_PATH = so
    import torch
    from nascargymnasium_amd.batched import BatchedCarEnv
    from nascargymnasium_amd.track import track_path
    L = _lib.lib()
    L.nascar_debug_profile.argtypes = [ctypes.c_void_p]
    env = BatchedCarEnv(a.envs, a.cars, track_path(a.track), device="cuda:0")
    if a.two_kernel:
        env.set_fused_logic(False)
    env.reset()
    g = torch.Generator(device="cuda:0")
    g.manual_seed(7)
    k0 = 0
    if a.load_state:
        blob = torch.load(a.load_state, map_location="cuda:0", weights_only=True)
        env.set_state(blob["state"])
        env.obs.copy_(blob["obs"])
        k0 = int(blob["step"])

    def actions(k):
        if a.load_state:
            return env.policy_actions(3, seed=0, step=k).clone()
        return torch.rand((a.envs, a.cars, 2), generator=g, device="cuda:0") * 2 - 1
    for k in range(a.warmup):
        env.step(actions(k0 + k), auto_reset=True)
    CPROF_BASE = LPROF_BASE + NW * 16
    N = a.envs * a.cars
    RPROF_BASE = CPROF_BASE + (1 << 19) * 48   # device: CPROF_STRIDE 48 per car
    TCAP_BASE, TCAP_MAX = RPROF_BASE + 65536 * 5, 16384
    buf = torch.zeros(TCAP_BASE + 8 + TCAP_MAX * 8, dtype=torch.int64, device="cuda:0")
    caps = []
    L.nascar_debug_profile(ctypes.c_void_p(buf.data_ptr()))
    for s in range(a.steps):
        acts = actions(k0 + a.warmup + s)
        buf.zero_()
        torch.cuda.synchronize()
        if a.sharded:
            env.rollout(3, a.sharded, seed=0, step0=k0 + a.warmup + s * a.sharded)
        else:
            env.launch_step(acts, auto_reset=True)
        torch.cuda.synchronize()
        b = buf.cpu().numpy()
        if a.capture:   # -DNASCAR_TOI_CAPTURE builds: this step's b2TimeOfImpact jobs (sweep s0, s1, wall record)
            nc = min(int(b[TCAP_BASE]), TCAP_MAX)
            caps.append(b[TCAP_BASE + 8:TCAP_BASE + 8 + nc * 8].copy().view(np.float32).reshape(nc, 16))
            print(f"captured {nc} TOI jobs")
        model = b[:NW * 16].reshape(NW, 16)
        sens = b[NW * 16:2 * NW * 16].reshape(NW, 16)
        cnt = b[2 * NW * 16:2 * NW * 16 + 8]
        tcnt = b[2 * NW * 16 + 11:2 * NW * 16 + 16]
        print(f"TOI calls computed {tcnt[1]}, culled {tcnt[2]}, culled but TOUCHING (check builds) {tcnt[0]}, "
              f"events {tcnt[4]}")
        logic = b[LPROF_BASE:LPROF_BASE + NW * 16].reshape(NW, 16)
        print(f"--- step {s}")
        m = phases(model, MODEL, 0, "model_kernel")
        if len(m) and a.up:
            sub = np.stack([m[:, 11] - m[:, 2], m[:, 12] - m[:, 11], m[:, 13] - m[:, 12], m[:, 3] - m[:, 13]], 1)
            for k, name in enumerate(["engine force", "brake/drag/rolling + acc history", "weight transfer + tyres",
                                      "lateral..end"]):
                print(f"    update_physics/{name:32s} mean {sub[:, k].mean():9.0f}")
        elif len(m):
            sub = np.stack([m[:, 11] - m[:, 3], m[:, 12] - m[:, 11], m[:, 13] - m[:, 12], m[:, 4] - m[:, 13]], 1)
            for k, name in enumerate(["collide", "solve", "sync_fixtures+find_new_contacts", "solve_toi"]):
                print(f"    b2_step/{name:38s} mean {sub[:, k].mean():9.0f}")
        if len(m):
            st, en = m[:, 14], m[:, 15]
            print(f"    realtime us: last start {(st.max() - st.min()) / 100:.1f}, median end {(np.median(en) - st.min()) / 100:.1f}, "
                  f"last end {(en.max() - st.min()) / 100:.1f}")
        cp = b[CPROF_BASE:CPROF_BASE + N * 48].reshape(N, 48)   # CPROF_STRIDE
        if cp[:, 0].any():
            cyc = cp[:, 0]
            print(f"  per-car b2_step cycles: mean {cyc.mean():.0f}, p50 {np.percentile(cyc, 50):.0f}, "
                  f"p99 {np.percentile(cyc, 99):.0f}, p99.9 {np.percentile(cyc, 99.9):.0f}, max {cyc.max()}")
            print("  slowest waves' cars: car, wave b2 cycles, contacts at start (+1000 per FAILED TOI), TOI solved, TOI culled, "
                  "TOI events, contact updates, TOI outer iterations, root-finder iterations")
            info = env.info_tensor().cpu().numpy().reshape(N, -1)
            F = _lib.INFO_FIELDS
            for i in np.argsort(-cyc)[:24]:
                if cp[i, 1] or cp[i, 9]:
                    print("   ", i, *cp[i, [0, 1, 2, 3, 4, 5, 6, 7]].tolist(), f"| bp full scans {cp[i, 8]}, candidates {cp[i, 9]}"
                          f" | x {info[i, F.index('x')]:.1f} y {info[i, F.index('y')]:.1f} v ({info[i, F.index('vx')]:.1f}, "
                          f"{info[i, F.index('vy')]:.1f}) angle {info[i, F.index('angle')]:.2f} disabled {info[i, F.index('disabled')]:.0f} n_contacts {info[i, F.index('n_contacts')]:.0f}")
            per = (128 // a.cars) * a.cars                 # cars per workgroup (SBLOCK 128, whole envs)
            i0 = np.argsort(-cyc)[0]
            w0 = i0 // per * per + (i0 % per) // 64 * 64   # first car of the slowest car's wave
            w1 = min(w0 + 64, i0 // per * per + per, len(cp))
            print(f"  slowest wave (cars {w0}..{w1 - 1}): solve_toi scans {cp[w0, 14]}, TOI job rounds {cp[w0, 13]} cycles, "
                  f"event processing {cp[w0, 15]} cycles")
            for i in range(w0, w1):
                if cp[i, 26]:
                    print(f"    car {i}: island of {cp[i, 26]} touching contacts, island solve {cp[i, 25]} cycles")
            for i in range(w0, w1):
                if cp[i, 4] or cp[i, 2]:
                    print(f"    car {i}: events {cp[i, 4]}, island solve {cp[i, 11]}, event contact updates {cp[i, 12]}, "
                          f"TOI calls computed by this lane {cp[i, 2]}: outer iters {cp[i, 6]}, root iters {cp[i, 7]}, "
                          f"GJK cycles {cp[i, 9]}, separation-fn cycles {cp[i, 10]}")
            print(f"  rescans after a car's TOI event: TOIs computed {cp[:, 27].sum()} (TOUCHING {cp[:, 28].sum()}), "
                  f"culled {cp[:, 29].sum()}; slowest wave's cars: computed {cp[w0:w1, 27].sum()} "
                  f"(TOUCHING {cp[w0:w1, 28].sum()}), culled {cp[w0:w1, 29].sum()}")
            tc = cp[:, 2].sum()
            if tc:
                print(f"  all TOI calls {tc}: outer iters/call {cp[:, 6].sum() / tc:.2f}, root iters/call {cp[:, 7].sum() / tc:.2f}, "
                      f"GJK cycles/call {cp[:, 9].sum() / tc:.0f}, separation-fn cycles/call {cp[:, 10].sum() / tc:.0f}")
            ev = np.argsort(-cp[:, 4])[:12]
            print("  cars with the most TOI events: car, wave b2 cycles, events, TOI solved, contacts at start, "
                  "TOI-call cycles, island-solve cycles, event contact-update cycles, outer iterations")
            for i in ev:
                if cp[i, 4]:
                    print("   ", i, cp[i, 0], cp[i, 4], cp[i, 2], cp[i, 1], cp[i, 10], cp[i, 11], cp[i, 12], cp[i, 6])
            ne = cp[:, 4].sum()
            if ne:
                print(f"  per TOI event (all {ne} events): island solve {cp[:, 11].sum() / ne:.0f} cycles (position iterations "
                      f"{cp[:, 19].sum() / ne:.2f}, {cp[:, 20].sum() / ne:.0f} cycles; island contacts {cp[:, 18].sum() / ne:.2f}), "
                      f"contact updates {cp[:, 12].sum() / ne:.0f}, sync_fixtures+flags {cp[:, 17].sum() / ne:.0f}, "
                      f"find_new_contacts {cp[:, 16].sum() / ne:.0f}")
                print(f"    event sub-phases (cycles per event): scan + advance {cp[:, 38].sum() / ne:.0f}, manifold round "
                      f"{cp[:, 32].sum() / ne:.0f}, event contact's update {cp[:, 33].sum() / ne:.0f}; TOI island: init "
                      f"{cp[:, 34].sum() / ne:.0f}, position iterations {cp[:, 20].sum() / ne:.0f}, velocity init "
                      f"{cp[:, 35].sum() / ne:.0f}, 6 velocity iterations {cp[:, 36].sum() / ne:.0f}, integrate + transform + "
                      f"report {cp[:, 37].sum() / ne:.0f}")
                per = (128 // a.cars) * a.cars             # cars per workgroup (SBLOCK 128, whole envs)
                l0 = np.sort(np.concatenate([np.arange(0, N, per), np.arange(64, N, per)]))
                l0 = l0[l0 < N]                            # lane 0 of each wave
                w = cp[l0]
                print(f"  scans per wave: mean {w[:, 14].mean():.2f}, max {w[:, 14].max()}; job-round cycles per scan "
                      f"{w[:, 13].sum() / max(1, w[:, 14].sum()):.0f}, event-processing cycles per scan "
                      f"{w[:, 15].sum() / max(1, w[:, 14].sum()):.0f}")
            nc = cp[:, 1]
            print(f"  per car (mean over cars): collide {cp[:, 23].mean():.0f} cycles (cars with contacts: "
                  f"{cp[nc > 0, 23].mean() if (nc > 0).any() else 0:.0f}), sync_fixtures {cp[:, 22].mean():.0f}, "
                  f"find_new_contacts {cp[:, 21].mean():.0f} (moved cars {cp[:, 24].mean():.3f}; per moved car "
                  f"{cp[cp[:, 24] > 0, 21].mean() if (cp[:, 24] > 0).any() else 0:.0f}, p99 {np.percentile(cp[:, 21], 99):.0f})")
            evw = cp[cp[:, 4] > 0, 0]
            if len(evw):
                print(f"  b2 cycles of cars with TOI events: mean {evw.mean():.0f}, max {evw.max()}; cars with events {len(evw)}")
            wv = m[np.argmax(m[:, 4] - m[:, 3])]
            print("  slowest wave's b2_step phases (cycles): collide", wv[11] - wv[3], "solve", wv[12] - wv[11],
                  "sync+find", wv[13] - wv[12], "toi", wv[4] - wv[13])
            # the wave with the longest solve phase and its islands (stamp rows: blockIdx.x * 4 + wave of the block)
            ok = (model[:, 12] != 0) & (model[:, 11] != 0)
            sol = np.where(ok, model[:, 12] - model[:, 11], -1)
            ws = int(np.argmax(sol))
            per_w = (128 // a.cars) * a.cars
            blk, wi = divmod(ws, 4)
            c0 = blk * per_w + wi * 64
            lanes = [i for i in range(c0, min(c0 + 64, blk * per_w + per_w, len(cp))) if cp[i, 26]]
            print(f"  longest solve phase {sol[ws]} cycles (block {blk} wave {wi}); its islands (touching contacts: "
                  f"solve cycles): " + ", ".join(f"{cp[i, 26]}: {cp[i, 25]}" for i in lanes))
            isl = cp[:, 26]
            for lo, hi in [(1, 3), (3, 4), (4, 9)]:
                sel = (isl >= lo) & (isl < hi)
                if sel.any():
                    print(f"  islands of {lo}-{hi - 1} contacts: {sel.sum()} cars, solve cycles mean {cp[sel, 25].mean():.0f} "
                          f"max {cp[sel, 25].max()}")
            print(f"  broadphase full scans per car-step {cp[:, 8].mean():.4f}, cars with a full scan {(cp[:, 8] > 0).sum()}")
            it = cp[:, 7]
            print(f"  root-finder iterations per car-step: mean {it.mean():.2f}, max {it.max()}, cars > 100: {(it > 100).sum()}, "
                  f"FAILED TOIs {(cp[:, 1] // 1000).sum()}")
            for lo, hi in [(0, 1), (1, 2), (2, 4), (4, 8), (8, 17)]:
                m = (cp[:, 1] >= lo) & (cp[:, 1] < hi)
                if m.any():
                    print(f"  cars with {lo}-{hi - 1} contacts: {m.mean() * 100:5.1f}%  mean b2 cycles {cyc[m].mean():.0f}")
        fz = model[(model[:, 6] != 0) & (model[:, 8] != 0) & (model[:, 15] != 0)].astype(np.float64)
        if len(fz):   # the fused model_logic_kernel's logic half: barrier wait, loads + staging, logic_run
            i_last = np.argmax(fz[:, 9])
            rt0 = fz[:, 14].min()
            print(f"model_logic_kernel logic half: waves {len(fz)}; barrier wait (model end -> block barrier) mean "
                  f"{(fz[:, 6] - fz[:, 5]).mean():.0f}, loads + staging mean {(fz[:, 7] - fz[:, 6]).mean():.0f}, logic_run mean "
                  f"{(fz[:, 8] - fz[:, 7]).mean():.0f} cycles; realtime us: median model end {(np.median(fz[:, 15]) - rt0) / 100:.1f}, "
                  f"median logic end {(np.median(fz[:, 9]) - rt0) / 100:.1f}, last logic end {(fz[:, 9].max() - rt0) / 100:.1f}")
            w = fz[i_last]
            print(f"  last-ending wave: model half {w[5] - w[0]:.0f} cycles (b2_step {w[4] - w[3]:.0f}), barrier wait "
                  f"{w[6] - w[5]:.0f}, loads + staging {w[7] - w[6]:.0f}, logic_run {w[8] - w[7]:.0f}; model end "
                  f"{(w[15] - rt0) / 100:.1f} us, logic end {(w[9] - rt0) / 100:.1f} us")
            # logic_run's own stamps (LPROF 1-8, same wave rows) from the logic half's start (PROF 7)
            lz = logic.copy()
            lz[:, 0] = np.where((model[:, 7] != 0) & (model[:, 8] != 0), model[:, 7], 0)
            lr = phases(lz, ["(entry)", "bank / impulse / stuck / lap timer", "barrier + env pass 1 + stuck disable",
                             "car_obs", "rewards (progress)", "barrier + env pass 2 + barrier + flags", "reset / pose B / state store",
                             "barrier + obs rows"], 0, "  model_logic_kernel logic_run")
            if len(lr):
                j = int(np.argmax(model[:, 9]))
                if lz[j, 0] and lz[j, 8]:
                    print("    last-ending wave's logic_run phases:", np.diff(lz[j, :9]).astype(int).tolist())
        phases(logic, LOGIC, 0, "logic_kernel")
        if a.raw:
            live = sens[sens[:, 0] != 0]
            print("raw sensor stamps (first rows, slots 0-6):")
            for row in live[:a.raw]:
                print("   ", row[:7] - row[0], " realtime us:", (row[15] - row[14]) / 100)
            rt = live[:, 15] - live[:, 14]
            print(f"  sensor realtime per wave us: mean {rt.mean() / 100:.1f} max {rt.max() / 100:.1f}; "
                  f"kernel span {(live[:, 15].max() - live[:, 14].min()) / 100:.1f}")
        n = cnt[6]
        extra = ""
        if n:
            extra = (f"\n  per active lane: groups visited {cnt[0] / n:.1f}, in range {cnt[1] / n:.1f}, open {cnt[2] / n:.1f}, "
                     f"walls {cnt[3] / n:.1f}, wall-ray pairs {cnt[4] / n:.1f}, exact casts {cnt[5] / n:.1f}")
        rs = sens[(sens[:, 0] != 0) & (sens[:, 7] != 0) & (sens[:, 2] != 0)].astype(np.float64)
        if len(rs):   # ray_sensor_kernel at 16 lanes per car (PROFR stamps)
            d = np.diff(rs[:, 0:8], axis=1)
            names = ["wall image staging + barrier", "pose load", "beam cell lookup", "ray end point (f64)", "list head load",
                     "walk", "store"]
            tot = d.sum(1)
            print(f"ray_sensor_kernel: waves {len(rs)}, mean wave cycles {tot.mean():.0f} (p50 {np.median(tot):.0f}, max "
                  f"{tot.max():.0f}); realtime us: last start {(rs[:, 14].max() - rs[:, 14].min()) / 100:.1f}, median end "
                  f"{(np.median(rs[:, 15]) - rs[:, 14].min()) / 100:.1f}, last end {(rs[:, 15].max() - rs[:, 14].min()) / 100:.1f}")
            for k, nm in enumerate(names):
                print(f"  {nm:34s} mean {d[:, k].mean():9.0f}  p50 {np.median(d[:, k]):9.0f}  max {d[:, k].max():9.0f}")
            w = rs[np.argmax(rs[:, 15])]
            print("  last-ending wave: " + ", ".join(f"{nm} {w[k + 1] - w[k]:.0f}" for k, nm in enumerate(names)))
        phases(sens, SENSOR, 0, "sensor_kernel", extra)
        if a.sharded and len(rs):
            shard_timeline(model, sens, env, a)
        cb = b[2 * NW * 16 + 8:2 * NW * 16 + 16]
        if cb[4] or cb[5] or cb[6]:
            ncar = a.envs * a.cars
            print(f"model counters per car-step: TOI solved {cb[4] / ncar:.3f}, TOI culled {cb[5] / ncar:.3f}, "
                  f"contact updates {cb[6] / ncar:.3f}, TOI events {cb[7] / ncar:.4f}")
        ck = b[2 * NW * 16 + 16:2 * NW * 16 + 18]
        if ck[0]:
            print(f"TOI cull check: culled TOIs re-run {ck[0]}, of which TOUCHING (cull violations) {ck[1]}")
        if cb[0]:
            print(f"ray_sensor_kernel: rays {cb[0]}, fallback rays {cb[1]} ({100 * cb[1] / cb[0]:.2f}%), "
                  f"list entries per ray {cb[3] / max(1, cb[0] - cb[1]):.2f}, walked {cb[2] / max(1, cb[0] - cb[1]):.2f}")
    if a.capture and caps:
        np.save(a.capture, np.concatenate(caps))
    if a.rollout:
        import time
        buf.zero_()
        env.set_rollout_streams(0)   # the fused rollout kernel (its per-wave phase counters)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        env.rollout(3 if a.load_state else 0, a.rollout, seed=0, step0=k0 + a.warmup + a.steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        r = buf[RPROF_BASE:RPROF_BASE + 65536 * 4].cpu().numpy().reshape(-1, 4)
        r = r[r[:, 3] > 0].astype(np.float64)
        per = r[:, :3] / r[:, 3:4]
        tot = per.sum(1)
        print(f"rollout_kernel: {a.rollout} steps in {dt * 1e3:.1f} ms ({dt / a.rollout * 1e6:.1f} us/step incl. launch), "
              f"waves {len(r)}; cycles per step per wave: total mean {tot.mean():.0f} (max wave {tot.max():.0f})")
        for k, name in enumerate(["policy + model (+ barrier)", "logic (+ barrier)", "sensors (+ barrier)"]):
            print(f"  {name:28s} mean {per[:, k].mean():9.0f}  p90 {np.percentile(per[:, k], 90):9.0f}  "
                  f"max {per[:, k].max():9.0f}")
        print(f"  per-wave totals over the launch (cycles per step): p50 {np.percentile(tot, 50):.0f}, p90 "
              f"{np.percentile(tot, 90):.0f}, p99 {np.percentile(tot, 99):.0f}, max {tot.max():.0f} -- the launch lasts as "
              f"long as its slowest workgroup's sum over the steps")
    L.nascar_debug_profile(ctypes.c_void_p(0))
    env.close()


if __name__ == "__main__":
    main()

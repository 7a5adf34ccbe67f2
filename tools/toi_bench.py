"""b2TimeOfImpact micro-benchmark on captured steady-state jobs (tools/toi_bench.hip).  Not product code.

    python tools/toi_bench.py --jobs tools/data/toi_jobs_r05.npy --libs tools/toi_bench_base.so tools/toi_bench_x.so

The jobs come from a -DNASCAR_PROFILE -DNASCAR_TOI_CAPTURE build (tools/phase_profile.py --capture).  For each library
(variants of nascar_device.h's toi_alpha built with different -D flags) and each (lanes, workgroups) setting it prints
s_memtime cycles per round -- lanes = 1: one call at a time, a lone TOI chain as in the slowest wave's scans -- split by
outcome (alpha < 1: TOUCHING, the event-producing calls), and checks that every variant's alphas equal the first's
bit for bit.
"""
import argparse
import ctypes

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", required=True)
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--lanes", type=int, nargs="+", default=[1, 16, 64])
    ap.add_argument("--blocks", type=int, nargs="+", default=[1, 1024])
    ap.add_argument("--max-jobs", type=int, default=4096)
    a = ap.parse_args()
    jobs = np.load(a.jobs)[:a.max_jobs].astype(np.float32)
    n = len(jobs)
    dj = torch.from_numpy(jobs).cuda()
    alpha = torch.ones(n, dtype=torch.float32, device="cuda")
    cyc = torch.zeros(n, dtype=torch.int64, device="cuda")
    ref = None
    print(f"{n} jobs")
    for path in a.libs:
        L = ctypes.CDLL(path)
        L.toi_bench.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_void_p]
        det = torch.zeros(n, 5, dtype=torch.int32, device="cuda")
        for lanes in a.lanes:
            for blocks in a.blocks:
                alpha.fill_(2.0)
                cyc.zero_()
                L.toi_bench(dj.data_ptr(), n, 1, 1, alpha.data_ptr(), cyc.data_ptr(), det.data_ptr())     # warm
                assert L.toi_bench(dj.data_ptr(), n, lanes, blocks, alpha.data_ptr(), cyc.data_ptr(), det.data_ptr()) == 0
                al = alpha.cpu().numpy().copy()
                rounds = (n + lanes - 1) // lanes
                c = cyc.cpu().numpy()[:rounds].astype(np.float64)
                if ref is None:
                    ref = al
                same = np.array_equal(al.view(np.uint32), ref.view(np.uint32))
                txt = f"{path.split('/')[-1]:28s} lanes {lanes:2d} wgs {blocks:5d}: cycles/round mean {c.mean():8.0f} p50 " \
                      f"{np.median(c):8.0f} p99 {np.percentile(c, 99):8.0f} max {c.max():8.0f}"
                if lanes == 1:
                    t = al < 1.0
                    txt += f" | TOUCHING {t.sum()} calls mean {c[t].mean() if t.any() else 0:8.0f}, others {c[~t].mean():8.0f}"
                print(txt + ("" if same else "  ALPHAS DIFFER"), flush=True)
                d = det.cpu().numpy().astype(np.float64)
                if lanes == 1 and blocks == 1 and d[:, 0].any():   # detail build (-DNASCAR_PROFILE)
                    cyc1 = c
                    print(f"    per call: outer iters {d[:, 0].mean():.2f}, root iters {d[:, 1].mean():.2f}, GJK iters "
                          f"{d[:, 2].mean():.2f}; GJK cycles {d[:, 3].mean():.0f}, separation-fn cycles {d[:, 4].mean():.0f}, "
                          f"rest {cyc1.mean() - d[:, 3].mean() - d[:, 4].mean():.0f}")
                    X = np.stack([np.ones(n), d[:, 0], d[:, 1], d[:, 2]], 1)
                    coef = np.linalg.lstsq(X, cyc1, rcond=None)[0]
                    print(f"    least squares cycles = {coef[0]:.0f} + {coef[1]:.0f} x outer + {coef[2]:.0f} x root + "
                          f"{coef[3]:.0f} x GJK iteration")


if __name__ == "__main__":
    main()

"""s_memtime phase profile of actor_kernel (profile build, -DNASCAR_PROFILE).

    python tools/actor_profile.py [N] [--no-build]

Per wave: slot 0 kernel entry, 1 after the weight staging barrier, 1+k after its k-th tile (k <= 5),
7-10 phases of the first tile,
14/15 s_memrealtime (100 MHz) at entry/exit.  Prints the staging cycles, per-tile cycles (by tile
index) and the realtime spread of wave starts/ends.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from nascargymnasium_amd import _lib  # noqa: E402

BASE = 2 * 65536 * 16 + 64


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else 81920
    so = os.path.join(ROOT, "tools", "libnascar_prof.so")
    if "--no-build" not in sys.argv:
        subprocess.run(["hipcc"] + _lib.HIPCC_FLAGS + ["-DNASCAR_PROFILE", "-o", so,
                        os.path.join(_lib.CSRC, "nascar_kernels.hip")], check=True)
    _lib.LIB_PATH = so
    import torch
    from nascargymnasium_amd.batched import BatchedCarEnv
    from nascargymnasium_amd.policy import random_actor
    L = _lib.lib()
    L.nascar_debug_profile.argtypes = [ctypes.c_void_p]
    env = BatchedCarEnv(1, 1, "daytona", device="cuda:0")
    env.set_actor(random_actor(0))
    x = torch.rand(n, 38, device="cuda:0")
    for _ in range(5):
        env.actor_forward(x)
    nw = 4096
    buf = torch.zeros(BASE + nw * 16, dtype=torch.int64, device="cuda:0")
    L.nascar_debug_profile(ctypes.c_void_p(buf.data_ptr()))
    runs = []
    for _ in range(3):
        buf.zero_()
        torch.cuda.synchronize()
        env.actor_forward(x)
        torch.cuda.synchronize()
        runs.append(buf[BASE:].view(nw, 16).cpu().numpy().astype(np.float64))
    L.nascar_debug_profile(ctypes.c_void_p(0))
    for b in runs:
        b = b[b[:, 0] != 0]
        stage = b[:, 1] - b[:, 0]
        print(f"waves {len(b)}: staging cycles mean {stage.mean():.0f} max {stage.max():.0f}")
        f = b[(b[:, 7] != 0) & (b[:, 10] != 0)]
        if len(f):
            ph = np.diff(np.concatenate([f[:, 1:2], f[:, 7:11], f[:, 2:3]], 1), axis=1)
            for name, col in zip(["loop top", "fetch+layer 1+relu/cvt", "layer 2 half 0 + epi", "layer 2 half 1 + epi",
                                  "layer 3 finish + store"], ph.T):
                print(f"  first tile {name:26s} mean {col.mean():8.0f}  max {col.max():8.0f}")
        for t in range(1, 6):
            m = b[:, 1 + t] != 0
            if not m.any():
                break
            d = b[m, 1 + t] - b[m, t]
            print(f"  tile {t}: waves {m.sum():5d}  cycles mean {d.mean():8.0f}  max {d.max():8.0f}")
        st, en = b[:, 14], b[:, 15]
        t0 = st.min()
        print(f"  realtime us: last start {(st.max() - t0) / 100:.2f}  median end {(np.median(en) - t0) / 100:.2f}  "
              f"last end {(en.max() - t0) / 100:.2f}")
    env.close()


if __name__ == "__main__":
    main()

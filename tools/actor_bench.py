"""Time the fused SAC actor kernel alone (HIP events): python tools/actor_bench.py [N] [iters]

Launches go straight through the C ABI with preallocated buffers so that host dispatch stays below
the kernel time (BatchedCarEnv.actor_forward allocates its output per call)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nascargymnasium_amd.batched import BatchedCarEnv  # noqa: E402
from nascargymnasium_amd.policy import random_actor  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 81920
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 200
env = BatchedCarEnv(1, 1, "daytona", device="cuda:0")
env.set_actor(random_actor(0))
x = torch.rand(N, 38, device="cuda:0")
out = torch.empty(N, 2, device="cuda:0")
fwd, h = env.L.nascar_actor_forward, env.h
args = (h, ctypes.c_void_p(x.data_ptr()), N, ctypes.c_void_p(out.data_ptr()),
        ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
for _ in range(10):
    fwd(*args)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(iters):
    fwd(*args)
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / iters
flop = 2.0 * N * (38 * 256 + 256 * 256 + 256 * 2)
mfma_flop = 2.0 * N * (64 * 256 + 256 * 256)
print(f"actor N={N}: {ms * 1e3:.1f} us/launch, {N / ms * 1e3:.3e} actions/s, "
      f"{flop / ms / 1e9:.1f} TFLOP/s algorithmic ({mfma_flop / ms / 1e9:.1f} TFLOP/s on the MFMA shapes)")
env.close()

"""Host enqueue time of one nascar_rollout call vs its device time, per shard count (is the sharded rollout
launch-bound?).  Usage: python tools/ro_host_time.py"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from nascargymnasium_amd.batched import BatchedCarEnv  # noqa: E402
from nascargymnasium_amd.track import track_path  # noqa: E402

env = BatchedCarEnv(8192, 10, track_path("daytona"), device="cuda:0")
env.reset()
env.rollout(3, int(sys.argv[1]) if len(sys.argv) > 1 else 3000, seed=1)   # leave the start (contacts, spread)
torch.cuda.synchronize()
snap, obs0 = env.get_state(), env.obs.clone()
R = 50
for S in (1, 2, 4, 6, 8):
    env.set_state(snap)                # every S from the same state (the synchronized-start workload drifts)
    env.obs.copy_(obs0)
    env.set_rollout_streams(S)
    env.rollout(3, R, seed=1, step0=3000)
    torch.cuda.synchronize()
    host, dev = [], []
    for it in range(4):
        t0 = time.perf_counter()
        env.rollout(3, R, seed=1, step0=3000 + R * (it + 1))
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        host.append((t1 - t0) / R * 1e6)
        dev.append((t2 - t0) / R * 1e6)
    print(f"S={S}: host enqueue {min(host):.1f} us/step, wall {min(dev):.1f} us/step "
          f"({3 * S} launches per step, {(t1 - t0) / (3 * S * R) * 1e6:.2f} us per launch)", flush=True)

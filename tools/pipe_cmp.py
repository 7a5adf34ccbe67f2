"""Pipelined rollout vs the sharded one from the same state: which outputs differ after K steps (diagnostic)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from nascargymnasium_amd.batched import BatchedCarEnv  # noqa: E402

E, C, grid = int(os.environ.get("E", 48)), int(os.environ.get("C", 10)), int(os.environ.get("GRID", 64))
a = BatchedCarEnv(E, C, "daytona", device="cuda:0", envs_per_block=12)
b = BatchedCarEnv(E, C, "daytona", device="cuda:0", envs_per_block=12)
a.reset()
a.rollout(3, 600, seed=5, step0=0, auto_reset=True)
b.set_rollout_pipe(grid)
for K in (1, 1, 2, 5):
    b.set_state(a.get_state()); b.obs.copy_(a.obs)
    ra = a.rollout(3, K, seed=5, step0=600, auto_reset=True, trajectory=True)
    rb = b.rollout(3, K, seed=5, step0=600, auto_reset=True, trajectory=True)
    torch.cuda.synchronize()
    st = b.rollout_pipe_status()
    d = (a.obs != b.obs).reshape(-1, 38)
    cols = torch.nonzero(d.any(0)).flatten().tolist()
    cars = torch.nonzero(d.any(1)).flatten().tolist()
    print(f"K={K} status {st}: obs differ in {len(cars)} cars, cols {cols[:40]}; rewards equal per step "
          f"{[bool(torch.equal(ra[1][k], rb[1][k])) for k in range(K)]}; state equal {torch.equal(a.get_state(), b.get_state())}",
          flush=True)
    for n in ([cars[0]] if cars else []) + [33, 34, 153]:
        print("  car", n, "a", a.obs.reshape(-1, 38)[n].tolist()[20:38], flush=True)
        print("  car", n, "b", b.obs.reshape(-1, 38)[n].tolist()[20:38], flush=True)
    b.set_state(a.get_state()); b.obs.copy_(a.obs)

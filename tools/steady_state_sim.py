"""CPU oracle run of the bench's steady-state workload (noisy rule driver, auto-reset) to characterise
it: per window of steps, the fraction of car-steps with a wall-contact impulse, lap completions,
disabled cars and env resets.  Test/diagnostic tooling (uses the oracle), never the product.

    python tools/steady_state_sim.py [--track daytona] [--envs 4] [--cars 10] [--steps 10800] [--window 900]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from drivers import NoisyRuleDriver  # noqa: E402
from oracle_lib import OracleEnv  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--track", default="daytona")
    ap.add_argument("--envs", type=int, default=4)
    ap.add_argument("--cars", type=int, default=10)
    ap.add_argument("--steps", type=int, default=10800)
    ap.add_argument("--window", type=int, default=900)
    args = ap.parse_args()
    E, C = args.envs, args.cars
    env = OracleEnv(os.path.join(ROOT, "nascargymnasium_amd", "tracks", args.track + ".track"), E, C)
    obs = env.reset()[0]
    drv = NoisyRuleDriver(E * C)
    acc = np.zeros(5)
    laps = np.zeros(E * C)
    for k in range(args.steps):
        a = drv.actions(obs, k)
        obs, rew, cf, ef = env.step(a.reshape(E, C, 2))
        done = (ef[:, 0] != 0) | (ef[:, 1] != 0)
        lc = np.array([env.car_info(i)["lap_count"] for i in range(E * C)])
        acc += [(obs[..., 19] > 0).mean(), (lc > laps).mean(), (cf & 1).astype(bool).mean(),
                done.mean(), np.abs(obs[..., 4]).mean() * 111.1]
        laps = lc
        for e in np.nonzero(done)[0]:
            env.reset(int(e))
            laps[e * C:(e + 1) * C] = 0
            obs = env.outputs()[0]
        if (k + 1) % args.window == 0:
            m = acc / args.window
            print(f"steps {k + 1 - args.window:5d}-{k + 1:5d}: contact {m[0]:.4f} lap {m[1]:.5f} disabled {m[2]:.3f} "
                  f"env-reset {m[3]:.5f} speed {m[4]:.1f} m/s", flush=True)
            acc[:] = 0


if __name__ == "__main__":
    main()

"""Fixture for the fused SAC actor: the actor tensors of the reference's own checkpoint
game/control/models/sac_1235.zip plus float32 reference actions on observations from the golden env traces.
TEST INFRASTRUCTURE (run here, where /root/reference exists; the npz travels, the reference does not).

The checkpoint is opened with zipfile and policy.pth with torch.load(weights_only=True) (nascargymnasium_amd.
policy.load_sb3_actor) -- nothing in it is executed.  Its JSON `data` records action_space Box(-1, 1, (2,),
float32), observation_space Box((38,)) and policy_kwargs {use_sde: False}: SB3's SAC MlpPolicy actor with
net_arch [256, 256].  stable_baselines3 is not installed here, so its deterministic predict()
(game/control/sac_control_class.py:80-115 -> SACPolicy._predict -> Actor.forward(deterministic=True)) is
restated in PyTorch float32: FlattenExtractor (identity), latent_pi = Linear-ReLU-Linear-ReLU, mu = Linear,
action = tanh(mu) (SquashedDiagGaussianDistribution.mode), then BasePolicy.unscale_action in numpy float32.

    python oracle/gen_actor_fixture.py [--ref /root/reference]  ->  tests/golden/sac_1235_actor.npz
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def sb3_predict_fp32(w, obs):
    import torch
    t = {k: torch.from_numpy(v) for k, v in w.items()}
    with torch.no_grad():
        x = torch.from_numpy(np.ascontiguousarray(obs, np.float32))
        h = torch.relu(torch.nn.functional.linear(x, t["actor.latent_pi.0.weight"], t["actor.latent_pi.0.bias"]))
        h = torch.relu(torch.nn.functional.linear(h, t["actor.latent_pi.2.weight"], t["actor.latent_pi.2.bias"]))
        a = torch.tanh(torch.nn.functional.linear(h, t["actor.mu.weight"], t["actor.mu.bias"])).numpy()
    low, high = np.float32(-1.0), np.float32(1.0)
    return (low + (np.float32(0.5) * (a + np.float32(1.0)) * (high - low))).astype(np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden", "sac_1235_actor.npz"))
    a = ap.parse_args()
    from nascargymnasium_amd.policy import load_sb3_actor
    w = load_sb3_actor(os.path.join(a.ref, "game", "control", "models", "sac_1235.zip"))
    gold = os.path.join(ROOT, "tests", "golden")
    rows = []
    for name in ["env_daytona_long", "env_talladega_10car", "env_martinsville_lap", "env_daytona_damage",
                 "env_nascar_backward", "env_michigan_banked"]:
        d = np.load(os.path.join(gold, name + ".npz"))
        o = d["obs"].reshape(-1, 38)
        rows.append(o[np.linspace(0, len(o) - 1, min(len(o), 400)).astype(int)])
    obs = np.ascontiguousarray(np.concatenate(rows), np.float32)
    act = sb3_predict_fp32(w, obs)
    np.savez_compressed(a.out, obs=obs, actions_fp32=act, **{k.replace(".", "__"): v for k, v in w.items()})
    print(a.out, obs.shape, "action range", act.min(0), act.max(0))


if __name__ == "__main__":
    main()

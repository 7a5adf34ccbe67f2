"""SAC actor weights for the fused device policy.

The reference's SACController loads a Stable-Baselines3 checkpoint with ``SAC.load``
(game/control/sac_control_class.py:48-76) and calls ``model.predict(obs, deterministic=True)``.
Here the checkpoint zip is opened with ``zipfile`` and ``policy.pth`` with
``torch.load(weights_only=True)`` -- nothing in the file is executed -- and only the actor
tensors are kept; inference runs in ``actor_kernel`` (csrc/nascar_actor.h).
"""
import io
import zipfile

import numpy as np

ACTOR_KEYS = ("actor.latent_pi.0.weight", "actor.latent_pi.0.bias", "actor.latent_pi.2.weight",
              "actor.latent_pi.2.bias", "actor.mu.weight", "actor.mu.bias")
SHAPES = ((256, 38), (256,), (256, 256), (256,), (2, 256), (2,))


def load_sb3_actor(zip_path: str) -> dict:
    """Actor tensors of an SB3 SAC checkpoint (MlpPolicy, net_arch [256, 256])."""
    import torch
    with zipfile.ZipFile(zip_path) as z:
        sd = torch.load(io.BytesIO(z.read("policy.pth")), weights_only=True, map_location="cpu")
    missing = [k for k in ACTOR_KEYS if k not in sd]
    if missing:
        raise ValueError(f"{zip_path}: not an SB3 SAC MlpPolicy checkpoint (missing {missing})")
    return {k: sd[k].float().numpy() for k in ACTOR_KEYS}


def random_actor(seed: int = 0) -> dict:
    """Random-init actor of the reference architecture (PyTorch nn.Linear default init)."""
    rng = np.random.default_rng(seed)
    out = {}
    for k, shp in zip(ACTOR_KEYS, SHAPES):
        fan_in = 38 if "latent_pi.0" in k else 256
        bound = 1.0 / np.sqrt(fan_in)
        out[k] = rng.uniform(-bound, bound, shp).astype(np.float32)
    return out


def actor_arrays(weights: dict):
    arrs = []
    for k, shp in zip(ACTOR_KEYS, SHAPES):
        a = np.ascontiguousarray(np.asarray(weights[k], np.float32))
        if a.shape != shp:
            raise ValueError(f"{k}: shape {a.shape}, expected {shp}")
        arrs.append(a)
    return arrs

"""Closed-loop GPU-vs-oracle comparison at several workgroup layouts.  TEST INFRASTRUCTURE.

The device noisy rule driver (policy 3, nascar_step_driven: the driver inside model_kernel, as the bench runs it)
drives one BatchedCarEnv per layout (envs per 128-lane workgroup, nascar_set_envs_per_block); the host restatement
of the same driver (tests/drivers.py) drives the oracle.  Every step, every layout's observations, rewards,
disabled flags, done flags and termination reasons must equal the oracle's bit for bit.  The layouts replace the
reference's per-env / per-car loops (src/car_env.py:567-570, 1115-1158), so the results may not depend on them.
"""
import numpy as np


def make_envs(E, C, tracks, layouts, fused=(), **kw):
    """one BatchedCarEnv per layout (None: the engine's automatic choice), asserting that the layout took; the
    engines whose positions are listed in `fused` step through the fused model + logic kernel"""
    from nascargymnasium_amd.batched import BatchedCarEnv
    envs = []
    for i, epb in enumerate(layouts):
        env = BatchedCarEnv(E, C, tracks, device="cuda:0", envs_per_block=epb, **kw)
        if epb is not None:
            assert env.envs_per_block == epb
        env.set_fused_logic(i in fused)   # explicit either way (the engine's default is the fused kernel)
        envs.append(env)
    return envs


def closed_loop_vs_oracle(envs, orc, steps, seed, stagger, check_actions=False):
    """Drive every env of `envs` (BatchedCarEnv, same E x C) with device policy 3 and `orc` (OracleEnv /
    OracleGroups) with the host restatement; compare every step.  stagger: {step: env} masked resets.
    check_actions: also compare the device driver's actions (nascar_policy_actions) with the host's, stepping the
    first layout through policy_actions + nascar_step instead of nascar_step_driven.  Returns event tallies."""
    import torch
    from drivers import NoisyRuleDriver
    E, C = envs[0].E, envs[0].C
    drv = NoisyRuleDriver(E * C, seed=seed)
    oo = orc.reset()[0]
    for env in envs:
        assert np.array_equal(env.reset().cpu().numpy(), oo), f"reset obs (envs per block {env.envs_per_block})"
    t = dict(contact=0, disabled=0, resets=0, laps=0, reasons=set(), max_age=0)
    age = np.zeros(E, np.int64)
    for k in range(steps):
        if k in stagger:
            e = stagger[k]
            m = torch.zeros(E, dtype=torch.uint8, device=envs[0].device)
            m[e] = 1
            for env in envs:
                env.reset(m)
            orc.reset([e])
            oo = orc.outputs()[0]
            age[e] = 0
        ha = drv.actions(oo, k)
        for i, env in enumerate(envs):
            if check_actions and i == 0:
                ga = env.policy_actions(3, seed=seed, step=k).clone()
                assert np.array_equal(ga.cpu().numpy().reshape(-1, 2), ha), f"step {k}: driver actions differ"
                env.launch_step(ga, auto_reset=True)
            else:
                env.step_driven(3, seed=seed, step=k, auto_reset=True)
        oo, orw, ocf, oef = orc.step(ha)
        done = (oef[:, 0] != 0) | (oef[:, 1] != 0)
        if done.any():
            orc.reset(np.nonzero(done)[0])
            oo = orc.outputs()[0]
        for env in envs:
            lay = f"envs per block {env.envs_per_block}" + (", fused model + logic" if env.fused_logic else ", model_kernel + logic_kernel")
            gr, gcf, gef = env.reward.cpu().numpy(), env.car_flags.cpu().numpy(), env.env_flags.cpu().numpy()
            assert np.array_equal(gr, orw), f"step {k} ({lay}): reward mismatch at {np.argwhere(gr != orw)[:5].tolist()}"
            assert np.array_equal(gcf & 5, ocf & 5), f"step {k} ({lay}): disabled / collision flags"
            assert np.array_equal((gef & 3) != 0, done), f"step {k} ({lay}): done flags"
            assert np.array_equal(((gef >> 4) & 7)[done], oef[done, 2]), f"step {k} ({lay}): termination reasons"
            go = env.obs.cpu().numpy()
            bad = np.argwhere(go != oo)
            assert len(bad) == 0, (f"step {k} ({lay}): obs mismatch at {bad[:5].tolist()} gpu {go[tuple(bad[0])]} "
                                   f"oracle {oo[tuple(bad[0])]}")
        age += 1
        if done.any():
            t["reasons"] |= set(oef[done, 2].tolist())
            t["max_age"] = max(t["max_age"], int(age[done].max()))
            t["resets"] += int(done.sum())
            age[done] = 0
        t["contact"] += int(((gcf & 4) != 0).sum())
        t["disabled"] += int(((gcf & 2) != 0).sum())
        t["laps"] += int(((gcf & 8) != 0).sum())
    t["max_age"] = max(t["max_age"], int(age.max()))
    for env in envs:
        assert not (env.car_flags.cpu().numpy() & 128).any(), "contact buffer overflow"
    return t

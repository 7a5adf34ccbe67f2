"""Before/after of the drop-in VecCarEnv path (round 6): the same measurement as bench.drop_in_pass's random-track
rows, run on the round-5 package (tools/r05_tree: `git archive 8194fc8`, its own libnascar.so), whose random-track mode
synchronised with the host every step (done flags, Python redraws, host block-map rebuild, masked reset).
    mkdir tools/r05_tree && git archive 8194fc8 nascargymnasium_amd include | tar -x -C tools/r05_tree
    (cd tools/r05_tree && python -c "from nascargymnasium_amd import _lib; _lib.build()")
    python tools/vec_before.py [E] [C] [K]    (GPU; prints one JSON line; profiles/r06_vec_env_before.jsonl)"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "r05_tree"))
import nascargymnasium_amd  # noqa: E402  (the round-5 package, before bench puts the repo on the path)
sys.path.insert(1, os.path.dirname(HERE))
import bench  # noqa: E402
import torch  # noqa: E402


def main():
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    C = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    from nascargymnasium_amd import VecCarEnv
    assert "r05_tree" in nascargymnasium_amd.__file__
    dev = torch.device("cuda", 0)
    venv = VecCarEnv(E, None, num_cars=C, return_tensors=True, seed=1000)
    eng = venv.engine
    venv.reset()
    t0 = time.perf_counter()
    bench.settle(eng, bench.Stepper(eng, "noisy", 0, None, None, 0), bench.EPISODE_STEPS, True, dev)
    torch.cuda.synchronize()
    t_settle = time.perf_counter() - t0
    holder = [eng.obs]

    def one(i):
        a = eng.policy_actions(3, seed=0, step=i, obs=holder[0])
        holder[0] = venv.step(a)[0]
    bench._window(one, 0, 5, dev)
    dones = [0]
    el = bench._window(one, 5, K, dev)
    print(json.dumps({"package": "round 5 (8194fc8)", "config": f"VecCarEnv(track_file=None) {E} envs x {C} cars, "
                      f"return_tensors=True, steady state after {bench.EPISODE_STEPS} steps ({t_settle:.1f} s)",
                      "vec_env": E * C * K / el, "ms_per_step": el / K * 1e3, "steps": K}), flush=True)
    venv.close()


if __name__ == "__main__":
    main()

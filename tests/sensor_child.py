"""Child process of tests/test_gpu_sensors.py::test_coop_walk_round_cap_fallback: the 16 distance sensors of the given
poses through the library named by NASCAR_LIB (a tools variant build), written to an .npy file.
    NASCAR_LIB=<variant.so> python tests/sensor_child.py <track> <E> <C> <poses.npy> <out.npy>"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from nascargymnasium_amd import _lib
    from nascargymnasium_amd.batched import BatchedCarEnv
    path, E, C, pf, of = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5]
    assert os.path.samefile(_lib.LIB_PATH, os.environ["NASCAR_LIB"])
    env = BatchedCarEnv(E, C, path, device="cuda:0")
    p = torch.from_numpy(np.load(pf)).cuda()
    obs = torch.full((env.N, 38), -7.0, dtype=torch.float32, device="cuda")
    _lib.check(env.L.nascar_debug_sensors(env.h, ctypes.c_void_p(p.data_ptr()), ctypes.c_void_p(obs.data_ptr()), 1,
                                          ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    torch.cuda.synchronize()
    np.save(of, obs.cpu().numpy())
    env.close()


if __name__ == "__main__":
    main()

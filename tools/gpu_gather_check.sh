#!/bin/bash
# gather + rollout GPU tests, then the cfg4 per-rank bench line with the trajectory gather
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_extra.py tests/test_gpu_rollout.py tests/test_gpu_api.py > gpurun_out/t_gather.log 2>&1 || exit $?
echo tests ok
timeout -k 10 300 python3 bench.py --envs 8192 --cars 4 --gather --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/b_gather.log 2>&1 || exit $?
echo gather bench ok
timeout -k 10 300 python3 bench.py --envs 8192 --cars 4 --steps 200 --warmup 20 --no-cpu-baseline --no-secondary > gpurun_out/b_cfg4.log 2>&1 || exit $?
echo cfg4 bench ok

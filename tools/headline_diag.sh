#!/bin/bash
# where the 20-step window's wall time goes (NASCAR_BENCH_DIAG: GPU span vs host enqueue vs sync)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export NASCAR_BENCH_DIAG=1
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/hd_drv.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline --no-secondary > gpurun_out/hd_200.log 2>&1 || exit $?

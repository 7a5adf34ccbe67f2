#!/bin/bash
# Round-5 baseline on a fresh box: the driver's command twice and bench.py defaults (no CPU baseline).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/r05b_drv$i.log 2>&1 || exit $?
  echo "drv$i done"
done
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-secondary > gpurun_out/r05b_200.log 2>&1 || exit $?
echo "200 done"

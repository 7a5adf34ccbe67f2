#!/bin/bash
# Headline reconciliation (round-3 verdict item 2): the driver's exact command twice, then longer windows.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/hc_drv$i.log 2>&1 || exit $?
  echo "drv$i done"
done
timeout -k 10 200 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline --no-secondary > gpurun_out/hc_200.log 2>&1 || exit $?
echo "200 done"
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --rollout 20 > gpurun_out/hc_r20.log 2>&1 || exit $?
echo "r20 done"

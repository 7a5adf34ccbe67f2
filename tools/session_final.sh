#!/bin/bash
# Round-end session: the driver's exact bench command twice on this box, then tools/gpu_session.sh (smoke, every
# GPU test, the default bench with the CPU baseline, rocprofv3 kernel stats + FETCH/WRITE + SQ passes).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/drv$i.log 2>&1 || exit $?
  echo "drv$i done"
done
TAG=${TAG:-r03} bash tools/gpu_session.sh

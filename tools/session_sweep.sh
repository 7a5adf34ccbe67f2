#!/bin/bash
# Round-end numbers: the driver's exact bench command twice, then every BASELINE config shape (tools/config_sweep.sh)
# and the SAC closed loop.  Logs -> gpurun_out/drv*.log, gpurun_out/sweep_*.log
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/drv$i.log 2>&1 || exit $?
  echo "drv$i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/drv$i.log | head -1)"
done
bash tools/config_sweep.sh || exit 1
timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --policy sac --no-secondary --no-cpu-baseline > gpurun_out/sweep_sac.log 2>&1 || exit $?
echo "sac $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sweep_sac.log | head -1)"

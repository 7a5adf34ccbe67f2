#!/bin/bash
# Round-3 session B: the driver's exact bench command twice on a fresh box, then the per-phase / per-car
# s_memtime profile (tools/libnascar_prof.so) of model_kernel on a saved steady state.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/drv$i.log 2>&1 || exit $?
  echo "drv$i done"
done
LIBS=libnascar_prof.so bash tools/gpu_phase.sh

#!/bin/bash
# GPU box, after tools/gpu_prof.sh + tools/pmc_summary.py of the same sources: the driver's command twice, the default
# bench line (drop-in, CPU baseline, secondary), then every BASELINE config shape and the SAC closed loop (200 steps)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/lines"; mkdir -p "$OUT"
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ge 124 ]; then exit "$rc"; fi; }
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/drv$i.log" 2>&1; stop $? drv$i
  echo "drv$i $(grep -o '"ms_per_step": [0-9.]*' "$OUT/drv$i.log" | head -1)"
done
timeout -k 10 400 python3 bench.py > "$OUT/default.log" 2>&1; stop $? default
echo "default $(grep -o '"ms_per_step": [0-9.]*' "$OUT/default.log" | head -1)"
run() {
  name=$1; shift
  timeout -k 10 400 python3 bench.py --steps 200 --warmup 20 --no-drop-in "$@" > "$OUT/sweep_$name.log" 2>&1; stop $? $name
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/sweep_$name.log" | head -1)"
}
run cfg2 --envs 4096 --cars 1 --no-secondary
run cfg3_talladega --track talladega --no-secondary
run cfg3_talladega_carcontact --track talladega --car-contact --no-secondary --no-cpu-baseline
run cfg4_rank --envs 8192 --cars 4 --gather --no-cpu-baseline
run cfg5_rank --envs 4096 --cars 10 --mixed --no-secondary --no-cpu-baseline
run sac --policy sac --no-secondary --no-cpu-baseline
echo lines-ok

#!/bin/bash
# GPU box: sharded rollout with more hardware queues (GPU_MAX_HW_QUEUES) and shards -- saved steady state, 200 steps
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/queues"; mkdir -p "$OUT"
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ge 124 ]; then exit "$rc"; fi; }
B="--no-cpu-baseline --no-secondary --no-drop-in"
timeout -k 10 300 python bench.py $B --steps 20 --warmup 5 --save-state /tmp/ss.pt > "$OUT/save.log" 2>&1; stop $? save
for rep in 1 2; do
for cfg in "4 4" "8 8" "6 6" "8 6" "16 8"; do
  set -- $cfg
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 200 python bench.py $B --load-state /tmp/ss.pt --steps 200 --warmup 20 --rollout-streams $2 > "$OUT/q$1_s$2_$rep.log" 2>&1; stop $? "q$1 s$2"
  echo "q$1 s$2 rep$rep $(grep -o '"ms_per_step": [0-9.]*' "$OUT/q$1_s$2_$rep.log" | head -1)"
done
done

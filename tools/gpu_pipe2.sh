#!/bin/bash
# GPU box: pipelined vs sharded rollout at smaller batches (the step kernel's workgroups all resident beside the sensors)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/pipe2"; rm -rf "$OUT"; mkdir -p "$OUT"
B="--no-cpu-baseline --no-secondary --no-drop-in"
for E in ${PIPE_ENVS:-2048 4096}; do
  timeout -k 10 300 python bench.py $B --envs $E --steps 20 --warmup 5 --save-state /tmp/ss_$E.pt > "$OUT/save_$E.log" 2>&1 || { echo "save $E failed"; exit 1; }
  for v in ${PIPE_GRIDS:-0 1024 2048}; do
    timeout -k 10 200 python bench.py $B --envs $E --load-state /tmp/ss_$E.pt --steps 50 --warmup 5 --rollout-pipe $v \
        > "$OUT/b_${E}_$v.log" 2>&1 || { echo "bench $E $v failed"; exit 1; }
    echo "envs $E pipe $v $(grep -o '"ms_per_step": [0-9.]*' "$OUT/b_${E}_$v.log" | head -1)"
  done
done

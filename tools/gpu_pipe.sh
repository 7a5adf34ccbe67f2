#!/bin/bash
# GPU box: pipelined rollout (nascar_set_rollout_pipe) -- the rollout parity tests (sharded / fused / pipelined), then the
# driver's command from one saved steady state with the sharded schedule and with the pipe at several sensor grids
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/pipe"; rm -rf "$OUT"; mkdir -p "$OUT"
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_rollout.py -k "${PIPE_TESTS:-rollout_equals_per_step}" -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > "$OUT/tests.log" 2>&1; stop $? tests
B="--no-cpu-baseline --no-secondary --no-drop-in"
timeout -k 10 300 python bench.py $B --steps 20 --warmup 5 --save-state /tmp/ss.pt > "$OUT/save.log" 2>&1; stop $? save
for v in ${PIPE_GRIDS:-0 512 1024 2048 0 512 1024 2048}; do
  timeout -k 10 200 python bench.py $B --load-state /tmp/ss.pt --steps ${PIPE_STEPS:-20} --warmup 5 --rollout-pipe $v \
      > "$OUT/b_$v.log" 2>&1; stop $? "bench $v"
  echo "pipe $v $(grep -o '"ms_per_step": [0-9.]*' "$OUT/b_$v.log" | head -1)"
done

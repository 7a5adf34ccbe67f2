#!/bin/bash
# Every BASELINE.json config shape on one GPU (per-rank shapes for the 8-GPU configs), steady-state workload,
# CPU baseline of the same config in the same run.  Lines -> gpurun_out/sweep_<name>.log
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$ROOT/gpurun_out"
run() {
  name=$1; shift
  timeout -k 10 400 python "$ROOT/bench.py" --steps 200 --warmup 20 "$@" > "$ROOT/gpurun_out/sweep_$name.log" 2>&1 || { echo "$name rc=$?"; return 1; }
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$ROOT/gpurun_out/sweep_$name.log")"
}
run cfg3_daytona --no-secondary ${SWEEP_ARGS} || exit 1
run cfg2 --envs 4096 --cars 1 --no-secondary ${SWEEP_ARGS} || exit 1
run cfg3_talladega --track talladega --no-secondary ${SWEEP_ARGS} || exit 1
run cfg3_talladega_carcontact --track talladega --car-contact --no-secondary --no-cpu-baseline ${SWEEP_ARGS} || exit 1
run cfg4_rank --envs 8192 --cars 4 --gather --no-cpu-baseline ${SWEEP_ARGS} || exit 1
run cfg5_rank --envs 4096 --cars 10 --mixed --no-secondary --no-cpu-baseline ${SWEEP_ARGS} || exit 1

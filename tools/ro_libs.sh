#!/bin/bash
# Fused-rollout timing per library (NASCAR_LIB) from one settled steady state: tools/ro_libs.sh R ab/a.so ...
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$ROOT/gpurun_out"
R=$1; shift
timeout -k 10 300 python "$ROOT/bench.py" --save-state /tmp/nascar_ss.pt --no-cpu-baseline --no-secondary --steps 100 \
    > "$ROOT/gpurun_out/ro_settle.log" 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' "$ROOT/gpurun_out/ro_settle.log"
for L in "$@"; do
  tag=$(basename "$L" .so)
  NASCAR_LIB="$ROOT/$L" timeout -k 10 200 python "$ROOT/bench.py" --load-state /tmp/nascar_ss.pt --rollout $R --steps 200 \
      --warmup 10 --no-cpu-baseline --no-secondary > "$ROOT/gpurun_out/ro_$tag.log" 2>&1 || { echo "$tag failed"; exit 1; }
  echo "$tag $(grep -o '"ms_per_step": [0-9.]*' "$ROOT/gpurun_out/ro_$tag.log")"
done

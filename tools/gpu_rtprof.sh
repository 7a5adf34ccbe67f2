#!/bin/bash
# GPU box: rocprofv3 kernel stats of a bench run whose drop-in pass times random-track mode (rt_switch_kernel,
# block_map_kernel, vec_post_kernel, action_check_kernel per launch)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/rtprof"; rm -rf "$OUT"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > "$OUT/bench.log" 2>&1
echo "rc=$?"
rm -f "$OUT/kt/run_kernel_trace.csv"
tail -5 "$OUT/bench.log"

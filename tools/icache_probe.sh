#!/bin/bash
# instruction-cache hit rate per kernel (SQC_ICACHE_HITS / SQC_ICACHE_MISSES, one pass) on the per-step and the
# sharded schedule, from a saved steady state
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/ic"; rm -rf "$OUT"; mkdir -p "$OUT"
timeout -k 10 200 python bench.py --save-state /tmp/nascar_ss.pt --no-cpu-baseline --no-secondary --steps 20 --warmup 5 \
  > "$OUT/save.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for mode in 0 50; do
  timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --kernel-trace --output-format csv -d "$OUT/p$mode" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --load-state /tmp/nascar_ss.pt --no-cpu-baseline --no-secondary --steps 10 --warmup 2 \
    --rollout $mode > "$OUT/p$mode.log" 2>&1 || { echo "pmc rc=$?"; exit 1; }
  python3 "$GRAFT_REPO_ROOT/tools/sq_summary.py" "$OUT/p$mode" | sed "s/^/rollout=$mode /"
done

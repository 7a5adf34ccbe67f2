#!/bin/bash
# round-4 final profiles: the default bench + rocprofv3 kernel stats / PMC passes on its saved steady state
# (tools/gpu_session.sh, TAG=r04), then cfg2 (4096 x 1) under rocprofv3 --kernel-trace --stats.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
SKIP_TESTS=1 TAG=r04 bash tools/gpu_session.sh || exit $?
cd /tmp && export TMPDIR=/tmp
rm -rf "$OUT/prof_cfg2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg2" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --envs 4096 --cars 1 --steps 200 --warmup 20 --no-cpu-baseline --no-secondary \
    > "$OUT/prof_cfg2.log" 2>&1 || exit $?
echo r04-prof-ok

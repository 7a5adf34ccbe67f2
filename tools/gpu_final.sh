#!/bin/bash
# A round's final measurements on one GPU box (gpurun): the driver's bench command (ROUNDS runs), the default bench
# with its saved steady state, rocprofv3 kernel stats + FETCH/WRITE + SQ passes on that state (tools/gpu_session.sh),
# and cfg2 (4096 x 1) under rocprofv3 --kernel-trace --stats.  Summaries: python tools/pmc_summary.py gpurun_out/prof TAG
#   TAG=r05 bash tools/gpu_final.sh
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG="${TAG:-r05}"
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ge 124 ]; then exit "$rc"; fi; }
for r in $(seq 1 ${ROUNDS:-2}); do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > "$OUT/driver_cmd_$r.log" 2>&1; stop $? "driver's command $r"
  tail -1 "$OUT/driver_cmd_$r.log"
done
SKIP_TESTS=1 TAG=$TAG bash tools/gpu_session.sh || exit $?
tail -1 "$OUT/bench.log"
cd /tmp && export TMPDIR=/tmp
rm -rf "$OUT/prof_cfg2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg2" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --envs 4096 --cars 1 --steps 200 --warmup 20 --no-cpu-baseline --no-secondary \
    > "$OUT/prof_cfg2.log" 2>&1; stop $? cfg2
tail -1 "$OUT/prof_cfg2.log"
echo final-ok

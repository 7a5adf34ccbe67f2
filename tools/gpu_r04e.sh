#!/bin/bash
# round-4 session E: parity of the in-model sensor pass (parity / rollout / full-episode tests), then the driver's
# command A/B: previous build (tools/ab_base.so) vs the sensor pass inside model_kernel (tools/ab_sens.so).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ge 124 ]; then exit "$rc"; fi; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; stop $? smoke
[ "$rc" = 0 ] || exit 1
timeout -k 10 800 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_rollout.py} -m gpu -x -v --timeout 240 \
    --timeout-method thread -p no:cacheprovider > "$OUT/gpu_tests_e.log" 2>&1; stop $? tests
tail -3 "$OUT/gpu_tests_e.log"
ROUNDS=${ROUNDS:-2} bash tools/ab3.sh ${LIBS:-tools/ab_base.so tools/ab_sens.so}

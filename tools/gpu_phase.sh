#!/bin/bash
# Steady-state phase profile session: settle once (bench --save-state), then per-phase s_memtime profiles of
# prebuilt profile libraries (LIBS, tools/*.so) on that state, then optional parity tests (TESTS).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ge 124 ]; then exit "$rc"; fi; }
timeout -k 10 300 python bench.py --save-state /tmp/nascar_ss.pt --no-cpu-baseline --no-secondary --steps 100 $BENCH_ARGS \
    > "$OUT/phase_bench.log" 2>&1; stop $? bench
for L in ${LIBS:-libnascar_prof.so}; do
  C=""; case "$L" in *cnt*) C="--count";; esac
  timeout -k 10 200 python tools/phase_profile.py --no-build --lib "$L" $C --load-state /tmp/nascar_ss.pt --warmup 20 --steps 2 $PHASE_ARGS \
      > "$OUT/phase_${L%.so}.log" 2>&1; stop $? "phase $L"
done
if [ -n "$TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest $TESTS -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
      > "$OUT/gpu_tests.log" 2>&1; stop $? tests
fi
echo phase-ok

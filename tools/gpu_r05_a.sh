#!/bin/bash
# round 5 session A: smoke, the new full-size schedule test + sensor workgroup test, then a steady-state phase profile
# (tools/libnascar_prof.so, -DNASCAR_PROFILE) with the post-event rescan counters.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ge 124 ]; then exit "$rc"; fi; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/r05_smoke.log" 2>&1; stop $? smoke
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_configs.py::test_bench_steady_state_full_size_vs_oracle tests/test_gpu_sensors.py::test_sensor_workgroup_sizes_identical \
  > "$OUT/r05_sel1.log" 2>&1; stop $? tests
tail -3 "$OUT/r05_sel1.log"
PHASE_ARGS="--steps 3" LIBS=libnascar_prof.so bash tools/gpu_phase.sh

#!/bin/bash
# GPU box session: host facts, smoke, the GPU test suite with per-test durations, then the driver's bench command.
#   TESTS="tests/test_x.py" (default tests) / SKIP_BENCH=1 / PYTEST_ARGS="-k ..."
# A fault, abort or time limit (rc >= 124) ends the session; ordinary test failures do not.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TESTS="${TESTS:-tests}"
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ge 124 ]; then exit "$rc"; fi; }
{ echo "nproc $(nproc) affinity $(python3 -c 'import os; print(len(os.sched_getaffinity(0)))') OMP_NUM_THREADS=$OMP_NUM_THREADS";
  cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo; } > "$OUT/host.txt"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; stop $? smoke
timeout -k 10 1300 python -u -m pytest $TESTS -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
    --durations=60 $PYTEST_ARGS > "$OUT/gpu_tests.log" 2>&1; stop $? tests
[ -n "$SKIP_BENCH" ] && exit 0
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_drv.log" 2>&1; stop $? bench

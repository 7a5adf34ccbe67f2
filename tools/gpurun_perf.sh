#!/bin/bash
# GPU perf iteration: smoke (parity) -> phase profile -> short bench -> rocprofv3 kernel stats.
# Stops at the first failure.  Optional: TESTS=1 also runs pytest -m gpu first.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; exit 1; }
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed rc=$?"; exit 1; }
fi
timeout -k 10 300 python tools/phase_profile.py --no-build $PHASE_ARGS > gpurun_out/phase.log 2>&1 || { echo "phase failed rc=$?"; exit 1; }
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { echo "bench failed rc=$?"; exit 1; }
rm -rf gpurun_out/kt && cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/kt" -o run -- \
    python3 "$ROOT/bench.py" --steps 50 --warmup 5 --no-cpu-baseline > "$ROOT/gpurun_out/kt.log" 2>&1 || { echo "rocprof failed rc=$?"; exit 1; }
echo perf-ok

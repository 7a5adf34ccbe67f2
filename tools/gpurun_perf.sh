#!/bin/bash
# GPU perf iteration: smoke (parity) -> phase profile -> short bench.  Stops at the first failure.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; exit 1; }
timeout -k 10 300 python tools/phase_profile.py --no-build $PHASE_ARGS > gpurun_out/phase.log 2>&1 || { echo "phase failed rc=$?"; exit 1; }
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { echo "bench failed rc=$?"; exit 1; }
echo perf-ok

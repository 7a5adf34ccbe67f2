#!/bin/bash
# GPU box: smoke, then the whole GPU test suite (per-test durations), no bench.  A fault / abort / time limit ends it.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ge 124 ]; then exit "$rc"; fi; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; stop $? smoke
timeout -k 10 1050 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider \
    --durations=40 $PYTEST_ARGS > "$OUT/gpu_tests.log" 2>&1; stop $? tests

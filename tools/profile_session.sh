#!/bin/bash
# GPU profiling session (run through gpurun):
#   1. rocprofv3 --kernel-trace --stats of the default bench workload
#   2. separate PMC passes (FETCH_SIZE, then WRITE_SIZE) with --kernel-trace only
#   3. tools/pmc_summary.py -> gpurun_out/prof/summary.json + profiles/pmc_traffic.json
# Each GPU step has its own time limit; the script stops at the first failure.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/prof"
TAG="${1:-r01}"
STEPS="${STEPS:-50}"
BENCH_ARGS="${BENCH_ARGS:-}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- \
    python3 "$ROOT/bench.py" --steps "$STEPS" --warmup 5 --no-cpu-baseline $BENCH_ARGS > "$OUT/kt.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline $BENCH_ARGS > "$OUT/fetch.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline $BENCH_ARGS > "$OUT/write.log" 2>&1 || exit $?
echo "profile-ok: run python tools/pmc_summary.py gpurun_out/prof $TAG locally"

#!/bin/bash
# Round-3 profiling session (through gpurun): settle once and save the steady state (no profiler), then from it
#   1. rocprofv3 --kernel-trace --stats of the bench (the driver's --steps 20 --warmup 5)
#   2. separate PMC passes FETCH_SIZE, WRITE_SIZE (--kernel-trace only)
# then locally: python tools/pmc_summary.py gpurun_out/prof r03
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/prof"; rm -rf "$OUT"; mkdir -p "$OUT"
python3 -c "import sys; sys.path.insert(0, '$ROOT'); import bench; print(bench.source_sha())" > "$ROOT/gpurun_out/prof_source_sha.txt"
timeout -k 10 200 python3 "$ROOT/bench.py" --save-state /tmp/nascar_ss.pt --steps 20 --warmup 5 --no-cpu-baseline --no-secondary \
  > "$OUT/save.log" 2>&1 || exit $?
ARGS="--load-state /tmp/nascar_ss.pt --steps 20 --warmup 5 --no-cpu-baseline --no-secondary"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- \
    python3 "$ROOT/bench.py" $ARGS > "$OUT/kt.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run -- \
    python3 "$ROOT/bench.py" $ARGS > "$OUT/fetch.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run -- \
    python3 "$ROOT/bench.py" $ARGS > "$OUT/write.log" 2>&1 || exit $?
echo "profile-ok"

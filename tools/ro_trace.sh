#!/bin/bash
# kernel trace of the driver's bench command from a saved steady state, then tools/ro_trace.py on the timed call
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/rotrace"; rm -rf "$OUT"; mkdir -p "$OUT"
timeout -k 10 200 python3 "$ROOT/bench.py" --save-state /tmp/nascar_ss.pt --steps 20 --warmup 5 --no-cpu-baseline --no-secondary \
  > "$OUT/save.log" 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt" -o run -- \
  python3 "$ROOT/bench.py" --load-state /tmp/nascar_ss.pt --steps 20 --warmup 5 --no-cpu-baseline --no-secondary $BENCH_EXTRA \
  > "$OUT/bench.log" 2>&1 || exit $?
python3 "$ROOT/tools/ro_trace.py" "$OUT/kt" > "$OUT/summary.txt" && cat "$OUT/summary.txt"

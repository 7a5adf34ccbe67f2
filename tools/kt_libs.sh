#!/bin/bash
# Per-kernel average durations (rocprofv3 --kernel-trace --stats) of the default bench for each library
# given (NASCAR_LIB); no parity check, so experimental / deliberately-wrong variants can be timed.
#   tools/kt_libs.sh tools/a.so tools/b.so ...      (BENCH_ARGS adds bench.py options)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$ROOT/gpurun_out"
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  tag=$(basename "$L" .so)
  rm -rf "$ROOT/gpurun_out/kt_$tag"
  NASCAR_LIB="$ROOT/$L" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/kt_$tag" -o run -- \
      python3 "$ROOT/bench.py" --steps 50 --warmup 10 --no-cpu-baseline $BENCH_ARGS > "$ROOT/gpurun_out/kt_$tag.log" 2>&1 || { echo "$tag failed"; exit 1; }
  python3 - "$ROOT/gpurun_out/kt_$tag" "$tag" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "at::" not in r["Name"]]
print(sys.argv[2], "  ".join(f"{r['Name'].split('(')[0].replace('void ', '')[:20]}={float(r['AverageNs'])/1000:.1f}us" for r in rows))
PY
done

#!/bin/bash
# Per-kernel average durations at the steady state: settle once with the default library (bench --save-state),
# then rocprofv3 --kernel-trace --stats of 50 steps from that state for each library given (NASCAR_LIB).
#   tools/kt_ss.sh ab/a.so ab/b.so,NASCAR_RBLOCK=128 ...   (",VAR=VAL" entries: environment for that run only)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$ROOT/gpurun_out"
timeout -k 10 300 python "$ROOT/bench.py" --save-state /tmp/nascar_ss.pt --no-cpu-baseline --no-secondary --steps 20 $BENCH_ARGS \
    > "$ROOT/gpurun_out/kt_ss_settle.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for spec in "$@"; do
  IFS=, read -r L envs <<< "$spec"
  tag=$(basename "$L" .so)${envs:+_${envs//[^A-Za-z0-9]/}}
  rm -rf "$ROOT/gpurun_out/kt_$tag"
  env ${envs//,/ } NASCAR_LIB="$ROOT/$L" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/kt_$tag" -o run -- \
      python3 "$ROOT/bench.py" --load-state /tmp/nascar_ss.pt --steps 50 --warmup 5 --no-cpu-baseline --no-secondary $BENCH_ARGS \
      > "$ROOT/gpurun_out/kt_$tag.log" 2>&1 || { echo "$tag failed"; exit 1; }
  python3 - "$ROOT/gpurun_out/kt_$tag" "$tag" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "at::" not in r["Name"]]
print(sys.argv[2], "  ".join(f"{r['Name'].split('(')[0].replace('void ', '')[:20]}={float(r['AverageNs'])/1000:.1f}us" for r in rows))
PY
  grep -o '"ms_per_step": [0-9.]*' "$ROOT/gpurun_out/kt_$tag.log"
  rm -rf "$ROOT/gpurun_out/kt_$tag"
done

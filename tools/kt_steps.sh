#!/bin/bash
# per-kernel durations on the per-step path (whole-grid launches): rocprofv3 --kernel-trace of bench.py --rollout 0,
# summarised as mean / p50 / max per kernel.  Usage: tools/kt_steps.sh TAG [lib.so]
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; LIB=${2:-}
OUT="$ROOT/gpurun_out/kt_$TAG"; rm -rf "$OUT"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
[ -n "$LIB" ] && export NASCAR_LIB="$ROOT/$LIB"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o run -- \
  python3 "$ROOT/bench.py" --rollout 0 --steps 100 --warmup 10 --no-cpu-baseline --no-secondary > "$OUT/bench.log" 2>&1 || exit $?
python3 - "$OUT" "$TAG" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    d[r["Kernel_Name"].split("(")[0]].append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000))
import statistics as st
for k in ("model_kernel", "logic_kernel", "ray_sensor_kernel"):
    v = [x for _, x in sorted(d.get(k, [(0, 0.0)]))[-150:]]   # the timed window + stats pass (time order)
    print(sys.argv[2], k, f"n {len(d.get(k, []))} mean {st.mean(v):.1f} p50 {st.median(v):.1f} max {max(v):.1f} us")
PY

#!/bin/bash
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  tag=$(basename "$L" .so)
  rm -rf "$ROOT/gpurun_out/kt_$tag"
  NASCAR_LIB="$ROOT/$L" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/kt_$tag" -o run -- python3 "$ROOT/bench.py" --steps 100 --warmup 10 --no-cpu-baseline > "$ROOT/gpurun_out/kt_$tag.log" 2>&1 || exit 1
  python3 - "$ROOT/gpurun_out/kt_$tag" "$tag" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
out = []
for r in csv.DictReader(open(f)):
    n = r["Name"].split("(")[0]
    if n in ("ray_sensor_kernel", "model_kernel", "logic_kernel"):
        out.append(f"{n[:6]} {float(r['AverageNs'])/1000:.1f}")
print(sys.argv[2], " ".join(out))
PY
done

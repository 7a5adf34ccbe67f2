#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per kernel (KiB per dispatch, gfx950: FETCH tallies half) for each library at the steady state
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$ROOT/gpurun_out"
[ -f /tmp/nascar_ss.pt ] || timeout -k 10 300 python "$ROOT/bench.py" --save-state /tmp/nascar_ss.pt --no-cpu-baseline --no-secondary --steps 20 > "$ROOT/gpurun_out/pmc_settle.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  tag=$(basename "$L" .so)
  for C in FETCH_SIZE WRITE_SIZE; do
    rm -rf "$ROOT/gpurun_out/pmc_$tag"
    NASCAR_LIB="$ROOT/$L" timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$ROOT/gpurun_out/pmc_$tag" -o run -- \
        python3 "$ROOT/bench.py" --load-state /tmp/nascar_ss.pt --steps 10 --warmup 2 --no-cpu-baseline --no-secondary > /dev/null 2>&1 || { echo "$tag $C failed"; exit 1; }
    python3 - "$ROOT/gpurun_out/pmc_$tag" "$tag" "$C" <<'PY'
import csv, glob, sys
from collections import defaultdict
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = defaultdict(list)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0]
    if k in ("model_kernel", "logic_kernel", "ray_sensor_kernel"):
        acc[k].append(float(r["Counter_Value"]))
print(sys.argv[2], sys.argv[3], "  ".join(f"{k}={sum(v)/len(v):.0f}KiB" for k, v in sorted(acc.items())))
PY
    rm -rf "$ROOT/gpurun_out/pmc_$tag"
  done
done

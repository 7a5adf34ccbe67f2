#!/bin/bash
# Knockout timing attribution: settle once with the shipped library and save the steady state, then per library
# (built with -DNASCAR_KO_* -- a phase skipped, wrong results, timing only) time 20 per-step-path steps from that
# state under rocprofv3 --kernel-trace and print each kernel's mean duration.  Usage: tools/ko_session.sh a.so b.so ...
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/ko"; rm -rf "$OUT"; mkdir -p "$OUT"
timeout -k 10 200 python3 "$ROOT/bench.py" --save-state /tmp/nascar_ss.pt --steps 20 --warmup 5 --no-cpu-baseline --no-secondary \
  > "$OUT/save.log" 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  tag=$(basename "$L" .so)
  NASCAR_LIB="$ROOT/$L" timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$tag" -o run -- \
    python3 "$ROOT/bench.py" --load-state /tmp/nascar_ss.pt --rollout 0 --steps 20 --warmup 2 --no-cpu-baseline --no-secondary \
    > "$OUT/$tag.log" 2>&1 || { echo "$tag failed"; exit 1; }
  python3 - "$OUT/$tag" "$tag" <<'PY'
import csv, glob, sys, collections, statistics as st
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    d[r["Kernel_Name"].split("(")[0].replace("void ", "")].append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000))
out = []
for k in ("model_kernel", "logic_kernel", "ray_sensor_kernel"):
    v = [x for _, x in sorted(d.get(k, [(0, 0.0)]))][2:22]
    out.append(f"{k} {st.mean(v):.1f} (p50 {st.median(v):.1f}, max {max(v):.1f})")
print(sys.argv[2], " | ".join(out))
PY
done

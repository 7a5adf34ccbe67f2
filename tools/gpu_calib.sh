#!/bin/bash
# GPU box: FETCH_SIZE / WRITE_SIZE calibration passes (tools/fetch_calib.py), one counter per pass
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/calib"; rm -rf "$OUT"; mkdir -p "$OUT"
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ge 124 ]; then exit "$rc"; fi; }
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/$C" -o run -- \
    python3 "$GRAFT_REPO_ROOT/tools/fetch_calib.py" > "$OUT/$C.log" 2>&1; stop $? $C
  rm -f "$OUT"/$C/*kernel_trace.csv
done
python3 "$GRAFT_REPO_ROOT/tools/fetch_calib.py" --summary "$OUT/FETCH_SIZE" "$OUT/WRITE_SIZE" | tee "$OUT/summary.txt"

#!/bin/bash
# GPU box A/B: round-5 tree vs variants of this one (tools/build/*.so via NASCAR_LIB), the driver's command, 3 rounds
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/abr05b"; mkdir -p "$OUT"
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ge 124 ]; then exit "$rc"; fi; }
N="--steps 20 --warmup 5 --no-cpu-baseline --no-secondary"
for r in 1 2 3; do
  timeout -k 10 300 python3 tools/r05_full/bench.py $N > "$OUT/r05_$r.log" 2>&1; stop $? r05
  echo "r05 $r $(grep -o '"ms_per_step": [0-9.]*' "$OUT/r05_$r.log" | head -1)"
  for v in prodab ng ngcc; do
    NASCAR_LIB=tools/build/libnascar_$v.so timeout -k 10 300 python3 bench.py $N --no-drop-in > "$OUT/${v}_$r.log" 2>&1; stop $? $v
    echo "$v $r $(grep -o '"ms_per_step": [0-9.]*' "$OUT/${v}_$r.log" | head -1)"
  done
done

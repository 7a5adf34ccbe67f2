#!/bin/bash
# GPU box A/B: the round-5 tree (tools/r05_full: git archive 8194fc8, its own bench.py and libnascar.so) against this
# tree, the driver's command alternating, 3 rounds (no CPU baseline / secondary / drop-in)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/abr05"; mkdir -p "$OUT"
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ge 124 ]; then exit "$rc"; fi; }
for r in 1 2 3; do
  timeout -k 10 300 python3 tools/r05_full/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > "$OUT/r05_$r.log" 2>&1; stop $? r05
  echo "r05 $r $(grep -o '"ms_per_step": [0-9.]*' "$OUT/r05_$r.log" | head -1)"
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-drop-in > "$OUT/r06_$r.log" 2>&1; stop $? r06
  echo "r06 $r $(grep -o '"ms_per_step": [0-9.]*' "$OUT/r06_$r.log" | head -1)"
done

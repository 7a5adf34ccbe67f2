#!/bin/bash
# GPU box A/B of library builds (tools/build/libnascar_<variant>.so, VARIANTS="a b ..."): per variant the step
# kernels' mean dispatch times (rocprofv3 --stats), their HBM bytes per car (FETCH_SIZE x2 + WRITE_SIZE), and the
# driver's command twice, all from one saved steady state
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/ablib"; rm -rf "$OUT"; mkdir -p "$OUT"
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ge 124 ]; then exit "$rc"; fi; }
B="--no-cpu-baseline --no-secondary --no-drop-in"
timeout -k 10 300 python bench.py $B --steps 20 --warmup 5 --save-state /tmp/ss.pt > "$OUT/save.log" 2>&1; stop $? save
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-base xcd}; do
  L=$GRAFT_REPO_ROOT/tools/build/libnascar_$v.so
  NASCAR_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt$v" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" $B --load-state /tmp/ss.pt --steps 50 --warmup 5 > "$OUT/kt$v.log" 2>&1; stop $? kt$v
  rm -f "$OUT"/kt$v/*kernel_trace.csv
  for C in FETCH_SIZE WRITE_SIZE; do
    NASCAR_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/p${v}_$C" -o run -- \
      python3 "$GRAFT_REPO_ROOT/bench.py" $B --load-state /tmp/ss.pt --steps 10 --warmup 2 > "$OUT/p${v}_$C.log" 2>&1; stop $? p$v$C
    rm -f "$OUT"/p${v}_$C/*kernel_trace.csv
  done
  for r in 1 2; do
    NASCAR_LIB=$L timeout -k 10 200 python3 "$GRAFT_REPO_ROOT/bench.py" $B --load-state /tmp/ss.pt --steps 20 --warmup 5 > "$OUT/drv${v}_$r.log" 2>&1; stop $? drv$v
    echo "$v drv$r $(grep -o '"ms_per_step": [0-9.]*' "$OUT/drv${v}_$r.log" | head -1)"
  done
done
python3 "$GRAFT_REPO_ROOT/tools/ab_lg_summary.py" "$OUT"

#!/bin/bash
# GPU box: the driver's bench command, the default bench (drop-in + CPU baseline), cfg5's rank shape with interleaved
# (product) and contiguous (tools A/B lib) shards, and a kernel trace of each cfg5 rollout call (tools/ro_trace.py).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ge 124 ]; then exit "$rc"; fi; }
export NASCAR_TRACK_CACHE=/tmp/nascar_tc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/b_drv.log" 2>&1; stop $? drv
timeout -k 10 400 python bench.py > "$OUT/b_def.log" 2>&1; stop $? default
C5="--envs 4096 --cars 10 --mixed --steps 200 --warmup 20 --no-secondary --no-cpu-baseline"
timeout -k 10 300 python bench.py $C5 > "$OUT/cfg5_new.log" 2>&1; stop $? cfg5_new
NASCAR_LIB=tools/build/libnascar_ab.so NASCAR_MAP_CONTIGUOUS=1 timeout -k 10 300 python bench.py $C5 > "$OUT/cfg5_old.log" 2>&1; stop $? cfg5_old
timeout -k 10 300 python bench.py --envs 4096 --cars 10 --mixed --steps 20 --warmup 5 --no-secondary --no-cpu-baseline --save-state /tmp/c5.pt > "$OUT/c5_save.log" 2>&1; stop $? c5save
cd /tmp && export TMPDIR=/tmp
for v in new old; do
  if [ $v = old ]; then export NASCAR_LIB=$GRAFT_REPO_ROOT/tools/build/libnascar_ab.so NASCAR_MAP_CONTIGUOUS=1; fi
  rm -rf "$OUT/rt_$v"; mkdir -p "$OUT/rt_$v"
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/rt_$v/kt" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --envs 4096 --cars 10 --mixed --load-state /tmp/c5.pt --steps 100 --warmup 50 --no-cpu-baseline --no-secondary \
    > "$OUT/rt_$v/bench.log" 2>&1; stop $? trace_$v
  python3 "$GRAFT_REPO_ROOT/tools/ro_trace.py" "$OUT/rt_$v/kt" > "$OUT/rt_$v/summary.txt" 2>&1; stop $? summ_$v
done

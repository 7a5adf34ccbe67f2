#!/bin/bash
# round 5 session B: capture the steady state's b2TimeOfImpact jobs (profile build), micro-benchmark toi_alpha variants
# on them (tools/toi_bench.py), then A/B whole libraries on the driver's command (tools/ab3.sh).
#   BENCH_LIBS="tools/toi_bench_base.so ..."  AB_LIBS="ab/prod.so ab/x.so"
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ge 124 ]; then exit "$rc"; fi; }
if [ ! -f "$OUT/toi_jobs.npy" ] || [ -n "$RECAPTURE" ]; then
  timeout -k 10 300 python bench.py --save-state /tmp/nascar_ss.pt --no-cpu-baseline --no-secondary --steps 20 \
      > "$OUT/b_settle.log" 2>&1; stop $? settle
  timeout -k 10 200 python tools/phase_profile.py --no-build --lib libnascar_cap.so --load-state /tmp/nascar_ss.pt \
      --warmup 10 --steps 10 --capture "$OUT/toi_jobs.npy" > "$OUT/b_capture.log" 2>&1; stop $? capture
fi
timeout -k 10 200 python tools/toi_bench.py --jobs "$OUT/toi_jobs.npy" --libs ${BENCH_LIBS} > "$OUT/b_toibench.log" 2>&1; stop $? toibench
cat "$OUT/b_toibench.log"
if [ -n "$AB_LIBS" ]; then
  ROUNDS=${ROUNDS:-2} bash tools/ab3.sh $AB_LIBS; stop $? ab3
fi

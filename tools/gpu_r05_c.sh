#!/bin/bash
# round 5 session C: latency calibration (sincos variants), TOI micro-benchmark variants, the sharded step's kernel
# timeline (rocprofv3 kernel trace -> tools/ro_trace.py), then whole-library A/B on the driver's command.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ge 124 ]; then exit "$rc"; fi; }
{ timeout -k 10 60 python tools/lat_bench.py tools/lat_bench_sc1.so && timeout -k 10 60 python tools/lat_bench.py tools/lat_bench_sc2.so; } > "$OUT/c_lat.log" 2>&1; stop $? lat
timeout -k 10 200 python tools/toi_bench.py --jobs tools/data/toi_jobs_r05.npy --libs ${BENCH_LIBS} --lanes 1 64 --blocks 1 \
    > "$OUT/c_toibench.log" 2>&1; stop $? toibench
if [ -n "$TRACE" ]; then bash tools/ro_trace.sh > "$OUT/c_rotrace.log" 2>&1; stop $? rotrace; fi
if [ -n "$AB_LIBS" ]; then ROUNDS=${ROUNDS:-3} bash tools/ab3.sh $AB_LIBS > "$OUT/c_ab3.log" 2>&1; stop $? ab3; fi
cat "$OUT/c_lat.log" "$OUT/c_toibench.log" "$OUT/c_ab3.log" 2>/dev/null | grep -v amdgpu.ids

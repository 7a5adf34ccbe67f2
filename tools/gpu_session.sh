#!/bin/bash
# One GPU session (run through gpurun): smoke -> gpu parity tests -> default bench (saves the settled
# steady state) -> rocprofv3 kernel stats + FETCH/WRITE + SQ passes on that saved state.
#   SKIP_TESTS=1 / SKIP_PROF=1 / TESTS="tests/test_x.py" / TAG=r02
# A fault, abort or time limit (rc >= 124) ends the session; ordinary test failures do not.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG="${TAG:-r02}"
TESTS="${TESTS:-tests}"
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ge 124 ]; then exit "$rc"; fi; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; stop $? smoke
  timeout -k 10 1000 python -u -m pytest $TESTS -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
      > "$OUT/gpu_tests.log" 2>&1; stop $? tests
fi
timeout -k 10 400 python bench.py --save-state /tmp/nascar_ss.pt $BENCH_ARGS > "$OUT/bench.log" 2>&1; stop $? bench
[ -n "$SKIP_PROF" ] && exit 0
[ -f /tmp/nascar_ss.pt ] || exit 1
P="$GRAFT_REPO_ROOT/bench.py --load-state /tmp/nascar_ss.pt --no-cpu-baseline --no-secondary $BENCH_ARGS"
python -c "import bench; print(bench.source_sha())" > "$OUT/prof_source_sha.txt"
cd /tmp && export TMPDIR=/tmp
rm -rf "$OUT/prof" && mkdir -p "$OUT/prof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof/kt" -o run -- \
    python3 $P --steps 100 --warmup 5 > "$OUT/prof/kt.log" 2>&1; stop $? kt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/prof/fetch" -o run -- \
    python3 $P --steps 10 --warmup 2 > "$OUT/prof/fetch.log" 2>&1; stop $? fetch
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/prof/write" -o run -- \
    python3 $P --steps 10 --warmup 2 > "$OUT/prof/write.log" 2>&1; stop $? write
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
    --kernel-trace --output-format csv -d "$OUT/prof/sq" -o run -- python3 $P --steps 10 --warmup 2 > "$OUT/prof/sq.log" 2>&1; stop $? sq
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD \
    --kernel-trace --output-format csv -d "$OUT/prof/sq2" -o run -- python3 $P --steps 10 --warmup 2 > "$OUT/prof/sq2.log" 2>&1; stop $? sq2
echo "session-ok: python tools/pmc_summary.py gpurun_out/prof $TAG"

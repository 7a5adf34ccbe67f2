#!/bin/bash
# round-4 session D: the default bench (saves the settled steady state) + rocprofv3 kernel stats / PMC passes on it
# (tools/gpu_session.sh, TAG=r04), the per-phase profile of the product build on the same state, then the driver's
# command with the fused model + logic kernel vs the two-launch product (2 rounds), and cfg2 (4096 x 1) at its
# automatic layout.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ge 124 ]; then exit "$rc"; fi; }
if [ -n "$TESTS" ]; then   # the GPU tests first (ordinary failures do not stop the session)
  timeout -k 10 700 python -u -m pytest $TESTS -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
      --durations=30 > "$OUT/gpu_tests_d.log" 2>&1; stop $? tests
fi
if [ "${PART:-12}" != 2 ]; then
  SKIP_TESTS=1 TAG=r04 bash tools/gpu_session.sh || exit $?
  cd "$GRAFT_REPO_ROOT" || exit 1
fi
[ "${PART:-12}" = 1 ] && { echo r04d-part1-ok; exit 0; }
[ -f /tmp/nascar_ss.pt ] || { timeout -k 10 300 python bench.py --save-state /tmp/nascar_ss.pt --no-cpu-baseline --no-secondary \
    --steps 20 > "$OUT/bench_ss.log" 2>&1; stop $? bench-ss; }
timeout -k 10 200 python tools/phase_profile.py --no-build --lib libprof_cnt.so --count --load-state /tmp/nascar_ss.pt \
    --warmup 20 --steps 2 > "$OUT/phase_cnt.log" 2>&1; stop $? phase
for r in 1 2; do
  for F in 0 1; do
    NASCAR_FUSE_ML=$F timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary \
      > "$OUT/ab_fuse${F}_$r.log" 2>&1 || exit $?
    python -c "import json;d=json.loads(open('$OUT/ab_fuse${F}_$r.log').read().strip().splitlines()[-1]);print('fuse$F', $r, round(d['value']/1e6,1), 'M car-steps/s', round(d['ms_per_step']*1000,1), 'us/step', {k: round(v*1000,1) for k, v in d['roofline']['kernel_times_ms'].items()})"
  done
done
timeout -k 10 200 python bench.py --envs 4096 --cars 1 --steps 200 --warmup 20 --no-cpu-baseline --no-secondary \
  > "$OUT/cfg2.log" 2>&1 || exit $?
python -c "import json;d=json.loads(open('$OUT/cfg2.log').read().strip().splitlines()[-1]);print('cfg2', round(d['value']/1e6,1), 'M car-steps/s', round(d['ms_per_step']*1000,1), 'us/step', {k: round(v*1000,1) for k, v in d['roofline']['kernel_times_ms'].items()})"
echo r04d-ok

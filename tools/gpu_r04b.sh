#!/bin/bash
# round-4 session B: phase profiles (general island in scratch vs LDS; unrolled/inlined vs rolled/outlined code) on
# one saved steady state, single-env replays of the busiest envs, instruction-cache counters, the driver's command
# A/B of the library variants, and cfg2 with 16 vs 4 sensor lanes per car.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ge 124 ]; then exit "$rc"; fi; }
LIBS="libprof_ilds0.so libprof_base.so libprof_small.so" bash tools/gpu_phase.sh || exit $?
for L in libprof_base.so libprof_small.so; do
  timeout -k 10 120 python tools/env_replay.py --load-state /tmp/nascar_ss.pt --lib $L --auto 6 --steps 3 \
    > "$OUT/replay_${L%.so}.log" 2>&1; stop $? "replay $L"
done
cd /tmp && export TMPDIR=/tmp
for L in ab_base ab_small; do
  NASCAR_LIB="$GRAFT_REPO_ROOT/tools/$L.so" timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES \
    --kernel-trace --output-format csv -d "$OUT/ic_$L" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --load-state /tmp/nascar_ss.pt \
    --no-cpu-baseline --no-secondary --steps 10 --warmup 2 --rollout 0 > "$OUT/ic_$L.log" 2>&1; stop $? "icache $L"
  python3 "$GRAFT_REPO_ROOT/tools/sq_summary.py" "$OUT/ic_$L" | sed "s/^/$L /"
done
cd "$GRAFT_REPO_ROOT"
ROUNDS=2 bash tools/ab3.sh tools/ab_ilds0.so tools/ab_base.so tools/ab_rolled.so tools/ab_small.so || exit $?
for r in 1 2; do   # the fused model + logic kernel on the product library
  NASCAR_FUSE_ML=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary \
    > "$OUT/ab3_fused_$r.log" 2>&1 || exit $?
  python -c "import json;d=json.loads(open('$OUT/ab3_fused_$r.log').read().strip().splitlines()[-1]);print('fused', $r, round(d['value']/1e6,1), 'M car-steps/s', round(d['ms_per_step']*1000,1), 'us/step', {k: round(v*1000,1) for k, v in d['roofline']['kernel_times_ms'].items()})"
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > "$OUT/ab3_prod_$r.log" 2>&1 || exit $?
  python -c "import json;d=json.loads(open('$OUT/ab3_prod_$r.log').read().strip().splitlines()[-1]);print('product', $r, round(d['value']/1e6,1), 'M car-steps/s', round(d['ms_per_step']*1000,1), 'us/step', {k: round(v*1000,1) for k, v in d['roofline']['kernel_times_ms'].items()})"
done
for r in 1 2; do
  for L in 16 4; do
    NASCAR_RAY_LPC=$L timeout -k 10 200 python bench.py --envs 4096 --cars 1 --steps 200 --warmup 20 --no-cpu-baseline \
      --no-secondary > "$OUT/cfg2_lpc${L}_$r.log" 2>&1 || exit $?
    python -c "import json;d=json.loads(open('$OUT/cfg2_lpc${L}_$r.log').read().strip().splitlines()[-1]);print('cfg2 lpc$L', $r, round(d['ms_per_step']*1000,1), 'us/step', {k: round(v*1000,1) for k, v in d['roofline']['kernel_times_ms'].items()})"
  done
done

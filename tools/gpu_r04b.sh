#!/bin/bash
# round-4 session B: phase profiles of the general island in scratch (ilds0) vs LDS (ilds1) on one saved steady
# state, the driver's command A/B of the same two builds, and cfg2 with 4 vs 16 sensor lanes per car.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
LIBS="libprof_ilds0.so libprof_ilds1.so" bash tools/gpu_phase.sh || exit $?
ROUNDS=3 bash tools/ab3.sh tools/ab_ilds0.so tools/ab_ilds1.so || exit $?
for r in 1 2; do
  for L in 16 4; do
    NASCAR_RAY_LPC=$L timeout -k 10 200 python bench.py --envs 4096 --cars 1 --steps 200 --warmup 20 --no-cpu-baseline \
      --no-secondary > "$OUT/cfg2_lpc${L}_$r.log" 2>&1 || exit $?
    python -c "import json;d=json.loads(open('$OUT/cfg2_lpc${L}_$r.log').read().strip().splitlines()[-1]);print('cfg2 lpc$L', $r, round(d['ms_per_step']*1000,1), 'us/step', {k: round(v*1000,1) for k, v in d['roofline']['kernel_times_ms'].items()})"
  done
done

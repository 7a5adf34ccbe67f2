#!/bin/bash
# round-4 session G: the driver's command (2 rounds each) with the ray sensor kernel's workgroup at 256 / 512 / 1024
# threads (16 lanes per car), the step workgroups at 12 vs 6 envs, and 64-thread step workgroups (-DSBLOCK=64: one wave
# of 60 cars per fused workgroup; with 4 / 3 LDS contact slots per lane), each variant's smoke first.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], round(d['value']/1e6,1), 'M car-steps/s', round(d['ms_per_step']*1000,1), 'us/step', {k: round(v*1000,1) for k, v in d['roofline']['kernel_times_ms'].items()})" "$1" "$2"; }
for L in ${SMOKE_LIBS:-tools/ab_sb64.so tools/ab_sb64c3.so}; do   # parity first: smoke (GPU == oracle) under each variant
  NASCAR_LIB="$GRAFT_REPO_ROOT/$L" timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/g_smoke_$(basename $L .so).log" 2>&1 || { echo "smoke $L failed"; tail -5 "$OUT/g_smoke_$(basename $L .so).log"; exit 1; }
  echo "smoke $L ok"
done
for r in 1 2; do
  for V in ${VARIANTS:-"base:" "rb512:NASCAR_RBLOCK=512" "rb1024:NASCAR_RBLOCK=1024" "epb6:NASCAR_EPB=6" "sb64:NASCAR_LIB=$GRAFT_REPO_ROOT/tools/ab_sb64.so" "sb64c3:NASCAR_LIB=$GRAFT_REPO_ROOT/tools/ab_sb64c3.so"}; do
    tag=${V%%:*}; ev=${V#*:}
    env $ev timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > "$OUT/g_${tag}_$r.log" 2>&1 || exit $?
    line "$OUT/g_${tag}_$r.log" "$tag $r"
  done
done
PHASE_ARGS="--rollout 50" LIBS="libprof_base.so" bash tools/gpu_phase.sh || exit $?
echo r04g-ok

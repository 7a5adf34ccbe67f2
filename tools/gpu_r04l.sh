#!/bin/bash
# round-4 session L: the general island's constraints copied LDS -> registers per loop body (-DISLAND_COPY_GENERAL=1,
# point loops unrolled) vs the product and vs the unrolled point loops alone: smoke under each, the driver's command
# A/B (2 rounds), then the variant's phase profile (3-contact island solve cycles).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
for L in tools/ab_copy.so tools/ab_unr.so; do
  NASCAR_LIB="$GRAFT_REPO_ROOT/$L" timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/l_smoke.log" 2>&1 || { tail -5 "$OUT/l_smoke.log"; exit 1; }
  echo "smoke $L ok"
done
ROUNDS=2 bash tools/ab3.sh tools/ab_prod.so tools/ab_copy.so tools/ab_unr.so || exit $?
LIBS="libprof_copy.so" bash tools/gpu_phase.sh || exit $?
grep -E "slowest wave's b2_step|islands of|longest solve|model_kernel: waves|realtime" "$OUT/phase_libprof_copy.log"
echo r04l-ok

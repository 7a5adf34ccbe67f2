#!/bin/bash
# round-4 session I: 3-contact islands through the LDS general solver (-DISLAND_MID=2: no register-resident
# 3-contact solver, model kernels spill-free) vs the product: smoke under the variant, the driver's command A/B
# (3 rounds), then phase profiles of both on one saved steady state.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
NASCAR_LIB="$GRAFT_REPO_ROOT/tools/ab_mid2.so" timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/i_smoke.log" 2>&1 || { tail -5 "$OUT/i_smoke.log"; exit 1; }
echo "smoke mid2 ok"
ROUNDS=3 bash tools/ab3.sh tools/ab_prod.so tools/ab_mid2.so || exit $?
LIBS="libprof_base.so libprof_mid2.so" bash tools/gpu_phase.sh || exit $?
for L in libprof_base libprof_mid2; do grep -E "slowest wave's b2_step|islands of|model_kernel: waves|realtime" "$OUT/phase_$L.log" | sed "s/^/$L /"; done
echo r04i-ok

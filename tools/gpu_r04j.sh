#!/bin/bash
# round-4 session J: the full GPU suite on the product build (tools/gpu_tests.sh, no bench), then the 3-contact island
# A/B of session I (smoke under the variant, the driver's command, 2 rounds).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
SKIP_BENCH=1 bash tools/gpu_tests.sh || exit $?
grep -E "passed|failed" "$OUT/gpu_tests.log" | tail -1
NASCAR_LIB="$GRAFT_REPO_ROOT/tools/ab_mid2.so" timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/j_smoke.log" 2>&1 || { tail -5 "$OUT/j_smoke.log"; exit 1; }
echo "smoke mid2 ok"
ROUNDS=2 bash tools/ab3.sh tools/ab_prod.so tools/ab_mid2.so || exit $?
echo r04j-ok

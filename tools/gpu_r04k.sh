#!/bin/bash
# round-4 session K: SolveTOI wall-record prefetch (-DTOI_WALL_PREFETCH=2 / 3) vs the product: smoke under each,
# then the driver's command A/B (2 rounds).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
for L in tools/ab_twp2.so tools/ab_twp3.so; do
  NASCAR_LIB="$GRAFT_REPO_ROOT/$L" timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/k_smoke.log" 2>&1 || { tail -5 "$OUT/k_smoke.log"; exit 1; }
  echo "smoke $L ok"
done
ROUNDS=2 bash tools/ab3.sh tools/ab_prod.so tools/ab_twp2.so tools/ab_twp3.so || exit $?
echo r04k-ok

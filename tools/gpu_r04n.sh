#!/bin/bash
# round-4 session N: wave priority raised (s_setprio 3) only for the waves with a TOI event, from their first event
# to the end of SolveTOI (-DMODEL_PRIO=3) vs the product: smoke, then the driver's command A/B (3 rounds).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
NASCAR_LIB="$GRAFT_REPO_ROOT/tools/ab_prio3.so" timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/n_smoke.log" 2>&1 || { tail -5 "$OUT/n_smoke.log"; exit 1; }
echo "smoke prio3 ok"
ROUNDS=3 bash tools/ab3.sh tools/ab_prod.so tools/ab_prio3.so || exit $?
echo r04n-ok

#!/bin/bash
# round-4 session P: LDS contact slots per lane 3 / 2 (-DCT_LDS_CAP) vs the product's 4 with the fused kernel (less LDS
# per step workgroup leaves room for the other shards' sensor workgroups): smoke under each, the driver's command A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
for L in tools/ab_ct3.so tools/ab_ct2.so; do
  NASCAR_LIB="$GRAFT_REPO_ROOT/$L" timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/p_smoke.log" 2>&1 || { tail -5 "$OUT/p_smoke.log"; exit 1; }
  echo "smoke $L ok"
done
ROUNDS=3 bash tools/ab3.sh tools/ab_prod.so tools/ab_ct3.so tools/ab_ct2.so || exit $?
echo r04p-ok

#!/bin/bash
# round-4 session M: the 16-lane sensor walks reading the global (L2-resident) wall image without LDS staging
# (NASCAR_SENSOR_GW=1) vs the product: smoke under the variant, the driver's command A/B (3 rounds).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], round(d['value']/1e6,1), 'M car-steps/s', round(d['ms_per_step']*1000,1), 'us/step', {k: round(v*1000,1) for k, v in d['roofline']['kernel_times_ms'].items()})" "$1" "$2"; }
NASCAR_SENSOR_GW=1 NASCAR_LIB="$GRAFT_REPO_ROOT/tools/ab_gw.so" timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/m_smoke.log" 2>&1 || { tail -5 "$OUT/m_smoke.log"; exit 1; }
echo "smoke gw ok"
for r in 1 2 3; do
  for V in "prod:NASCAR_LIB=$GRAFT_REPO_ROOT/tools/ab_prod.so" "gw:NASCAR_LIB=$GRAFT_REPO_ROOT/tools/ab_gw.so NASCAR_SENSOR_GW=1"; do
    tag=${V%%:*}; ev=${V#*:}
    env $ev timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > "$OUT/m_${tag}_$r.log" 2>&1 || exit $?
    line "$OUT/m_${tag}_$r.log" "$tag $r"
  done
done
echo r04m-ok

#!/bin/bash
# A/B of library builds: smoke parity, then the headline bench (200 steps + the driver's 20-step window) per lib.
# Usage: tools/ab2.sh lib1.so lib2.so ...   (BENCH_EXTRA: more bench.py flags)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT" && mkdir -p gpurun_out
for L in "$@"; do
  tag=$(basename "$L" .so)
  NASCAR_LIB="$ROOT/$L" timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/ab2_smoke_$tag.log" 2>&1 || { echo "$tag smoke failed"; exit 1; }
  NASCAR_LIB="$ROOT/$L" timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-secondary $BENCH_EXTRA > "gpurun_out/ab2_$tag.log" 2>&1 || { echo "$tag bench failed"; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab2_$tag.log').read().strip().splitlines()[-1]);print('$tag', round(d['value']/1e6,1), 'M car-steps/s', round(d['ms_per_step']*1000,1), 'us/step; per-step path', round(d.get('per_step',{}).get('ms_per_step',0)*1000,1), 'us')"
done

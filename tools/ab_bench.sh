#!/bin/bash
# A/B: for each library given, smoke parity + a short bench.  Usage: tools/ab_bench.sh lib1.so lib2.so ...
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT" && mkdir -p gpurun_out
for L in "$@"; do
  tag=$(basename "$L" .so)
  NASCAR_LIB="$ROOT/$L" timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/ab_smoke_$tag.log" 2>&1 || { echo "$tag smoke failed"; exit 1; }
  NASCAR_LIB="$ROOT/$L" timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > "gpurun_out/ab_$tag.log" 2>&1 || { echo "$tag bench failed"; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab_$tag.log').read().strip().splitlines()[-1]);print('$tag', round(d['value']/1e6,1), 'M car-steps/s', round(d['roofline']['kernel_ms']*1000,1), 'us/step')"
done

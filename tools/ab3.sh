#!/bin/bash
# A/B of library builds on the driver's exact command (bench.py --steps 20 --warmup 5), ROUNDS rounds alternating
# the libs (default 3); prints ms_per_step per run.  Usage: tools/ab3.sh a.so b.so ...
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT" && mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-3}); do
  for spec in "$@"; do
    IFS=, read -r L envs <<< "$spec"   # "lib.so,VAR=VAL,...": environment for that run only
    tag=$(basename "$L" .so)${envs:+_${envs//[^A-Za-z0-9]/}}
    env ${envs//,/ } NASCAR_LIB="$ROOT/$L" timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary $BENCH_EXTRA \
      > "gpurun_out/ab3_${tag}_$r.log" 2>&1 || { echo "$tag bench failed"; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ab3_${tag}_$r.log').read().strip().splitlines()[-1]);print('$tag', $r, round(d['value']/1e6,1), 'M car-steps/s', round(d['ms_per_step']*1000,1), 'us/step')"
  done
done

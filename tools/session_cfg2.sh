#!/bin/bash
# cfg2 (4096 envs x 1 car): workgroup spreading (NASCAR_EPB) A/B, base library for reference
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 200 env "$@" python3 bench.py --envs 4096 --cars 1 --steps 200 --warmup 20 --no-cpu-baseline --no-secondary > gpurun_out/cfg2_$tag.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/cfg2_$tag.log').read().strip().splitlines()[-1]);print('$tag', round(d['value']/1e6,2), 'M car-steps/s', round(d['ms_per_step']*1000,1), 'us/step; per-step', round(d.get('per_step',{}).get('ms_per_step',0)*1000,1))"; }
run base NASCAR_LIB=$GRAFT_REPO_ROOT/ab/base.so
run epb128 NASCAR_EPB=128
run auto X=1
run epb4 NASCAR_EPB=4
run epb2 NASCAR_EPB=2
run epb1 NASCAR_EPB=1
run epb16 NASCAR_EPB=16
run auto2 X=1

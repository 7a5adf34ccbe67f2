#!/bin/bash
# cfg4 rank shape (8192 x 4) and cfg5 rank shape (4096 x 10, 8 tracks): auto workgroup spreading vs full workgroups
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() { tag=$1; shift; args=$1; shift; timeout -k 10 300 env "$@" python3 bench.py $args --steps 200 --warmup 20 --no-cpu-baseline --no-secondary > gpurun_out/c45_$tag.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/c45_$tag.log').read().strip().splitlines()[-1]);print('$tag', round(d['value']/1e6,1), 'M car-steps/s', round(d['ms_per_step']*1000,1), 'us/step; per-step', round(d.get('per_step',{}).get('ms_per_step',0)*1000,1))"; }
run cfg4_full "--envs 8192 --cars 4" NASCAR_EPB=32
run cfg4_auto "--envs 8192 --cars 4" X=1
run cfg5_full "--envs 4096 --cars 10 --mixed" NASCAR_EPB=12
run cfg5_auto "--envs 4096 --cars 10 --mixed" X=1
run cfg4_full2 "--envs 8192 --cars 4" NASCAR_EPB=32
run cfg4_auto2 "--envs 8192 --cars 4" X=1

#!/bin/bash
# rollout schedules on the current build: fused kernel (0 streams) and 2 / 3 / 4 / 6 shards
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for S in 0 4 2 3 6 0 4; do
  timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-secondary --rollout-streams $S > gpurun_out/sched_$S.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/sched_$S.log').read().strip().splitlines()[-1]);print('streams $S', round(d['value']/1e6,1), 'M car-steps/s', round(d['ms_per_step']*1000,1), 'us/step')"
done

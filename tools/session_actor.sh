#!/bin/bash
# fp32 actor on the f32 MFMA: parity tests, kernel time (HIP events + rocprofv3), SAC closed loop bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_actor.py tests/test_gpu_rollout.py > gpurun_out/t_actor.log 2>&1 || { echo tests failed; exit 1; }
echo tests ok
timeout -k 10 120 python3 tools/actor_bench.py 81920 200 > gpurun_out/actor_mfma32.log 2>&1 || exit $?
NASCAR_ACTOR_FP32_VALU=1 timeout -k 10 120 python3 tools/actor_bench.py 81920 200 > gpurun_out/actor_valu32.log 2>&1 || exit $?
tail -1 gpurun_out/actor_mfma32.log; tail -1 gpurun_out/actor_valu32.log
rm -rf gpurun_out/actor_kt; cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/actor_kt" -o run -- python3 "$GRAFT_REPO_ROOT/tools/actor_bench.py" 81920 100 > "$GRAFT_REPO_ROOT/gpurun_out/actor_kt.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 bench.py --policy sac --steps 200 --warmup 20 --no-cpu-baseline --no-secondary > gpurun_out/b_sac.log 2>&1 || exit $?
NASCAR_ACTOR_FP32_VALU=1 timeout -k 10 300 python3 bench.py --policy sac --steps 200 --warmup 20 --no-cpu-baseline --no-secondary > gpurun_out/b_sac_valu.log 2>&1 || exit $?
for f in b_sac b_sac_valu; do python3 -c "import json;d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]);print('$f', round(d['value']/1e6,1), 'M car-steps/s', round(d['ms_per_step']*1000,1), 'us/step')"; done

#!/bin/bash
# TOI cull A/B session: check build counts (culled calls that would be TOUCHING must be 0), A/B on the driver's
# command, then parity tests.  A fault / time limit ends it.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
timeout -k 10 300 python bench.py --save-state /tmp/nascar_ss.pt --no-cpu-baseline --no-secondary --steps 20 --warmup 5 \
    > gpurun_out/cull_bench.log 2>&1; stop $? bench
timeout -k 10 200 python tools/phase_profile.py --no-build --lib libnascar_chk.so --load-state /tmp/nascar_ss.pt --warmup 20 --steps 4 \
    > gpurun_out/cull_chk.log 2>&1; stop $? chk
ROUNDS=${ROUNDS:-3} timeout -k 10 600 bash tools/ab3.sh nascargymnasium_amd/libnascar.so ab/cull1.so $ABLIBS > gpurun_out/cull_ab.log 2>&1; stop $? ab
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_configs.py} -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/cull_tests.log 2>&1; stop $? tests
echo cull-ok

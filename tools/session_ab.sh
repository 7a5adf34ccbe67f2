#!/bin/bash
# A/B session: ab3.sh of the in-tree library against $ABLIBS on the driver's command, an optional phase profile of
# $PLIB (tools/) on a saved steady state, then the GPU tests ($TESTS, default all).  A failure ends it.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
ROUNDS=${ROUNDS:-3} timeout -k 10 700 bash tools/ab3.sh nascargymnasium_amd/libnascar.so $ABLIBS > gpurun_out/ab.log 2>&1; stop $? ab
if [ -n "$PLIB" ]; then
  timeout -k 10 300 python bench.py --save-state /tmp/nascar_ss.pt --no-cpu-baseline --no-secondary --steps 20 --warmup 5 \
      > gpurun_out/ab_bench.log 2>&1; stop $? bench
  timeout -k 10 200 python tools/phase_profile.py --no-build --lib $PLIB --load-state /tmp/nascar_ss.pt --warmup 20 --steps 3 \
      > gpurun_out/ab_phase.log 2>&1; stop $? phase
fi
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/ab_tests.log 2>&1; stop $? tests
echo ab-ok

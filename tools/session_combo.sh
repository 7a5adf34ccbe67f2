#!/bin/bash
# full GPU tests -> A/B of LIBS -> steady-state phase profile of the profile build
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 1200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_full.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gpu_full.log; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$LIBS" ]; then bash tools/ab2.sh $LIBS || exit 1; fi
if [ -n "$PHASE" ]; then LIBS=libnascar_prof.so bash tools/gpu_phase.sh || exit 1; fi
exit 0

#!/bin/bash
# full GPU test suite, then A/B of the libs given in LIBS
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 1200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_full.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_full.log; [ $rc -ne 0 ] && exit $rc
[ -n "$LIBS" ] && bash tools/ab2.sh $LIBS
exit 0

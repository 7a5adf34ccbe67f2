#!/bin/bash
# one GPU session: smoke -> gpu parity tests -> short bench. Stops on faults (rc >= 124).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -ge 124 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-budget 5 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"
exit $rc

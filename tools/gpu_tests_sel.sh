#!/bin/bash
# selected GPU tests: usage tools/gpu_tests_sel.sh <log-name> <pytest args...>
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
name=$1; shift
timeout -k 10 1500 python -u -m pytest -x -v --timeout 1200 --timeout-method thread -p no:cacheprovider "$@" > gpurun_out/$name.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/$name.log; exit $rc

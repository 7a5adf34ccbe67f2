#!/bin/bash
# GPU box: selected tests -- usage: tools/gpu_sel.sh <log-name> <pytest args...>
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
name=$1; shift
timeout -k 10 1100 python -u -m pytest -v --timeout 600 --timeout-method thread -p no:cacheprovider --durations=20 "$@" > gpurun_out/$name.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/$name.log | tail -2; exit $rc

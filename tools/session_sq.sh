#!/bin/bash
# SQ counters of the steady state without profiling the settle: save the settled state once, then each PMC pass
# runs a short per-step bench from it (tools/pmc_sq.sh with --load-state)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python3 bench.py --save-state /tmp/nascar_ss.pt --no-cpu-baseline --no-secondary --steps 20 --warmup 5 \
  > gpurun_out/sq_save.log 2>&1 || exit $?
PROG="bench.py --load-state /tmp/nascar_ss.pt --rollout 0 --steps 5 --warmup 2 --no-cpu-baseline --no-secondary" bash tools/pmc_sq.sh || exit $?

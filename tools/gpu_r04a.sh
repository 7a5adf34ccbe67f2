#!/bin/bash
# round-4 session A: GPU tests (layouts + LDS general islands), then A/B of the general island in scratch vs LDS
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_tests.sh || exit $?
ROUNDS=3 bash tools/ab3.sh tools/ab_ilds0.so tools/ab_ilds1.so

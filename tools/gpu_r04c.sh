#!/bin/bash
# round-4 session C: code-size variants of model_kernel on the driver's command (2 rounds each): the product build
# (rolled solver loops, out-of-line large-argument sincosf), sincosf out of line entirely, one small-island solver,
# and both.
cd "$GRAFT_REPO_ROOT" || exit 1
ROUNDS=${ROUNDS:-2} bash tools/ab3.sh tools/ab_small.so tools/ab_sincall.so tools/ab_two0.so tools/ab_tiny.so

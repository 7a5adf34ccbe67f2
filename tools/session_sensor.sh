#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
for L in cur sh snw; do bash tools/kt_steps.sh $L ab/$L.so || exit 1; done
bash tools/ab2.sh ab/cur.so ab/sh.so ab/cur.so ab/sh.so || exit 1
PROG="bench.py --rollout 0 --steps 5 --warmup 2 --no-cpu-baseline --no-secondary" bash tools/pmc_sq.sh || exit 1

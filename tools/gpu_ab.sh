#!/bin/bash
# A/B session: per-kernel mean durations from one saved steady state (tools/kt_ss.sh, KT_LIBS), the driver's
# command alternated over libraries (tools/ab3.sh, AB3_LIBS, ROUNDS), the driver's command at S env shards on S hardware
# queues (QUEUES="4 6 8", ROUNDS), a kernel-trace timeline of the sharded rollout (TRACE=1, tools/ro_trace.sh), then GPU
# tests (TESTS, pytest paths/args).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ge 124 ]; then exit "$rc"; fi; }
if [ -n "$KT_LIBS" ]; then bash tools/kt_ss.sh $KT_LIBS > "$OUT/ab_kt.log" 2>&1; stop $? kt; cat "$OUT/ab_kt.log"; fi
if [ -n "$AB3_LIBS" ]; then ROUNDS=${ROUNDS:-3} bash tools/ab3.sh $AB3_LIBS > "$OUT/ab_ab3.log" 2>&1; stop $? ab3; cat "$OUT/ab_ab3.log"; fi
if [ -n "$QUEUES" ]; then
  for r in $(seq 1 ${ROUNDS:-2}); do for q in $QUEUES; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary \
        --rollout-streams $q > "$OUT/q${q}_$r.log" 2>&1; stop $? "queues $q"
    python -c "import json;d=json.loads(open('$OUT/q${q}_$r.log').read().strip().splitlines()[-1]);print('queues $q', $r, round(d['ms_per_step']*1000,1), 'us/step')"
  done; done
fi
if [ -n "$TRACE" ]; then bash tools/ro_trace.sh > "$OUT/ab_trace.log" 2>&1; stop $? trace; tail -20 "$OUT/ab_trace.log"; fi
if [ -n "$TESTS" ]; then
  timeout -k 10 1100 python -u -m pytest -x -q --timeout 900 --timeout-method thread -p no:cacheprovider -m gpu $TESTS \
      > "$OUT/ab_tests.log" 2>&1; stop $? tests; tail -3 "$OUT/ab_tests.log"
fi

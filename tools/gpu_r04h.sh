#!/bin/bash
# round-4 session H: smoke, then the driver's command (2 rounds each) at 4 (default) / 3 / 2 / 6 env shards, and cfg2
# (4096 x 1, 200 steps) on the product build.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], round(d['value']/1e6,1), 'M car-steps/s', round(d['ms_per_step']*1000,1), 'us/step', {k: round(v*1000,1) for k, v in d['roofline']['kernel_times_ms'].items()})" "$1" "$2"; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/h_smoke.log" 2>&1 || { tail -5 "$OUT/h_smoke.log"; exit 1; }
for r in 1 2; do
  for S in 4 3 2 6; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --rollout-streams $S > "$OUT/h_s${S}_$r.log" 2>&1 || exit $?
    line "$OUT/h_s${S}_$r.log" "streams$S $r"
  done
done
timeout -k 10 200 python bench.py --envs 4096 --cars 1 --steps 200 --warmup 20 --no-cpu-baseline --no-secondary > "$OUT/h_cfg2.log" 2>&1 || exit $?
line "$OUT/h_cfg2.log" cfg2
echo r04h-ok

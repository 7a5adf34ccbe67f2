#!/bin/bash
# round-4 session F: A/B knobs on the driver's command (2 rounds each): ray sensor at 16 vs 4 lanes per car, fused
# model + logic kernel; the 200-step default window with and without the fused kernel; cfg2 fused vs not; cfg5's
# beam-list memory and build time at 1 / 2 m cells.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], round(d['value']/1e6,1), 'M car-steps/s', round(d['ms_per_step']*1000,1), 'us/step', {k: round(v*1000,1) for k, v in d['roofline']['kernel_times_ms'].items()})" "$1" "$2"; }
for r in 1 2; do
  for V in "base:" "lpc16:NASCAR_RAY_LPC=16" "fuse:NASCAR_FUSE_ML=1"; do
    tag=${V%%:*}; ev=${V#*:}
    env $ev timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > "$OUT/f_${tag}_$r.log" 2>&1 || exit $?
    line "$OUT/f_${tag}_$r.log" "$tag $r"
  done
done
for V in "base200:" "fuse200:NASCAR_FUSE_ML=1"; do
  tag=${V%%:*}; ev=${V#*:}
  env $ev timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-secondary > "$OUT/f_${tag}.log" 2>&1 || exit $?
  line "$OUT/f_${tag}.log" "$tag"
done
for V in "cfg2:" "cfg2fuse:NASCAR_FUSE_ML=1"; do
  tag=${V%%:*}; ev=${V#*:}
  env $ev timeout -k 10 200 python bench.py --envs 4096 --cars 1 --steps 200 --warmup 20 --no-cpu-baseline --no-secondary > "$OUT/f_${tag}.log" 2>&1 || exit $?
  line "$OUT/f_${tag}.log" "$tag"
done
for c in 1 2; do timeout -k 10 200 python tools/cfg5_memory.py --cell $c > "$OUT/f_mem_$c.log" 2>&1 || exit $?; cat "$OUT/f_mem_$c.log"; done
echo r04f-ok

#!/bin/bash
# GPU box A/B: the product library (car-car phase called inside model_logic_kernel) vs tools/build/libnascar_ccsplit.so
# (-DCC_FUSED=0: no call in the fused kernel): the driver's command (contact off) x 3 rounds, then cfg3 + contact
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/abcc"; mkdir -p "$OUT"
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ge 124 ]; then exit "$rc"; fi; }
B="--no-cpu-baseline --no-secondary --no-drop-in"
timeout -k 10 300 python bench.py $B --steps 20 --warmup 5 --save-state /tmp/ss.pt > "$OUT/save.log" 2>&1; stop $? save
for rep in 1 2 3; do
  for v in fused split; do
    if [ $v = split ]; then L=tools/build/libnascar_ccsplit.so; else L=nascargymnasium_amd/libnascar.so; fi
    NASCAR_LIB=$L timeout -k 10 200 python bench.py $B --load-state /tmp/ss.pt --steps 20 --warmup 5 > "$OUT/drv_${v}_$rep.log" 2>&1; stop $? "$v $rep"
    echo "drv $v $rep $(grep -o '"ms_per_step": [0-9.]*' "$OUT/drv_${v}_$rep.log" | head -1)"
  done
done
for v in fused split; do
  if [ $v = split ]; then L=tools/build/libnascar_ccsplit.so; else L=nascargymnasium_amd/libnascar.so; fi
  NASCAR_LIB=$L timeout -k 10 300 python bench.py $B --track talladega --car-contact --steps 200 --warmup 20 > "$OUT/cc_$v.log" 2>&1; stop $? "cc $v"
  echo "cc $v $(grep -o '"ms_per_step": [0-9.]*' "$OUT/cc_$v.log" | head -2 | tr '\n' ' ')"
done

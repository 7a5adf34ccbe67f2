cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
B="python bench.py --no-cpu-baseline --no-secondary --steps 200"
timeout -k 10 200 $B --save-state /tmp/ss.pt > $OUT/ro_0.log 2>&1 || exit $?
for R in 10 50 200; do timeout -k 10 200 $B --load-state /tmp/ss.pt --rollout $R > $OUT/ro_$R.log 2>&1 || exit $?; done
timeout -k 10 200 python tools/phase_profile.py --no-build --lib libnascar_prof.so --load-state /tmp/ss.pt --warmup 5 --steps 1 --rollout 50 > $OUT/ro_phase.log 2>&1

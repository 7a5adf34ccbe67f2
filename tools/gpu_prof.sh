#!/bin/bash
# GPU box: the round's profiles of the frozen build (rocprofv3 kernel stats + FETCH/WRITE + SQ passes from one saved
# steady state, then cfg2 kernel stats); the bench lines are taken in a later call, after tools/pmc_summary.py has
# written profiles/pmc_traffic.json for these sources, so their roofline.traffic is the current build's
#   TAG=r06 bash tools/gpu_prof.sh ; python tools/pmc_summary.py gpurun_out/prof r06
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ge 124 ]; then exit "$rc"; fi; }
N="--no-cpu-baseline --no-secondary --no-drop-in"
timeout -k 10 300 python bench.py $N --steps 20 --warmup 5 --save-state /tmp/nascar_ss.pt > "$OUT/prof_save.log" 2>&1; stop $? save
[ -f /tmp/nascar_ss.pt ] || exit 1
P="$GRAFT_REPO_ROOT/bench.py --load-state /tmp/nascar_ss.pt $N"
python -c "import bench; print(bench.source_sha())" > "$OUT/prof_source_sha.txt"
cd /tmp && export TMPDIR=/tmp
rm -rf "$OUT/prof" && mkdir -p "$OUT/prof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof/kt" -o run -- \
    python3 $P --steps 100 --warmup 5 > "$OUT/prof/kt.log" 2>&1; stop $? kt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/prof/fetch" -o run -- \
    python3 $P --steps 10 --warmup 2 > "$OUT/prof/fetch.log" 2>&1; stop $? fetch
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/prof/write" -o run -- \
    python3 $P --steps 10 --warmup 2 > "$OUT/prof/write.log" 2>&1; stop $? write
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
    --kernel-trace --output-format csv -d "$OUT/prof/sq" -o run -- python3 $P --steps 10 --warmup 2 > "$OUT/prof/sq.log" 2>&1; stop $? sq
rm -rf "$OUT/prof_cfg2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg2" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --envs 4096 --cars 1 --steps 200 --warmup 20 $N > "$OUT/prof_cfg2.log" 2>&1; stop $? cfg2
rm -f "$OUT"/prof_cfg2/*kernel_trace.csv
du -sh "$OUT"
echo prof-ok

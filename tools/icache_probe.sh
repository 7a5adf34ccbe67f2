cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ic
timeout -k 10 120 rocprofv3 -L > gpurun_out/ic/list.txt 2>&1; grep -i "icache\|SQC_" gpurun_out/ic/list.txt | head -40 > gpurun_out/ic/sqc.txt
timeout -k 10 300 python bench.py --save-state /tmp/nascar_ss.pt --no-cpu-baseline --no-secondary --steps 20 --rollout 0 > gpurun_out/ic/bench.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ic/p1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --load-state /tmp/nascar_ss.pt --no-cpu-baseline --no-secondary --steps 5 --warmup 1 --rollout 0 > $GRAFT_REPO_ROOT/gpurun_out/ic/p1.log 2>&1
echo pmc rc=$?

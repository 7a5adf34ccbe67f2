cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
stop() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ge 124 ]; then exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_random_tracks.py tests/test_gpu_api.py tests/test_gpu_rollout.py -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider --durations=30 > gpurun_out/t1.log 2>&1; stop $? tests
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/b1.log 2>&1; stop $? bench

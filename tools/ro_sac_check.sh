set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rollout.py > gpurun_out/ro_tests.log 2>&1 && tail -1 gpurun_out/ro_tests.log &&
timeout -k 10 300 python -u bench.py --policy sac --no-secondary --no-cpu-baseline > gpurun_out/bench_sac.log 2>&1 && grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.e+]*' gpurun_out/bench_sac.log

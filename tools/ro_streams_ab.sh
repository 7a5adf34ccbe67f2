set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rollout.py > gpurun_out/ro_tests.log 2>&1 && tail -3 gpurun_out/ro_tests.log &&
for R in 100:3 100:4 100:5 50:4 20:4 100:8; do r=${R%%:*}; s=${R##*:}
  timeout -k 10 200 python -u bench.py --rollout $r --rollout-streams $s --no-secondary --no-cpu-baseline > gpurun_out/ro_b_${r}_${s}.log 2>&1 || exit 1
  echo "R=$r S=$s $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ro_b_${r}_${s}.log) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/ro_b_${r}_${s}.log)"
done

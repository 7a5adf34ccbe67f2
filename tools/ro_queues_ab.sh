# sharded rollout vs hardware queues per process (GPU_MAX_HW_QUEUES; the engine's default shard count follows it)
set -o pipefail
cd $GRAFT_REPO_ROOT
for Q in 4:4 8:8 8:6 8:4 6:6 12:12; do q=${Q%%:*}; s=${Q##*:}
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u bench.py --rollout-streams $s --no-secondary --no-cpu-baseline > gpurun_out/rq_${q}_${s}.log 2>&1 || exit 1
  echo "Q=$q S=$s $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rq_${q}_${s}.log | tr '\n' ' ')"
done

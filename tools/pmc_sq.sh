#!/bin/bash
# SQ counter pass (own run, --kernel-trace only): wave cycles, issue/wait breakdown, instruction mix.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
rm -rf "$ROOT/gpurun_out/sq" && mkdir -p "$ROOT/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
   --kernel-trace --output-format csv -d "$ROOT/gpurun_out/sq" -o run -- \
   python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$ROOT/gpurun_out/sq.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD \
   --kernel-trace --output-format csv -d "$ROOT/gpurun_out/sq2" -o run -- \
   python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$ROOT/gpurun_out/sq2.log" 2>&1 || exit $?
echo sq-ok

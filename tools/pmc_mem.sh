#!/bin/bash
# Memory-pipeline counter passes per kernel (each pass its own run, --kernel-trace only):
#   TA busy / wavefronts, L1 (TCP) accesses and L2 requests with latency, VMEM level and wave cycles.
# Summarise: python tools/sq_summary.py gpurun_out/pm1 gpurun_out/pm2 gpurun_out/pm3
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
PROG="${PROG:-bench.py --steps 5 --warmup 2 --no-cpu-baseline}"
rm -rf "$ROOT/gpurun_out/pm1" "$ROOT/gpurun_out/pm2" "$ROOT/gpurun_out/pm3" && mkdir -p "$ROOT/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_TOTAL_WAVEFRONTS_sum GRBM_GUI_ACTIVE \
   --kernel-trace --output-format csv -d "$ROOT/gpurun_out/pm1" -o run -- python3 $ROOT/$PROG > "$ROOT/gpurun_out/pm1.log" 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc TCP_TOTAL_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum \
   --kernel-trace --output-format csv -d "$ROOT/gpurun_out/pm2" -o run -- python3 $ROOT/$PROG > "$ROOT/gpurun_out/pm2.log" 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VALU_FLOPS_FP64 \
   --kernel-trace --output-format csv -d "$ROOT/gpurun_out/pm3" -o run -- python3 $ROOT/$PROG > "$ROOT/gpurun_out/pm3.log" 2>&1 || exit $?
echo pm-ok

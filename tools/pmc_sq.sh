#!/bin/bash
# SQ counter passes (each its own run, --kernel-trace only): wave cycles, issue/wait breakdown,
# instruction mix, MFMA/LDS activity.  PROG overrides the profiled program (default: the bench).
#   PROG="tools/actor_bench.py 81920 20" bash tools/pmc_sq.sh
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
PROG="${PROG:-bench.py --steps 5 --warmup 2 --no-cpu-baseline}"
rm -rf "$ROOT/gpurun_out/sq" "$ROOT/gpurun_out/sq2" "$ROOT/gpurun_out/sq3" && mkdir -p "$ROOT/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
   --kernel-trace --output-format csv -d "$ROOT/gpurun_out/sq" -o run -- \
   python3 $ROOT/$PROG > "$ROOT/gpurun_out/sq.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD \
   --kernel-trace --output-format csv -d "$ROOT/gpurun_out/sq2" -o run -- \
   python3 $ROOT/$PROG > "$ROOT/gpurun_out/sq2.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
   --kernel-trace --output-format csv -d "$ROOT/gpurun_out/sq3" -o run -- \
   python3 $ROOT/$PROG > "$ROOT/gpurun_out/sq3.log" 2>&1 || exit $?
echo sq-ok

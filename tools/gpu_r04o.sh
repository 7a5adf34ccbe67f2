#!/bin/bash
# round-4 session O: LDS-only workgroup barriers in the step kernels (-DLDS_BARRIER=1: no wait for outstanding global
# stores / loads at barriers that hand off only LDS) vs the product: smoke and the closed-loop / golden parity tests
# under the variant, then the driver's command A/B (3 rounds).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
export_lib="$GRAFT_REPO_ROOT/tools/ab_ldsb.so"
NASCAR_LIB="$export_lib" timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/o_smoke.log" 2>&1 || { tail -5 "$OUT/o_smoke.log"; exit 1; }
echo "smoke ldsb ok"
NASCAR_LIB="$export_lib" timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py::test_bench_workload_full_episode_vs_oracle \
    -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > "$OUT/o_tests.log" 2>&1
rc=$?; tail -2 "$OUT/o_tests.log"; [ $rc -ge 124 ] && exit $rc
ROUNDS=3 bash tools/ab3.sh tools/ab_prod.so tools/ab_ldsb.so || exit $?
echo r04o-ok

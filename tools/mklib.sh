#!/bin/bash
# build an A/B variant of libnascar.so (with -DNASCAR_AB_KNOBS: the A/B environment knobs NASCAR_EPB, NASCAR_RAY_LPC,
# NASCAR_FUSE_ML, NASCAR_RBLOCK, NASCAR_BEAM_CELL, NASCAR_SENSOR, NASCAR_NO_MAP_SHORTCUT, NASCAR_ACTOR_FP32_VALU, NASCAR_MAP_CONTIGUOUS are
# read only by such builds): tools/mklib.sh OUT.so [SRC_DIR(csrc)] [extra hipcc flags...]
out=$1; shift
src=${1:-nascargymnasium_amd/csrc}; shift
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-fast-math -fno-slp-vectorize -fPIC -shared -std=c++17 -Wno-unused-value \
  -Wno-unused-result -DNASCAR_AB_KNOBS "$@" -o "$out" "$src/nascar_kernels.hip"

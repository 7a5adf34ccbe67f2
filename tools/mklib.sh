#!/bin/bash
# build an A/B variant of libnascar.so: tools/mklib.sh OUT.so [SRC_DIR(csrc)] [extra hipcc flags...]
out=$1; shift
src=${1:-nascargymnasium_amd/csrc}; shift
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-fast-math -fPIC -shared -std=c++17 -Wno-unused-value \
  -Wno-unused-result "$@" -o "$out" "$src/nascar_kernels.hip"

#!/bin/bash
# A/B of fused encode + CRC variants: the product library and every tools/build/v_* build,
# alternated (A B A B ...) FUSED_ROUNDS times (default 2), so box drift shows as spread rather than
# as a difference between variants.
cd "$(dirname "$0")/.."
# FUSED_SHAPES: space-separated k,m,blocks,block_bytes shapes (default RS(10,4) 256 KiB and RS(16,4) 4 MiB)
for r in $(seq 1 ${FUSED_ROUNDS:-2}); do
 for sh in ${FUSED_SHAPES:-10,4,4096,262144 16,4,256,4194304}; do
  FUSED_SHAPE=$sh timeout -k 10 120 python tools/fusedab.py 2>&1 | grep -v amdgpu.ids || exit 1
  for d in tools/build/v_*/lib/librsmi.so; do
    [ -e "$d" ] || continue
    FUSED_SHAPE=$sh RSMI_LIB=$(pwd)/$d timeout -k 10 120 python tools/fusedab.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
 done
done

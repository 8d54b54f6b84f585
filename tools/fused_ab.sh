#!/bin/bash
# A/B of fused encode + CRC variants: the product library and every tools/build/v_* build,
# alternated (A B A B ...) FUSED_ROUNDS times (default 2), so box drift shows as spread rather than
# as a difference between variants.
cd "$(dirname "$0")/.."
for r in $(seq 1 ${FUSED_ROUNDS:-2}); do
  timeout -k 10 120 python tools/fusedab.py 2>&1 | grep -v amdgpu.ids || exit 1
  for d in tools/build/v_*/lib/librsmi.so; do
    [ -e "$d" ] || continue
    RSMI_LIB=$(pwd)/$d timeout -k 10 120 python tools/fusedab.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done

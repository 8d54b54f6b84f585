#!/bin/bash
# A/B of fused encode + CRC variants: the product library, then every tools/build/v_* build.
cd "$(dirname "$0")/.."
timeout -k 10 120 python tools/fusedab.py 2>&1 | grep -v amdgpu.ids || exit 1
for d in tools/build/v_*/lib/librsmi.so; do
  RSMI_LIB=$(pwd)/$d timeout -k 10 120 python tools/fusedab.py 2>&1 | grep -v amdgpu.ids || exit 1
done

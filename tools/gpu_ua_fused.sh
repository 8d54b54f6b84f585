#!/bin/bash
# GPU session for the unaligned-window (Split layout) fused encode + CRC-16 on the matrix cores:
# its parity tests, the fused-vs-encode A/B against the nibble fold (crc16_fused_fold=0), then the
# UA load-form variants' parity and A/B, and the NUMA-bound device-group tests.  Every GPU step
# has its own time limit; the script stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
step() { echo "== $*"; }

step fused tests
timeout -k 10 500 $PYT tests/test_crc16.py -m gpu -k "fused or verify_survivor" > gpurun_out/ua_fused_tests.log 2>&1 || { tail -30 gpurun_out/ua_fused_tests.log; exit 1; }
tail -2 gpurun_out/ua_fused_tests.log

step fused A/B: matrix-core fold vs nibble fold
for r in 1 2; do
  timeout -k 10 120 python tools/fusedab.py 2>&1 | grep -v amdgpu.ids || exit 1
  FUSED_OPT=crc16_fused_fold=0 timeout -k 10 120 python tools/fusedab.py 2>&1 | grep -v amdgpu.ids || exit 1
done | tee gpurun_out/ua_fused_ab.txt

if [ "${UA_VARIANTS:-1}" = 1 ]; then
  step UA4all variant parity
  RSMI_LIB=$PWD/tools/build/v_ua4all/lib/librsmi.so timeout -k 10 400 $PYT tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu > gpurun_out/ua4all_tests.log 2>&1 || { tail -30 gpurun_out/ua4all_tests.log; exit 1; }
  tail -2 gpurun_out/ua4all_tests.log
  step UA load-form A/B
  bash tools/ua4_ab.sh || exit 1
fi

step device group tests
timeout -k 10 200 $PYT tests/test_device_group.py -m gpu > gpurun_out/group_tests.log 2>&1 || { tail -30 gpurun_out/group_tests.log; exit 1; }
tail -2 gpurun_out/group_tests.log

#!/bin/bash
# CRC rows passes: parity (CRC-16 and CRC-32 suites), then the passes named in CRC_SWEEP_FOLDS
# (crcbench.py CRC_FOLDS syntax) at the grid caps in CRC_SWEEP_WPC (waves per CU; 0 = each
# pass's default: 48 pipelined, 96 plain).
set -o pipefail
mkdir -p gpurun_out
F=${CRC_SWEEP_FOLDS:-3,1,crc32,crc32pipe}
timeout -k 10 300 python -u -m pytest tests/test_crc16.py tests/test_crc32.py -x -q --timeout 120 --timeout-method thread > gpurun_out/crc_tests.log 2>&1 || { tail -30 gpurun_out/crc_tests.log; exit 1; }
tail -1 gpurun_out/crc_tests.log
for w in ${CRC_SWEEP_WPC:-0 48 96}; do
  echo "== waves_per_cu ${w}"
  CRC_FOLDS=$F CRC_WPC=$w timeout -k 10 120 python tools/crcbench.py 2>&1 | grep crc || exit 1
done

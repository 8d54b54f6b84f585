#!/bin/bash
# CRC-16 rows kernel: parity, then the pipelined and plain nibble folds at several grid caps.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_crc16.py -x -q --timeout 120 --timeout-method thread > gpurun_out/crc_tests.log 2>&1 || { tail -30 gpurun_out/crc_tests.log; exit 1; }
tail -1 gpurun_out/crc_tests.log
for w in 0 48 160; do
  echo "== waves_per_cu ${w} (0 = default 96)"
  CRC_FOLDS=3,1 CRC_WPC=$w timeout -k 10 120 python tools/crcbench.py 2>&1 | grep crc16 || exit 1
done

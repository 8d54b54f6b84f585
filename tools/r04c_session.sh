#!/bin/bash
# Round-4 session c: is the fused encode + CRC-16 issue-bound?  The product kernels against the
# cache-resident diagnostic build (RSMI_DIAG_CACHED: tiles wrap onto the first 16 blocks, so the
# launch time is the kernels' own issue time), the store-first variant's A/B, and the SQ counters
# of the fused and plain kernels (tools/pmc_fused.sh, incl. the MFMA-busy pass).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r04c
RSMI_LIB=$PWD/tools/build/v_pxis/lib/librsmi.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_crc16.py -k "fused or dev_crc" > gpurun_out/r04c/pytest_v_pxis.log 2>&1 || { echo "pytest v_pxis failed"; tail -30 gpurun_out/r04c/pytest_v_pxis.log; exit 1; }
echo "v_pxis: $(tail -1 gpurun_out/r04c/pytest_v_pxis.log)"
for rep in 1 2; do
  for lib in "" tools/build/diag-cached/lib/librsmi.so tools/build/v_pxis/lib/librsmi.so; do
    RSMI_LIB=${lib:+$PWD/$lib} timeout -k 10 200 python tools/fusedab.py >> gpurun_out/r04c/fused_ab.txt 2>gpurun_out/r04c/fused_ab.err || { echo "fusedab failed"; tail gpurun_out/r04c/fused_ab.err; exit 1; }
    RSMI_LIB=${lib:+$PWD/$lib} FUSED_SHAPE=16,4,256,4194304 timeout -k 10 200 python tools/fusedab.py >> gpurun_out/r04c/fused_ab.txt 2>>gpurun_out/r04c/fused_ab.err || { echo "fusedab failed"; tail gpurun_out/r04c/fused_ab.err; exit 1; }
  done
done
cat gpurun_out/r04c/fused_ab.txt
timeout -k 10 300 bash tools/pmc_fused.sh > gpurun_out/r04c/pmc_fused.txt 2>&1 || { echo "pmc failed"; tail gpurun_out/r04c/pmc_fused.txt; exit 1; }
cat gpurun_out/r04c/pmc_fused.txt

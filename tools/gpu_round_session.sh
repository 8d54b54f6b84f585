#!/bin/bash
# Round-end evidence: full GPU test suite, smoke, headline bench, rocprofv3 kernel trace +
# stats of the bench command, separate FETCH_SIZE / WRITE_SIZE PMC passes, a kernel-trace
# pass over the CRC kernel, and the C++ Dag Node suite.  Stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh tests || exit 1
bash tools/gpu_check.sh bench || exit 1
bash tools/gpu_check.sh prof || exit 1
rm -rf gpurun_out/prof_crc
(cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_crc" -o crc -- python3 "$R/tools/crcbench.py" > "$R/gpurun_out/prof_crc.txt" 2>&1) || { echo "crc prof failed"; tail -20 gpurun_out/prof_crc.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/prof_crc.txt
find gpurun_out/prof_crc -name "*stats*"

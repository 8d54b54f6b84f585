#!/bin/bash
# Round-4 session b2: after the lone-caller and in-place coalesced paths -- the coalesced GPU
# tests, the C++ Dag Node suite on the GPU, then the GPU-codec vs CPU-codec comparison.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r04b3
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_crc16.py -k "coalesced" > gpurun_out/r04b3/pytest_coalesced.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r04b3/pytest_coalesced.log; exit 1; }
tail -1 gpurun_out/r04b3/pytest_coalesced.log
timeout -k 10 600 ./tests/cpp/build/test_dagnode gpu > gpurun_out/r04b3/test_dagnode_gpu.log 2>&1 || { echo "test_dagnode gpu failed"; tail -30 gpurun_out/r04b3/test_dagnode_gpu.log; exit 1; }
tail -3 gpurun_out/r04b3/test_dagnode_gpu.log
timeout -k 10 900 bash tools/dagnode_cpu_vs_gpu.sh > gpurun_out/r04b3/dagnode_cpu_vs_gpu.txt 2>&1 || { echo "dagnode cmp failed"; tail -30 gpurun_out/r04b3/dagnode_cpu_vs_gpu.txt; exit 1; }
cp gpurun_out/dagnode_cmp.jsonl gpurun_out/dn_phases.jsonl gpurun_out/r04b3/
grep -v " done$" gpurun_out/r04b3/dagnode_cpu_vs_gpu.txt

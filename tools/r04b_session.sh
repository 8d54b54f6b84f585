#!/bin/bash
# Round-4 session b: the C++ Dag Node mirror on the GPU (suite, then the GPU-codec vs CPU-codec
# comparison with per-phase times), each step under its own time limit.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r04b
timeout -k 10 600 ./tests/cpp/build/test_dagnode gpu > gpurun_out/r04b/test_dagnode_gpu.log 2>&1 || { echo "test_dagnode gpu failed"; tail -30 gpurun_out/r04b/test_dagnode_gpu.log; exit 1; }
tail -2 gpurun_out/r04b/test_dagnode_gpu.log
timeout -k 10 900 bash tools/dagnode_cpu_vs_gpu.sh > gpurun_out/r04b/dagnode_cpu_vs_gpu.txt 2>&1 || { echo "dagnode cmp failed"; tail -30 gpurun_out/r04b/dagnode_cpu_vs_gpu.txt; exit 1; }
cp gpurun_out/dagnode_cmp.jsonl gpurun_out/dn_phases.jsonl gpurun_out/r04b/ 2>/dev/null
cat gpurun_out/r04b/dagnode_cpu_vs_gpu.txt

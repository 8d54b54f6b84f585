#!/bin/bash
# Round-4 session ad: the scratch pool by NUMA node
# -- CRC-16 / coalescing tests, the C++ Dag Node suite on the GPU, then the Dag Node
# GPU-vs-CPU codec comparison.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04ad
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_crc16.py -m gpu > $O/pytest_crc16.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_crc16.log; exit 1; }
tail -1 $O/pytest_crc16.log
timeout -k 10 600 ./tests/cpp/build/test_dagnode gpu > $O/test_dagnode_gpu.log 2>&1 || { echo "test_dagnode gpu failed"; tail -30 $O/test_dagnode_gpu.log; exit 1; }
tail -1 $O/test_dagnode_gpu.log
timeout -k 10 900 bash tools/dagnode_cpu_vs_gpu.sh > $O/dagnode_cpu_vs_gpu.txt 2>&1 || { echo "dagnode cmp failed"; tail -30 $O/dagnode_cpu_vs_gpu.txt; exit 1; }
cp gpurun_out/dagnode_cmp.jsonl gpurun_out/dn_phases.jsonl $O/
grep -v " done$" $O/dagnode_cpu_vs_gpu.txt | head -50

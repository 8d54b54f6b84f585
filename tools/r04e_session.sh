#!/bin/bash
# Round-4 session e: the in-kernel combine for small fused launches -- its tests, the per-block
# call latencies, then the Dag Node GPU-codec vs CPU-codec comparison.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r04e
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_crc16.py -m gpu > gpurun_out/r04e/pytest_crc16.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r04e/pytest_crc16.log; exit 1; }
tail -1 gpurun_out/r04e/pytest_crc16.log
timeout -k 10 120 ./tools/build/latency > gpurun_out/r04e/latency.txt 2>&1 || { echo "latency failed"; cat gpurun_out/r04e/latency.txt; exit 1; }
cat gpurun_out/r04e/latency.txt
timeout -k 10 600 ./tests/cpp/build/test_dagnode gpu > gpurun_out/r04e/test_dagnode_gpu.log 2>&1 || { echo "test_dagnode gpu failed"; tail -30 gpurun_out/r04e/test_dagnode_gpu.log; exit 1; }
tail -1 gpurun_out/r04e/test_dagnode_gpu.log
timeout -k 10 900 bash tools/dagnode_cpu_vs_gpu.sh > gpurun_out/r04e/dagnode_cpu_vs_gpu.txt 2>&1 || { echo "dagnode cmp failed"; tail -30 gpurun_out/r04e/dagnode_cpu_vs_gpu.txt; exit 1; }
cp gpurun_out/dagnode_cmp.jsonl gpurun_out/dn_phases.jsonl gpurun_out/r04e/
grep -v " done$" gpurun_out/r04e/dagnode_cpu_vs_gpu.txt | head -60

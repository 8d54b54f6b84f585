#!/bin/bash
# Round-4 session f: host calls that poll their stream (sync_spin_us) and read row CRCs back by
# kernel -- their tests, then the per-block call latencies per sync mode.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r04f
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_crc16.py tests/test_abi.py -m gpu > gpurun_out/r04f/pytest_crc16.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r04f/pytest_crc16.log; exit 1; }
tail -1 gpurun_out/r04f/pytest_crc16.log
timeout -k 10 200 ./tools/build/latency > gpurun_out/r04f/latency.txt 2>&1 || { echo "latency failed"; cat gpurun_out/r04f/latency.txt; exit 1; }
cat gpurun_out/r04f/latency.txt
timeout -k 10 200 ./tools/build/latency --sched-spin > gpurun_out/r04f/latency_sched_spin.txt 2>&1 || { echo "latency --sched-spin failed"; cat gpurun_out/r04f/latency_sched_spin.txt; exit 1; }
cat gpurun_out/r04f/latency_sched_spin.txt

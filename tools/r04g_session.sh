#!/bin/bash
# Round-4 session g: row CRCs read back by kernel (tests), per-block call latencies, and a
# kernel trace of the latency tool at 4 KiB and 256 KiB blocks (kernel time vs call time).
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out/r04g
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_crc16.py tests/test_abi.py -m gpu > gpurun_out/r04g/pytest_crc16.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r04g/pytest_crc16.log; exit 1; }
tail -1 gpurun_out/r04g/pytest_crc16.log
timeout -k 10 200 ./tools/build/latency > gpurun_out/r04g/latency.txt 2>&1 || { echo "latency failed"; cat gpurun_out/r04g/latency.txt; exit 1; }
cat gpurun_out/r04g/latency.txt
for B in 4096 262144; do
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r04g/prof_$B" -o lat -- "$R/tools/build/latency" $B > "$R/gpurun_out/r04g/prof_$B.log" 2>&1) || { echo "rocprof $B failed"; tail -20 gpurun_out/r04g/prof_$B.log; exit 1; }
done
find gpurun_out/r04g -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -d, -f1-8 "$f"; done

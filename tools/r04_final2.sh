#!/bin/bash
# Round-4 closing evidence on the last tree: tools/gpu_session.sh all, then tools/r04_final_b.sh
# (configs, Dag Node suite and GPU-vs-CPU codec, latencies).
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/gpu_session.sh all > gpurun_out/final2_a.log 2>&1 || { echo "part A failed"; tail -40 gpurun_out/final2_a.log; exit 1; }
grep -E "passed|value|encode only|fused CRC |rs_fast_kernel<|rs_fused" gpurun_out/final2_a.log | cut -c1-200
bash tools/r04_final_b.sh > gpurun_out/final2_b.log 2>&1 || { echo "part B failed"; tail -40 gpurun_out/final2_b.log; exit 1; }
grep -E "checks|Put, per block \||RepairDataNodeBatched|Put, 16|Get, 16" gpurun_out/final2_b.log | cut -c1-160

#!/bin/bash
# Round-4 session aj: RepairDataNodeBatched writes one flush's rebuilt rows on a helper thread
# while the next flush stages and codes -- the C++ Dag Node suite on the GPU, then the Dag Node
# GPU-vs-CPU codec comparison (both builds share the host flow).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04aj
mkdir -p $O
timeout -k 10 600 ./tests/cpp/build/test_dagnode gpu > $O/test_dagnode_gpu.log 2>&1 || { echo "test_dagnode gpu failed"; tail -30 $O/test_dagnode_gpu.log; exit 1; }
tail -1 $O/test_dagnode_gpu.log
timeout -k 10 900 bash tools/dagnode_cpu_vs_gpu.sh > $O/dagnode_cpu_vs_gpu.txt 2>&1 || { echo "dagnode cmp failed"; tail -30 $O/dagnode_cpu_vs_gpu.txt; exit 1; }
cp gpurun_out/dagnode_cmp.jsonl gpurun_out/dn_phases.jsonl $O/
grep -E "^\| (RepairDataNodeBatched|repair_batched|Put, per block \|)" $O/dagnode_cpu_vs_gpu.txt

#!/bin/bash
# Round-4 final evidence, part B (part A is tools/gpu_session.sh all): every BASELINE config
# as a side line, the C++ Dag Node GPU suite, the Dag Node GPU-vs-CPU codec comparison and the
# per-block call latencies.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04final
mkdir -p $O
timeout -k 10 900 bash tools/bench_all_configs.sh > $O/configs.txt 2>&1 || { echo "configs failed"; tail -30 $O/configs.txt; exit 1; }
cp gpurun_out/cfg_*.json $O/
cat $O/configs.txt
timeout -k 10 600 ./tests/cpp/build/test_dagnode gpu > $O/test_dagnode_gpu.log 2>&1 || { echo "test_dagnode gpu failed"; tail -30 $O/test_dagnode_gpu.log; exit 1; }
tail -1 $O/test_dagnode_gpu.log
timeout -k 10 900 bash tools/dagnode_cpu_vs_gpu.sh > $O/dagnode_cpu_vs_gpu.txt 2>&1 || { echo "dagnode cmp failed"; tail -30 $O/dagnode_cpu_vs_gpu.txt; exit 1; }
cp gpurun_out/dagnode_cmp.jsonl gpurun_out/dn_phases.jsonl $O/
grep -v " done$" $O/dagnode_cpu_vs_gpu.txt | head -70
timeout -k 10 200 ./tools/build/latency > $O/latency.txt 2>&1 || { echo "latency failed"; cat $O/latency.txt; exit 1; }
cat $O/latency.txt

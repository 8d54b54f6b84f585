#!/bin/bash
# Dag Node bench (GPU codec, RS(10,4) 256 KiB) with its threads on every CPU, on the GPU's NUMA node
# and on the other node, alternated NUMA_ROUNDS times (results in gpurun_out/r06ak/numa_ab.txt)
set -o pipefail
mkdir -p gpurun_out/r06ak
lscpu | grep -E "NUMA node[01] CPU" > gpurun_out/r06ak/lscpu.txt
N0=$(lscpu | grep "NUMA node0 CPU" | awk '{print $NF}')
N1=$(lscpu | grep "NUMA node1 CPU" | awk '{print $NF}')
for r in $(seq 1 ${NUMA_ROUNDS:-3}); do
  for mode in all node0 node1; do
    case $mode in all) pre="";; node0) pre="taskset -c $N0";; node1) pre="taskset -c $N1";; esac
    timeout -k 10 200 $pre ./tools/build/bench_dagnode 10 4 262144 512 > gpurun_out/r06ak/dn.log 2>&1 || { echo "fail $mode"; exit 1; }
    echo "$mode $(grep RESULT gpurun_out/r06ak/dn.log)" >> gpurun_out/r06ak/numa_ab.txt
  done
done
# the GPU-vs-CPU comparison with both codecs' processes on the GPU's socket (NUMA_CMP=1)
if [ -n "$NUMA_CMP" ]; then
  timeout -k 10 900 taskset -c $N0 bash tools/dagnode_cpu_vs_gpu.sh > gpurun_out/r06ak/dagnode_cpu_vs_gpu_node0.txt 2>&1 || { echo "cmp failed"; exit 1; }
fi

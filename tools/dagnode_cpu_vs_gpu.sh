#!/bin/bash
# The Dag Node mirror end to end (tools/bench_dagnode: in-process datanodes, host memory in,
# framed shard entries out) on the GPU codec (librsmi) and on a CPU codec (bench_dagnode_cpu:
# oracle/rs_cpu_fast.c on OMP_NUM_THREADS host threads), 3 alternated runs of each per shape:
# configs[0] RS(2,1) 256 KiB over 3 datanodes, RS(10,4) 256 KiB, RS(16,4) 4 MiB.  Summary
# (median and spread per leg) by tools/dagnode_table.py.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/dagnode_cmp.jsonl
: > $OUT
: > gpurun_out/dn_phases.jsonl
for shape in "2 1 262144 512" "10 4 262144 512" "16 4 4194304 64"; do
  for rep in 1 2 3; do
    timeout -k 10 300 ./tools/build/bench_dagnode $shape > gpurun_out/dn_gpu.log 2>&1 || { echo "gpu bench $shape failed"; tail gpurun_out/dn_gpu.log; exit 1; }
    grep '^RESULT ' gpurun_out/dn_gpu.log | sed 's/^RESULT //' >> $OUT
    grep '^PHASES ' gpurun_out/dn_gpu.log | sed 's/^PHASES //' >> gpurun_out/dn_phases.jsonl
    timeout -k 10 300 ./tools/build/bench_dagnode_cpu $shape > gpurun_out/dn_cpu.log 2>&1 || { echo "cpu bench $shape failed"; tail gpurun_out/dn_cpu.log; exit 1; }
    grep '^RESULT ' gpurun_out/dn_cpu.log | sed 's/^RESULT //' >> $OUT
    grep '^PHASES ' gpurun_out/dn_cpu.log | sed 's/^PHASES //' >> gpurun_out/dn_phases.jsonl
    echo "$shape run $rep done"
  done
done
python3 tools/dagnode_table.py $OUT gpurun_out/dn_phases.jsonl

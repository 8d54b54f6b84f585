#!/bin/bash
# Round-4 session ae: the Dag Node bench with glibc's mmap threshold fixed in both codec builds
# -- the GPU-vs-CPU codec comparison, then the 16-thread legs at RS(16,4) with glibc's
# dynamic threshold (BENCH_DAGNODE_DYNAMIC_MMAP=1) for the A/B.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04ae
mkdir -p $O
timeout -k 10 900 bash tools/dagnode_cpu_vs_gpu.sh > $O/dagnode_cpu_vs_gpu.txt 2>&1 || { echo "dagnode cmp failed"; tail -30 $O/dagnode_cpu_vs_gpu.txt; exit 1; }
cp gpurun_out/dagnode_cmp.jsonl gpurun_out/dn_phases.jsonl $O/
for b in bench_dagnode bench_dagnode_cpu; do
  for mode in fixed dynamic; do
    if [ $mode = dynamic ]; then export BENCH_DAGNODE_DYNAMIC_MMAP=1; else unset BENCH_DAGNODE_DYNAMIC_MMAP; fi
    timeout -k 10 300 ./tools/build/$b 16 4 4194304 64 > $O/ab.log 2>&1 || { echo "$b failed"; tail $O/ab.log; exit 1; }
    echo "$mode $b RS(16,4): $(grep -E "Put, 16|Get, 16" $O/ab.log | tr -s " " | tr "\n" ";")" >> $O/mmap_ab.txt
  done
done
cat $O/mmap_ab.txt
grep -v " done$" $O/dagnode_cpu_vs_gpu.txt | head -50

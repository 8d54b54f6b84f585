#!/bin/bash
# Round-4 session af: hardware queues per process (GPU_MAX_HW_QUEUES, HIP's default 4 on the box)
# against concurrent per-block callers -- tools/latency.cpp --threads over 1/4/8/16 contexts and
# the Dag Node bench's 16-thread legs, at 4, 8 and 16 queues.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04af
mkdir -p $O
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 ./tools/build/latency --threads > $O/threads_q$q.txt 2>&1 || { echo "latency q$q failed"; tail $O/threads_q$q.txt; exit 1; }
  for shape in "2 1 262144 512" "10 4 262144 512" "16 4 4194304 64"; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 ./tools/build/bench_dagnode $shape > $O/dn.log 2>&1 || { echo "bench q$q failed"; tail $O/dn.log; exit 1; }
    echo "q$q RS($shape): $(grep -E "Put, per block|Put, 16|Get, 16" $O/dn.log | tr -s " " | tr "\n" ";")" >> $O/dagnode_queues.txt
  done
done
cat $O/dagnode_queues.txt
for q in 4 8 16; do echo "== q$q"; grep -E "16 threads" $O/threads_q$q.txt; done

#!/bin/bash
# Round-4 session k: where a per-block call's time goes -- HIP runtime API trace and kernel trace
# of the latency tool at 4 KiB and 256 KiB blocks (launch call, launch -> kernel start, kernel,
# kernel end -> synchronise return).
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r04k
mkdir -p $O
for B in 4096 262144; do
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d "$R/$O/rt_$B" -o lat -- "$R/tools/build/latency" $B > "$R/$O/rt_$B.log" 2>&1) || { echo "rocprof $B failed"; tail -20 $O/rt_$B.log; exit 1; }
done
ls $O/rt_4096

#!/bin/bash
# Diagnostic session: new memory ceilings, then per-dispatch encode durations of the bench
# and of the clock probe on the SAME box (is the encode drift the box or the program?).
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/drift_*
timeout -k 10 200 python tools/ceilsweep.py > gpurun_out/ceilsweep.txt 2>&1 && \
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/drift_bench10" -o t -- python3 "$R/bench.py" --steps 10 --warmup 2 --cpu-seconds 0 > "$R/gpurun_out/drift_bench10.json" 2>/dev/null) && \
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/drift_probe" -o t -- python3 "$R/tools/clockprobe.py" both 100 > /dev/null 2>&1) && \
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/drift_bench100" -o t -- python3 "$R/bench.py" --steps 100 --warmup 2 --cpu-seconds 0 > "$R/gpurun_out/drift_bench100.json" 2>/dev/null) && \
timeout -k 10 200 python bench.py --cpu-seconds 0 > gpurun_out/drift_plain.json 2>/dev/null && \
timeout -k 10 200 python bench.py --cpu-seconds 0 --warmup 100 > gpurun_out/drift_plain_w100.json 2>/dev/null
cat gpurun_out/ceilsweep.txt

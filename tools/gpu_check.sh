#!/bin/bash
# One GPU session: tests, smoke, bench, rocprofv3 kernel trace.  Each step has its own
# time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
STEP=${1:-all}
if [[ $STEP == all || $STEP == tests ]]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
if [[ $STEP == all || $STEP == bench ]]; then
  timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 10 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
if [[ $STEP == all || $STEP == prof ]]; then
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OLDPWD/gpurun_out/prof" -o run -- python3 "$OLDPWD/bench.py" --steps 10 --warmup 2 --cpu-seconds 0 > "$OLDPWD/gpurun_out/prof_bench.json" 2> "$OLDPWD/gpurun_out/prof.err") || { echo "rocprof failed"; tail -20 gpurun_out/prof.err; exit 1; }
  find gpurun_out/prof -name "*stats*" | head
fi

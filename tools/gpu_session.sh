#!/bin/bash
# One GPU session: the GPU test suite, smoke, the headline bench, the side lines (Split
# layout, fused CRC-16, two ranks without a launcher), a rocprofv3 kernel trace of the
# headline bench and the FETCH_SIZE / WRITE_SIZE PMC passes.  Each step has its own time
# limit; the chain stops at the first failure.  Usage: gpu_session.sh [tests|bench|side|prof|all]...
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
for STEP in "${@:-all}"; do
if [[ $STEP == all || $STEP == tests ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
if [[ $STEP == all || $STEP == bench ]]; then
  timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }
  timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
if [[ $STEP == all || $STEP == side ]]; then
  for args in "--layout split" "--fused-crc" "--fused-crc --layout split" "--config rs10_4_1m --layout split" "--config rs16_4_4m --layout split"; do
    f=gpurun_out/side_$(echo $args | tr -d ' -').json
    timeout -k 10 300 python bench.py $args --cpu-seconds 0 > $f 2> $f.err || { echo "bench $args failed"; tail -30 $f.err; exit 1; }
    cat $f
  done
  timeout -k 10 300 python bench.py --config rs16_4_4m --copy-inclusive --group 0,0 --cpu-seconds 0 > gpurun_out/side_group.json 2> gpurun_out/side_group.err || { echo "bench --group failed"; tail -30 gpurun_out/side_group.err; exit 1; }
  cat gpurun_out/side_group.json
  timeout -k 10 300 python tools/crcbench.py > gpurun_out/crcbench.txt 2>&1 || { echo "crcbench failed"; tail -30 gpurun_out/crcbench.txt; exit 1; }
  cat gpurun_out/crcbench.txt
  timeout -k 10 300 python bench.py --gpus 2 --share-device --cpu-seconds 0 > gpurun_out/side_gpus2.json 2> gpurun_out/side_gpus2.err || { echo "bench --gpus 2 failed"; tail -30 gpurun_out/side_gpus2.err; exit 1; }
  cat gpurun_out/side_gpus2.json
fi
if [[ $STEP == all || $STEP == prof ]]; then
  rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o bench -- python3 "$R/bench.py" --cpu-seconds 0 > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof.err") || { echo "rocprof failed"; tail -20 gpurun_out/prof.err; exit 1; }
  python tools/trace_window.py gpurun_out/prof/bench_kernel_trace.csv gpurun_out/prof_bench.json | tee gpurun_out/prof_window.txt
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_fetch" -o pmc -- python3 "$R/tools/prof_kernels.py" 5 > "$R/gpurun_out/pmc_fetch.log" 2>&1) || { echo "pmc fetch failed"; tail -20 gpurun_out/pmc_fetch.log; exit 1; }
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_write" -o pmc -- python3 "$R/tools/prof_kernels.py" 5 > "$R/gpurun_out/pmc_write.log" 2>&1) || { echo "pmc write failed"; tail -20 gpurun_out/pmc_write.log; exit 1; }
  python tools/pmc_summary.py gpurun_out/pmc_fetch/pmc_counter_collection.csv gpurun_out/pmc_write/pmc_counter_collection.csv gpurun_out/pmc_traffic.json
  bash tools/pmc_layouts.sh || { echo "pmc layouts failed"; exit 1; }
fi
done

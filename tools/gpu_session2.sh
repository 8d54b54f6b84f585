#!/bin/bash
# full GPU test suite, smoke, headline bench, copy-inclusive side lines
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash tools/gpu_check.sh tests || exit 1
bash tools/gpu_check.sh bench || exit 1
timeout -k 10 300 python bench.py --config rs16_4_4m --copy-inclusive --cpu-seconds 0 > gpurun_out/bench_rs16_ci.json 2> gpurun_out/bench_rs16_ci.err || { tail -20 gpurun_out/bench_rs16_ci.err; exit 1; }
cat gpurun_out/bench_rs16_ci.json
timeout -k 10 300 python bench.py --copy-inclusive --cpu-seconds 0 > gpurun_out/bench_rs10_ci.json 2> gpurun_out/bench_rs10_ci.err || { tail -20 gpurun_out/bench_rs10_ci.err; exit 1; }
cat gpurun_out/bench_rs10_ci.json

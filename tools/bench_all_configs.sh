#!/bin/bash
# Every BASELINE config as a bench side line, with the copy-inclusive leg (host-resident
# data through page-locked buffers) and the CPU baseline.  One JSON line per config.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for c in rs10_4_256k rs4_2_256k rs10_4_1m rs16_4_4m rs2_1_256k; do
  timeout -k 10 300 python bench.py --config $c --copy-inclusive --cpu-seconds 5 > gpurun_out/cfg_$c.json 2> gpurun_out/cfg_$c.err || { tail -20 gpurun_out/cfg_$c.err; exit 1; }
  tail -1 gpurun_out/cfg_$c.json
done

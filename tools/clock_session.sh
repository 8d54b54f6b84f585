#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python tools/clockprobe.py both 400 > gpurun_out/clock_both.txt 2>&1 && \
timeout -k 10 200 python tools/clockprobe.py enc 400 > gpurun_out/clock_enc.txt 2>&1 && \
(cd /tmp && timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_clk" -o clk -- python3 "$R/tools/clockprobe.py" both 150 > "$R/gpurun_out/clock_pmc.txt" 2>&1)
cat gpurun_out/clock_both.txt gpurun_out/clock_enc.txt

#!/bin/bash
# Fused encode + CRC-16 work loop: the fused CRC tests, the A/B of tools/build/v_* variants
# against the product library (tools/fused_ab.sh), a kernel trace of the product's fused path
# (kernel vs combine) and its SQ counters (tools/pmc_fused.sh).  Usage: gpu_fused_prof.sh [test] [ab] [trace] [pmc]
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
for STEP in "${@:-test ab trace pmc}"; do for S in $STEP; do
case $S in
test) timeout -k 10 600 python -u -m pytest tests/test_crc16.py -x -q --timeout 120 --timeout-method thread -m gpu -k "fused" > gpurun_out/t_fused.log 2>&1 || { echo tests failed; tail -30 gpurun_out/t_fused.log; exit 1; }
      tail -2 gpurun_out/t_fused.log ;;
ab) timeout -k 10 400 bash tools/fused_ab.sh > gpurun_out/fused_ab.txt 2>&1 || { echo ab failed; tail gpurun_out/fused_ab.txt; exit 1; }
    cat gpurun_out/fused_ab.txt ;;
trace) (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/proff" -o f -- python3 "$R/tools/prof_fused.py" 30 > "$R/gpurun_out/proff.log" 2>&1) || { echo prof failed; tail gpurun_out/proff.log; exit 1; }
    python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/proff/f_kernel_stats.csv')):
    print(r['Name'][:70], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])" ;;
pmc) timeout -k 10 300 bash tools/pmc_fused.sh > gpurun_out/pmc_fused.txt 2>&1 || { echo pmc failed; tail gpurun_out/pmc_fused.txt; exit 1; }
    cat gpurun_out/pmc_fused.txt ;;
esac
done; done

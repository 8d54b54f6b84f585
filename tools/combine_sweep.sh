#!/bin/bash
# Fused encode + CRC-16: combine-kernel grid sweep (waves per CU; 0 = default 64), stats per run.
# CRC_COMBINE_FOLD=2 runs the combine with its six-bit powers.
set -o pipefail
mkdir -p gpurun_out
for w in ${COMBINE_WPC:-0 32 128 256}; do
  rm -rf gpurun_out/prof_comb_$w
  CRC_FOLDS=3 CRC_WPC=$w timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_comb_$w -o c -- python3 tools/crcbench.py > gpurun_out/comb_$w.txt 2>&1 || { tail gpurun_out/comb_$w.txt; exit 1; }
  echo "== waves_per_cu $w"; grep "fused" gpurun_out/comb_$w.txt
  python3 -c "import csv,sys; [print(r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us') for r in csv.DictReader(open('gpurun_out/prof_comb_$w/c_kernel_stats.csv')) if 'combine' in r['Name']]"
done

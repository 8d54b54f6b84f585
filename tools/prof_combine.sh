#!/bin/bash
# Kernel trace of the fused encode + CRC-16 path (tools/prof_fused.py) for the product library
# and every tools/build/v_* variant: the fused kernel's and the combine kernel's average
# durations side by side.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out
for lib in "" tools/build/v_*/lib/librsmi.so; do
  [ -z "$lib" ] || [ -e "$lib" ] || continue
  tag=$( [ -n "$lib" ] && echo "$lib" | cut -d/ -f3 || echo product )
  rm -rf "gpurun_out/pc_$tag"
  (cd /tmp && RSMI_LIB=${lib:+$R/$lib} timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/pc_$tag" -o f -- python3 "$R/tools/prof_fused.py" 40 > "$R/gpurun_out/pc_$tag.log" 2>&1) || { echo "prof $tag failed"; tail "gpurun_out/pc_$tag.log"; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/pc_$tag/f_kernel_stats.csv')):
    if 'rsmi' in r['Name']: print('$tag'.ljust(10), r['Name'].split('(')[0][5:60].ljust(56), r['Calls'], 'avg', round(float(r['AverageNs'])/1e3,1), 'min', round(float(r['MinNs'])/1e3,1), 'us')"
done

#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per launch for the Split-layout (UA) kernels and the fused encode +
# CRC-16, next to the pitched ones (one PMC pass per counter and mode; tools/pmc_summary.py).
cd "$(dirname "$0")/.."
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
for mode in split fused; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_${mode}_$ctr" -o pmc -- python3 "$R/tools/prof_kernels.py" 5 $mode > "$R/gpurun_out/pmc_${mode}_$ctr.log" 2>&1) || { echo "pmc $mode $ctr failed"; tail -20 gpurun_out/pmc_${mode}_$ctr.log; exit 1; }
  done
  python3 tools/pmc_summary.py gpurun_out/pmc_${mode}_FETCH_SIZE/pmc_counter_collection.csv gpurun_out/pmc_${mode}_WRITE_SIZE/pmc_counter_collection.csv gpurun_out/pmc_traffic_${mode}.json
done
# fold the UA kernels' figures into the bench's table (bench.py reads profiles/pmc_traffic.json
# by kernel label; the fused line's label names two kernels and stays without one)
python3 - <<'PY'
import json, os
path = "gpurun_out/pmc_traffic.json"
table = json.load(open(path)) if os.path.exists(path) else {}
table.update({k: v for k, v in json.load(open("gpurun_out/pmc_traffic_split.json")).items() if ",UA" in k})
json.dump(table, open(path, "w"), indent=1)
PY

#!/bin/bash
# Round-4 session j: small fused launches with the coding tables staged while the first rows load
# and 10 rows in flight -- tests, then kernel traces of the latency tool at 4 KiB, 256 KiB and
# 1 MiB for the product, the previous commit (prev) and 6 rows in flight (ring6).
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_crc16.py -m gpu > $O/pytest_crc16.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_crc16.log; exit 1; }
tail -1 $O/pytest_crc16.log
prof() {  # name, env..., then sizes
  local name=$1; shift
  for B in 4096 262144 1048576; do
    (cd /tmp && env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_${name}_$B" -o lat -- "$R/tools/build/latency" $B > "$R/$O/prof_${name}_$B.log" 2>&1) || { echo "rocprof $name $B failed"; tail -20 $O/prof_${name}_$B.log; return 1; }
  done
}
for rep in 1 2; do
  prof product$rep RSMI_NONE=1 || exit 1
  prof prev$rep LD_LIBRARY_PATH=$R/tools/build/v_prev/lib || exit 1
  prof ring6$rep LD_LIBRARY_PATH=$R/tools/build/v_ring6/lib || exit 1
done
python3 - <<'PY'
import csv, glob, re
for f in sorted(glob.glob("gpurun_out/r04j/prof_*/lat_kernel_stats.csv")):
    tag = f.split("/")[2]
    for r in csv.DictReader(open(f)):
        n = re.sub(r"\(.*", "", r["Name"]).replace("void rsmi::", "")
        if "fused" in n or "rs_fast_kernel" in n:
            print(f'{tag:28s} {n:50s} {r["Calls"]:>5} avg {float(r["AverageNs"])/1000:7.2f} us')
PY
grep -H "lone Put" $O/prof_*.log | sed "s|gpurun_out/r04j/||" | cut -c1-110
for rep in 1 2; do
  timeout -k 10 200 ./tools/build/latency > $O/latency_product$rep.txt 2>&1 || { echo "latency failed"; exit 1; }
  LD_LIBRARY_PATH=$R/tools/build/v_prev/lib timeout -k 10 200 ./tools/build/latency > $O/latency_prev$rep.txt 2>&1 || { echo "latency prev failed"; exit 1; }
done
grep -H "lone Put" $O/latency_*.txt | sed "s|gpurun_out/r04j/||" | cut -c1-110

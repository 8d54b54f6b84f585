#!/bin/bash
# SQ counters of the fused encode + CRC kernel next to the plain encode (two passes, each
# within the per-block counter limits).  Usage: pmc_fused.sh [lib-variant-path]
cd "$(dirname "$0")/.."
R=$(pwd)
export TMPDIR=/tmp
[ -n "$1" ] && export RSMI_LIB=$R/$1
mkdir -p gpurun_out
(cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d "$R/gpurun_out/pmcf1" -o pmc -- python3 "$R/tools/prof_fused.py" 3 > "$R/gpurun_out/pmcf1.log" 2>&1) || { echo pass1 failed; tail gpurun_out/pmcf1.log; exit 1; }
(cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$R/gpurun_out/pmcf2" -o pmc -- python3 "$R/tools/prof_fused.py" 3 > "$R/gpurun_out/pmcf2.log" 2>&1) || { echo pass2 failed; tail gpurun_out/pmcf2.log; exit 1; }
python3 - <<'PY'
import csv, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in ("gpurun_out/pmcf1/pmc_counter_collection.csv", "gpurun_out/pmcf2/pmc_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:24s} {sum(v) / len(v):16.0f}")
PY

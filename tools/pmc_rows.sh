#!/bin/bash
# SQ counters of the rows passes (tools/crcbench.py rows: the CRC-16 passes with both folds and
# the CRC-32 pass), two PMC passes within the per-block counter limits, averaged per kernel.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_rows1" -o pmc -- python3 "$R/tools/crcbench.py" rows > "$R/gpurun_out/pmc_rows1.log" 2>&1) || { echo pass1 failed; tail gpurun_out/pmc_rows1.log; exit 1; }
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_rows2" -o pmc -- python3 "$R/tools/crcbench.py" rows > "$R/gpurun_out/pmc_rows2.log" 2>&1) || { echo pass2 failed; tail gpurun_out/pmc_rows2.log; exit 1; }
python3 - <<'PY'
import csv, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in ("gpurun_out/pmc_rows1/pmc_counter_collection.csv", "gpurun_out/pmc_rows2/pmc_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "crc" not in k:
            continue
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.0f}   ({len(v)} dispatches)")
    g = sum(d["GRBM_GUI_ACTIVE"]) / max(1, len(d["GRBM_GUI_ACTIVE"])) / 8 if "GRBM_GUI_ACTIVE" in d else 0
    if g and "SQ_ACTIVE_INST_VALU" in d:
        valu = sum(d["SQ_ACTIVE_INST_VALU"]) / len(d["SQ_ACTIVE_INST_VALU"]) * 4 / 1024
        print(f"   VALU-busy ~{valu / g * 100:.0f}% of the SIMDs' cycles (quad-cycles x 4 / 1024 SIMDs / GRBM per XCD)")
    if g and "SQ_VALU_MFMA_BUSY_CYCLES" in d:
        mf = sum(d["SQ_VALU_MFMA_BUSY_CYCLES"]) / len(d["SQ_VALU_MFMA_BUSY_CYCLES"]) / 1024
        print(f"   MFMA-busy ~{mf / g * 100:.0f}%")
PY

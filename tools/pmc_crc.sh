set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
(cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_crc1" -o pmc -- python3 "$R/tools/crcbench.py" > "$R/gpurun_out/pmc_crc1.log" 2>&1) || { echo pass1 failed; tail gpurun_out/pmc_crc1.log; exit 1; }
(cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_crc2" -o pmc -- python3 "$R/tools/crcbench.py" > "$R/gpurun_out/pmc_crc2.log" 2>&1) || { echo pass2 failed; tail gpurun_out/pmc_crc2.log; exit 1; }
echo ok

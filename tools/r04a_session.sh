#!/bin/bash
# Round-4 session a: the new GPU tests (UA4 page-exact, host-fault status, in-place lone
# coalesced calls, launcher), the Split-layout UA bench twice, and the fused encode + CRC-16 A/B
# (product vs tools/build/v_idle), each step under its own time limit.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r04a
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py::test_ua4_page_exact_host_buffer tests/test_crc16.py::test_coalesced_host_fault_reports_err_host tests/test_crc16.py::test_coalesced_lone_call_in_place_on_page_locked_buffer tests/test_multirank.py tests/test_device_group.py > gpurun_out/r04a/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r04a/pytest.log; exit 1; }
tail -3 gpurun_out/r04a/pytest.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --layout split --cpu-seconds 0 --sustained-steps 0 > gpurun_out/r04a/ua_split_$i.json 2>gpurun_out/r04a/ua_split_$i.err || { echo "ua bench failed"; tail gpurun_out/r04a/ua_split_$i.err; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/r04a/ua_split_$i.json')); print('split: encode', j['roofline']['achieved'], 'reconstruct', j['reconstruct']['achieved_GBs'], j['reconstruct']['kernel'], j['verify']['verified'])"
done
# the fused variants must be bit-exact before they are timed
for v in v_px v_pxi v_pxis; do
  RSMI_LIB=$PWD/tools/build/$v/lib/librsmi.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_crc16.py -k "fused or dev_crc" > gpurun_out/r04a/pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -30 gpurun_out/r04a/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r04a/pytest_$v.log)"
done
for rep in 1 2; do
  for lib in "" tools/build/v_idle/lib/librsmi.so tools/build/v_px/lib/librsmi.so tools/build/v_pxi/lib/librsmi.so tools/build/v_pxis/lib/librsmi.so; do
    RSMI_LIB=${lib:+$PWD/$lib} timeout -k 10 200 python tools/fusedab.py >> gpurun_out/r04a/fused_ab.txt 2>gpurun_out/r04a/fused_ab.err || { echo "fusedab failed"; tail gpurun_out/r04a/fused_ab.err; exit 1; }
    RSMI_LIB=${lib:+$PWD/$lib} FUSED_SHAPE=16,4,256,4194304 timeout -k 10 200 python tools/fusedab.py >> gpurun_out/r04a/fused_ab.txt 2>>gpurun_out/r04a/fused_ab.err || { echo "fusedab failed"; tail gpurun_out/r04a/fused_ab.err; exit 1; }
  done
done
cat gpurun_out/r04a/fused_ab.txt

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_crc16.py -x -q --timeout 120 --timeout-method thread > gpurun_out/crc_tests.log 2>&1 || { tail -30 gpurun_out/crc_tests.log; exit 1; }
tail -1 gpurun_out/crc_tests.log
timeout -k 10 300 tests/cpp/build/test_dagnode gpu > gpurun_out/dagnode_gpu.log 2>&1 || { tail -30 gpurun_out/dagnode_gpu.log; exit 1; }
tail -2 gpurun_out/dagnode_gpu.log
timeout -k 10 300 tools/build/bench_dagnode 10 4 262144 512 > gpurun_out/dagnode_rs10_4.txt 2>&1 && cat gpurun_out/dagnode_rs10_4.txt

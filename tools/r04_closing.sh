#!/bin/bash
# Round-4 closing check on the last commit: the whole GPU suite, smoke, the headline bench line
# and the C++ Dag Node suite on the GPU.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04close
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log > $O/pytest_gpu_tail.txt; cat $O/pytest_gpu_tail.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 600 ./tests/cpp/build/test_dagnode gpu > $O/test_dagnode_gpu.log 2>&1 || { echo "test_dagnode gpu failed"; tail -30 $O/test_dagnode_gpu.log; exit 1; }
tail -1 $O/test_dagnode_gpu.log | tee $O/test_dagnode_gpu_tail.txt

#!/bin/bash
# Round-4 session ag: 8 contexts per (k, m, device) for concurrent per-block callers against 4
# -- the Dag Node bench on the GPU codec with the product library and with the lanes8 variant
# (make -C tools variant V=lanes8 FLAGS="-DRSMI_HOST_CALL_LANES=8"), alternated, 2 rounds.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04ag
mkdir -p $O
for r in 1 2; do
  for v in product lanes8; do
    if [ $v = lanes8 ]; then LP=$PWD/tools/build/v_lanes8/lib; else LP=$PWD/filedag-storage_amd/lib; fi
    for shape in "2 1 262144 512" "10 4 262144 512" "16 4 4194304 64"; do
      LD_LIBRARY_PATH=$LP timeout -k 10 300 ./tools/build/bench_dagnode $shape > $O/dn.log 2>&1 || { echo "bench $v failed"; tail $O/dn.log; exit 1; }
      echo "r$r $v RS($shape): $(grep -E "^RESULT" $O/dn.log | cut -c8-)" >> $O/lanes_ab.txt
    done
  done
done
cat $O/lanes_ab.txt

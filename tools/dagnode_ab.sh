#!/bin/bash
# Same-box A/B of library variants on the Dag Node bench, GPU codec only: the product library and
# every tools/build/v_*/lib/librsmi.so (through LD_LIBRARY_PATH), alternated DN_ROUNDS times (default
# 2) per shape, so box drift shows as spread, not as a difference; summary per leg by
# tools/dagnode_ab_table.py.  DN_SHAPES: "k m B N" shapes (default RS(2,1) / RS(10,4) 256 KiB x 512,
# RS(16,4) 4 MiB x 64).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${DN_OUT:-gpurun_out/dagnode_ab.jsonl}
: > $OUT
IFS=';' read -ra SHAPES <<< "${DN_SHAPES:-2 1 262144 512;10 4 262144 512;16 4 4194304 64}"
for r in $(seq 1 ${DN_ROUNDS:-2}); do
  for shape in "${SHAPES[@]}"; do
    for lib in filedag-storage_amd/lib tools/build/v_*/lib; do
      [ -e "$lib/librsmi.so" ] || continue
      v=$(basename $(dirname $lib)); [ "$lib" = filedag-storage_amd/lib ] && v=product
      LD_LIBRARY_PATH=$(pwd)/$lib timeout -k 10 300 ./tools/build/bench_dagnode $shape > gpurun_out/dn_ab.log 2>&1 || { echo "bench $v $shape failed"; tail gpurun_out/dn_ab.log; exit 1; }
      grep '^RESULT ' gpurun_out/dn_ab.log | sed "s/^RESULT {/{\"variant\": \"$v\", /" >> $OUT
    done
    echo "round $r $shape done"
  done
done
python3 tools/dagnode_ab_table.py $OUT

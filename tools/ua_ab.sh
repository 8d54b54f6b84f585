#!/bin/bash
# A/B of the Split-layout (UA) kernels in the bench's own context: the product library, then
# every tools/build/v_* variant (RSMI_LIB), twice, alternating.  Prints encode / reconstruct GB/s.
cd "$(dirname "$0")/.."
for rep in 1 2; do
  for lib in filedag-storage_amd/lib/librsmi.so tools/build/v_*/lib/librsmi.so; do
    for cfg in rs10_4_256k rs10_4_1m; do
      out=$(RSMI_LIB=$(pwd)/$lib timeout -k 10 200 python bench.py --config $cfg --layout split --steps 30 --sustained-steps 0 --cpu-seconds 0 2>/dev/null) || { echo "$lib $cfg failed"; exit 1; }
      echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('reconstruct',{}); print('$lib', '$cfg', 'enc', d['roofline']['achieved'], 'rec', r.get('achieved_GBs'), 'verified', d['verify']['verified'])"
    done
  done
done

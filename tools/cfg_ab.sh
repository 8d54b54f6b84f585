#!/bin/bash
# A/B of every BASELINE config's device-resident line: the product library against each
# tools/build/v_* variant (RSMI_LIB), twice, alternating.  Prints encode / reconstruct GB/s.
cd "$(dirname "$0")/.."
# REPS (default 2) alternations; CFGS (default every config) the configs
for rep in $(seq 1 ${REPS:-2}); do
  for lib in filedag-storage_amd/lib/librsmi.so tools/build/v_*/lib/librsmi.so; do
    for cfg in ${CFGS:-rs10_4_256k rs4_2_256k rs10_4_1m rs16_4_4m rs2_1_256k}; do
      out=$(RSMI_LIB=$(pwd)/$lib timeout -k 10 200 python bench.py --config $cfg --steps 30 --sustained-steps 0 --cpu-seconds 0 2>/dev/null) || { echo "$lib $cfg failed"; exit 1; }
      echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('reconstruct',{}); print('$lib'.split('/')[-3], '$cfg', 'value', d['value'], 'enc', d['roofline']['achieved'], 'rec', r.get('achieved_GBs'))"
    done
  done
done

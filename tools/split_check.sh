#!/bin/bash
# The Split-layout side lines next to the pitched ones on one box, twice (encode / reconstruct
# GB/s from bench.py), plus the fused CRC on the Split layout.
cd "$(dirname "$0")/.."
for rep in 1 2; do
  for args in "--config rs10_4_256k --layout split" "--config rs10_4_1m --layout split" "--config rs10_4_256k" "--config rs10_4_1m" "--fused-crc --layout split"; do
    out=$(timeout -k 10 200 python bench.py $args --steps 30 --sustained-steps 0 --cpu-seconds 0 2>/dev/null) || { echo "$args failed"; exit 1; }
    echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('reconstruct',{}); print('$args', 'enc', d['roofline']['achieved'], d['roofline']['frac'], 'rec', r.get('achieved_GBs'), 'value', d['value'], 'verified', d['verify']['verified'])"
  done
done

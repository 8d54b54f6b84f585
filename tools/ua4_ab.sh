#!/bin/bash
# A/B of the unaligned-window load forms on the Split layout (bench.py --layout split, RS(10,4)
# 256 KiB x 4096: UA encode + UA 1-row reconstruct): the product library against every
# tools/build/v_* variant (RSMI_UA_DWORD_LOADS 0 / 1 / 2), alternated twice.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in 1 2; do
  for lib in "" tools/build/v_*/lib/librsmi.so; do
    [ -z "$lib" ] || [ -e "$lib" ] || continue
    RSMI_LIB=${lib:+$PWD/$lib} timeout -k 10 200 python bench.py --layout split --cpu-seconds 0 --sustained-steps 0 ${UA_BENCH_ARGS:-} > gpurun_out/ua4.json 2> gpurun_out/ua4.err || { echo "bench failed"; tail gpurun_out/ua4.err; exit 1; }
    python3 -c "
import json; j=json.load(open('gpurun_out/ua4.json'))
print(('$lib'.split('/')[2] if '$lib' else 'product').ljust(10), 'encode', j['roofline']['achieved'], '| reconstruct', j['reconstruct']['achieved_GBs'], 'GB/s', j['reconstruct']['kernel'], 'verified', j['verify']['verified'])"
  done
done | tee gpurun_out/ua4_ab.txt

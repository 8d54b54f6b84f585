#!/bin/bash
# Split-layout reconstruct: is the gap to the pitched kernels the unaligned loads or the pitch?
# The same bench (RS(10,4) 256 KiB x 4096, encode + 1-row ReconstructData) on the Split layout
# (unaligned-window kernels at pitch S = 26 215), on an aligned layout at pitch roundup16(S) =
# 26 224 (the aligned kernels, nearly the same HBM mapping), and at the recommended 32 KiB pitch;
# two alternated rounds.  Output: encode / reconstruct kernel GB/s per layout.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in 1 2; do
  for args in "--layout split" "--pitch 26224" "--pitch 32768"; do
    timeout -k 10 200 python bench.py $args --cpu-seconds 0 --sustained-steps 0 > gpurun_out/uapitch.json 2> gpurun_out/uapitch.err || { echo "bench $args failed"; tail gpurun_out/uapitch.err; exit 1; }
    python3 -c "
import json; j=json.load(open('gpurun_out/uapitch.json'))
print('$args'.ljust(16), 'pitch', j['config']['row_pitch'], 'encode', j['roofline']['achieved'], 'GB/s', j['roofline']['kernel'], '| reconstruct', j['reconstruct']['achieved_GBs'], 'GB/s', j['reconstruct']['kernel'])"
  done
done | tee gpurun_out/ua_pitch_ab.txt

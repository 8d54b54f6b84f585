#!/bin/bash
# Row-pitch A/B in the bench's own context: bench.py --config C --pitch P for each pitch of
# PITCHES (0 = rsmi_recommended_pitch), alternated ROUNDS times (default 2).  Prints the encode
# and reconstruct kernel rates.  Usage: PITCHES="0 131072 ..." tools/pitch_ab.sh <config>
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for p in ${PITCHES:-0}; do
    timeout -k 10 200 python bench.py --config "$1" --pitch "$p" --cpu-seconds 0 --sustained-steps 0 \
      > gpurun_out/pab.json 2> gpurun_out/pab.err || { echo "bench failed"; tail gpurun_out/pab.err; exit 1; }
    python3 -c "
import json; j=json.load(open('gpurun_out/pab.json'))
rec=j.get('reconstruct') or {}
print('$1', 'pitch', j['config']['row_pitch'], 'encode', j['roofline']['achieved'], 'GB/s', j['roofline']['frac'], '| reconstruct', rec.get('achieved_GBs'), '| value', j['value'], 'verified', j['verify']['verified'])"
  done
done

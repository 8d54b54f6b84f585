#!/bin/bash
# A/B of kernel knobs in the bench's own context (bench.py --option KEY=VALUE), rounds
# interleaved across processes.  Interleaved in-process sweeps (optab.py, ntsweep.py) change
# what each kernel finds in the caches -- the store-policy A/B there pointed the wrong way.
# usage: [CFG=rs4_2_256k] tools/bench_ab.sh ROUNDS "" "lds_dma=1" "store_aux=18" ...   ("" = defaults)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
R=$1
CFG=${CFG:-rs10_4_256k}
shift
for i in $(seq 1 "$R"); do
  for v in "$@"; do
    args=()
    for kv in $v; do
      case $kv in pitch=*) args+=(--pitch "${kv#pitch=}") ;; *) args+=(--option "$kv") ;; esac
    done
    out=gpurun_out/ab_${CFG}_$(echo "${v:-default}" | tr ' =' '_-')_$i.json
    timeout -k 10 120 python bench.py --config "$CFG" --cpu-seconds 0 "${args[@]}" > "$out" 2>/dev/null || { echo "bench failed: $v"; exit 1; }
    python - "$out" "${v:-default}" <<'PY'
import json, sys
j = json.load(open(sys.argv[1]))
r = j.get("reconstruct") or {}
print(f"{j['config']['workload'][:44]:44s} {sys.argv[2]:18s} value {j['value']:8.1f}  enc {j['roofline']['achieved']:7.1f}  "
      f"rec {r.get('achieved_GBs', 0):7.1f}  {j['roofline']['kernel']} | {r.get('kernel', '-')}")
PY
  done
done

#!/bin/bash
# Same-box A/B of one environment variable on the Dag Node bench (GPU codec, product library):
# ENV_AB="NAME" with values ENV_VALUES (default "0 1"), alternated DN_ROUNDS times (default 2) per
# shape; summary per leg by tools/dagnode_ab_table.py (variants named NAME=value).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${DN_OUT:-gpurun_out/dagnode_env_ab.jsonl}
NAME=${ENV_AB:?set ENV_AB to the variable to vary}
: > $OUT
IFS=';' read -ra SHAPES <<< "${DN_SHAPES:-2 1 262144 512;10 4 262144 512;16 4 4194304 64}"
for r in $(seq 1 ${DN_ROUNDS:-2}); do
  for shape in "${SHAPES[@]}"; do
    for v in ${ENV_VALUES:-0 1}; do
      env "$NAME=$v" timeout -k 10 300 ./tools/build/bench_dagnode $shape > gpurun_out/dn_env_ab.log 2>&1 || { echo "bench $NAME=$v $shape failed"; tail gpurun_out/dn_env_ab.log; exit 1; }
      grep '^RESULT ' gpurun_out/dn_env_ab.log | sed "s/^RESULT {/{\"variant\": \"$NAME=$v\", /" >> $OUT
    done
    echo "round $r $shape done"
  done
done
python3 tools/dagnode_ab_table.py $OUT

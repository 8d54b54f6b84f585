#!/bin/bash
# Side measurements for every BASELINE config + multi-rank rehearsal on one GPU.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail gpurun_out/bench_default.err; exit 1; }
for cfg in rs4_2_256k rs10_4_1m rs16_4_4m rs2_1_256k; do
  timeout -k 10 300 python bench.py --config $cfg --copy-inclusive --cpu-seconds 5 > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err || { tail gpurun_out/bench_$cfg.err; exit 1; }
done
timeout -k 10 300 python bench.py --copy-inclusive --cpu-seconds 0 > gpurun_out/bench_default_copy.json 2> gpurun_out/bench_default_copy.err || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --share-device --steps 10 --warmup 2 --blocks 1024 > gpurun_out/bench_2rank_shared.json 2> gpurun_out/bench_2rank.err || { tail gpurun_out/bench_2rank.err; exit 1; }
cat gpurun_out/bench_*.json

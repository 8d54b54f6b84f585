#!/bin/bash
# One GPU session as a list of legs, run in order; each leg has its own time limit and the chain
# stops at the first failure (a GPU step that faults, aborts or times out ends the session).
#
#   tools/gpu_session.sh OUT leg [leg ...]      results under gpurun_out/OUT/
#
# Legs:
#   tests            the whole GPU suite (pytest -m gpu)
#   pytest:EXPR      the GPU tests matching -k EXPR
#   smoke            __graft_entry__.smoke()
#   bench            the headline bench line (bench.py, defaults)
#   side             side lines: Split layout, fused CRC-16, configs[4] device group, two ranks
#   configs          every BASELINE config as a bench line (tools/bench_all_configs.sh)
#   crcbench         the CRC passes and the fused encode + CRC-16 against the encode
#   fused_ab         the fused encode + CRC-16, product library against every tools/build/v_* variant
#   prof             rocprofv3 kernel trace of the headline bench (+ the trace-window cross-check)
#                    and the FETCH_SIZE / WRITE_SIZE passes (PMC traffic per kernel)
#   dagnode_suite    the C++ Dag Node suite on the GPU
#   dagnode_cmp      the Dag Node bench, GPU codec beside the CPU codec (tools/dagnode_cpu_vs_gpu.sh)
#   dagnode_ab       the Dag Node bench (GPU codec) on the product library and every tools/build/v_* variant
#   ua_ab            the Split-layout (UA) kernels: product library against every tools/build/v_*
#                    variant (tools/ua_ab.sh), then each library's FETCH_SIZE / WRITE_SIZE passes
#   dagnode_env_ab   the Dag Node bench with ENV_AB=<variable> at ENV_VALUES (default 0 1), alternated
#   latency          per-block call latencies (tools/latency)
#   dagnode_trace    the Dag Node bench with the batched repair's phase timeline (BENCH_DAGNODE_TRACE)
#   groupcost        a small zero-copy group's fixed cost: launch, dispatch, load round trip, tail
#   latency_ab       lone-call latencies on the product library and every tools/build/v_* variant
#   threads          concurrent coalesced encodes, contexts x lanes (tools/latency --threads)
#   threads_pipe     the same at 16 threads, option coalesce_pipeline off / on alternated (THREADS_CFG=pipe)
#   threads_ab       THREADS_AB_CFG (default flag) on the product library and each tools/build/v_* variant
#   threads_flag     1 and 16 threads, option coalesce_flag off / on alternated (THREADS_CFG=flag)
#   group_sweep      one thread, in-place host calls of 1..256 blocks back to back (tools/latency --group-sweep)
#   threads_traced   the same under rocprofv3 --kernel-trace (crash report: tools/latency.cpp)
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/${1:?usage: gpu_session.sh OUT leg...}
shift
mkdir -p "$O"
export TMPDIR=/tmp
fail() { echo "$1 failed"; tail -40 "$2"; exit 1; }
for LEG in "$@"; do
case $LEG in
tests)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || fail pytest $O/pytest_gpu.log
  tail -3 $O/pytest_gpu.log | tee $O/pytest_gpu_tail.txt ;;
pytest:*)
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${LEG#pytest:}" > $O/pytest_k.log 2>&1 || fail pytest $O/pytest_k.log
  tail -3 $O/pytest_k.log ;;
smoke)
  timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || fail smoke $O/smoke.log
  tail -1 $O/smoke.log ;;
bench)
  timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || fail bench $O/bench.err
  cat $O/bench.json ;;
side)
  for args in "--layout split" "--fused-crc" "--fused-crc --layout split"; do
    f=$O/side_$(echo $args | tr -d ' -').json
    timeout -k 10 300 python bench.py $args --cpu-seconds 0 > $f 2> $f.err || fail "bench $args" $f.err
    cat $f
  done
  timeout -k 10 300 python bench.py --config rs16_4_4m --copy-inclusive --group 0,0 --cpu-seconds 0 > $O/side_group.json 2> $O/side_group.err || fail "bench --group" $O/side_group.err
  cat $O/side_group.json
  timeout -k 10 300 python bench.py --gpus 2 --share-device --cpu-seconds 0 > $O/side_gpus2.json 2> $O/side_gpus2.err || fail "bench --gpus 2" $O/side_gpus2.err
  cat $O/side_gpus2.json ;;
configs)
  timeout -k 10 900 bash tools/bench_all_configs.sh > $O/configs.txt 2>&1 || fail configs $O/configs.txt
  cp gpurun_out/cfg_*.json $O/ 2>/dev/null; cat $O/configs.txt ;;
crcbench)
  timeout -k 10 300 python tools/crcbench.py > $O/crcbench.txt 2>&1 || fail crcbench $O/crcbench.txt
  cat $O/crcbench.txt ;;
fused_ab)
  FUSED_ROUNDS=${FUSED_ROUNDS:-2} timeout -k 10 600 bash tools/fused_ab.sh > $O/fused_ab.txt 2>&1 || fail fused_ab $O/fused_ab.txt
  cat $O/fused_ab.txt ;;
prof)
  rm -rf $O/prof $O/pmc_fetch $O/pmc_write
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o bench -- python3 "$R/bench.py" --cpu-seconds 0 > "$R/$O/prof_bench.json" 2> "$R/$O/prof.err") || fail rocprof $O/prof.err
  python tools/trace_window.py $O/prof/bench_kernel_trace.csv $O/prof_bench.json $O/trace_window.json | tee $O/prof_window.txt
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$R/$O/pmc_fetch" -o pmc -- python3 "$R/tools/prof_kernels.py" 5 > "$R/$O/pmc_fetch.log" 2>&1) || fail "pmc fetch" $O/pmc_fetch.log
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$R/$O/pmc_write" -o pmc -- python3 "$R/tools/prof_kernels.py" 5 > "$R/$O/pmc_write.log" 2>&1) || fail "pmc write" $O/pmc_write.log
  python tools/pmc_summary.py $O/pmc_fetch/pmc_counter_collection.csv $O/pmc_write/pmc_counter_collection.csv $O/pmc_traffic.json ;;
dagnode_suite)
  timeout -k 10 600 ./tests/cpp/build/test_dagnode gpu > $O/test_dagnode_gpu.log 2>&1 || fail test_dagnode $O/test_dagnode_gpu.log
  grep -E "concurrent|group commit" $O/test_dagnode_gpu.log; tail -1 $O/test_dagnode_gpu.log | tee $O/test_dagnode_gpu_tail.txt ;;
dagnode_cmp)
  timeout -k 10 900 bash tools/dagnode_cpu_vs_gpu.sh > $O/dagnode_cpu_vs_gpu.txt 2>&1 || fail "dagnode cmp" $O/dagnode_cpu_vs_gpu.txt
  cp gpurun_out/dagnode_cmp.jsonl gpurun_out/dn_phases.jsonl $O/
  grep -v " done$" $O/dagnode_cpu_vs_gpu.txt | head -60 ;;
dagnode_ab)
  DN_OUT=$O/dagnode_ab.jsonl timeout -k 10 1000 bash tools/dagnode_ab.sh > $O/dagnode_ab.txt 2>&1 || fail "dagnode ab" $O/dagnode_ab.txt
  grep -v " done$" $O/dagnode_ab.txt ;;
ua_ab)
  timeout -k 10 600 bash tools/ua_ab.sh > $O/ua_ab.txt 2>&1 || fail ua_ab $O/ua_ab.txt
  cat $O/ua_ab.txt
  for lib in filedag-storage_amd/lib/librsmi.so tools/build/v_*/lib/librsmi.so; do
    v=$(basename $(dirname $(dirname $lib))); [ "$v" = filedag-storage_amd ] && v=product
    export RSMI_LIB=$R/$lib
    for ctr in FETCH_SIZE WRITE_SIZE; do
      (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$R/$O/pmc_${v}_$ctr" -o pmc -- python3 "$R/tools/prof_kernels.py" 5 split > "$R/$O/pmc_${v}_$ctr.log" 2>&1) || fail "pmc $v $ctr" $O/pmc_${v}_$ctr.log
    done
    unset RSMI_LIB
    python tools/pmc_summary.py $O/pmc_${v}_FETCH_SIZE/pmc_counter_collection.csv $O/pmc_${v}_WRITE_SIZE/pmc_counter_collection.csv $O/pmc_ua_$v.json
    echo "$v: $(cat $O/pmc_ua_$v.json | tr -d '\n')"
  done ;;
dagnode_env_ab)
  DN_OUT=$O/dagnode_env_ab.jsonl timeout -k 10 1000 bash tools/dagnode_env_ab.sh > $O/dagnode_env_ab.txt 2>&1 || fail "dagnode env ab" $O/dagnode_env_ab.txt
  grep -v " done$" $O/dagnode_env_ab.txt ;;
latency)
  timeout -k 10 200 ./tools/build/latency > $O/latency.txt 2>&1 || fail latency $O/latency.txt
  cat $O/latency.txt ;;
dagnode_trace)
  # the Dag Node bench (GPU codec) with the batched repair's phase timeline (TRACE lines,
  # tools/trace_timeline.py), RS(16,4) 4 MiB and RS(10,4) 256 KiB, twice each
  : > $O/dagnode_trace.txt
  for rep in 1 2; do
    for shape in "16 4 4194304 64" "10 4 262144 512"; do
      BENCH_DAGNODE_TRACE=1 timeout -k 10 300 ./tools/build/bench_dagnode $shape >> $O/dagnode_trace.txt 2>&1 || fail "dagnode_trace $shape" $O/dagnode_trace.txt
    done
  done
  python3 tools/trace_timeline.py $O/dagnode_trace.txt
  grep -E "^(PutMany|Repair|RepairDataNode)" $O/dagnode_trace.txt ;;
groupcost)
  # a small zero-copy group's fixed cost split (tools/groupcost_probe.hip), page-locked host data,
  # then device data, twice each
  : > $O/groupcost.txt
  for rep in 1 2; do
    for a in "" --device-data; do
      timeout -k 10 120 ./tools/build/groupcost_probe $a >> $O/groupcost.txt 2>&1 || fail "groupcost $a" $O/groupcost.txt
    done
  done
  cat $O/groupcost.txt ;;
latency_ab)
  # lone-call latencies (256 KiB, 4 MiB) on the product library and every tools/build/v_* variant,
  # alternated three times
  : > $O/latency_ab.txt
  for rep in 1 2 3; do
    for lib in filedag-storage_amd/lib tools/build/v_*/lib; do
      v=$(basename $(dirname $lib)); [ "$lib" = filedag-storage_amd/lib ] && v=product
      echo "== $v (round $rep)" >> $O/latency_ab.txt
      LD_LIBRARY_PATH=$R/$lib timeout -k 10 200 ./tools/build/latency 262144 4194304 >> $O/latency_ab.txt 2>&1 || fail "latency_ab $v" $O/latency_ab.txt
    done
  done
  grep -E "^==|lone Put|Split copy" $O/latency_ab.txt | cut -c1-200 ;;
threads)
  timeout -k 10 300 ./tools/build/latency --threads > $O/threads.txt 2>&1 || fail threads $O/threads.txt
  cat $O/threads.txt ;;
threads_pipe)
  THREADS_CFG=pipe timeout -k 10 400 ./tools/build/latency --threads > $O/threads_pipe.txt 2>&1 || fail threads_pipe $O/threads_pipe.txt
  cat $O/threads_pipe.txt ;;
threads_ab)
  # the threads configuration THREADS_AB_CFG (default flag) on the product library and every
  # tools/build/v_* variant (LD_LIBRARY_PATH), alternated twice
  : > $O/threads_ab.txt
  for rep in 1 2; do
    for lib in filedag-storage_amd/lib tools/build/v_*/lib; do
      v=$(basename $(dirname $lib)); [ "$lib" = filedag-storage_amd/lib ] && v=product
      echo "== $v (round $rep)" >> $O/threads_ab.txt
      LD_LIBRARY_PATH=$R/$lib THREADS_CFG=${THREADS_AB_CFG:-flag} timeout -k 10 300 ./tools/build/latency --threads >> $O/threads_ab.txt 2>&1 || fail "threads_ab $v" $O/threads_ab.txt
    done
  done
  grep -E "^==|threads x" $O/threads_ab.txt | cut -c1-200 ;;
threads_flag)
  THREADS_CFG=flag timeout -k 10 400 ./tools/build/latency --threads > $O/threads_flag.txt 2>&1 || fail threads_flag $O/threads_flag.txt
  cat $O/threads_flag.txt ;;
group_sweep)
  timeout -k 10 300 ./tools/build/latency --group-sweep > $O/group_sweep.txt 2>&1 || fail group_sweep $O/group_sweep.txt
  cat $O/group_sweep.txt ;;
kernarg_trace)
  # the Dag Node bench (GPU codec, RS(10,4) 256 KiB) under a kernel trace with HIP_FORCE_DEV_KERNARG
  # 0 and 1: which kernels each setting dispatches, and their count and time (tools/kernel_counts.py)
  for v in 0 1; do
    rm -rf $O/kt_$v
    (cd /tmp && HIP_FORCE_DEV_KERNARG=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/kt_$v" -o t -- "$R/tools/build/bench_dagnode" 10 4 262144 512 > "$R/$O/kt_$v.log" 2>&1) || fail "kernarg trace $v" $O/kt_$v.log
  done
  python3 tools/kernel_counts.py $O/kt_0/t_kernel_trace.csv $O/kt_1/t_kernel_trace.csv | tee $O/kernarg_trace.txt ;;
threads_traced)
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$O/trace" -o t -- "$R/tools/build/latency" --threads > "$R/$O/threads_traced.txt" 2>&1) || fail "traced threads" $O/threads_traced.txt
  tail -5 $O/threads_traced.txt ;;
*)
  echo "unknown leg $LEG"; exit 2 ;;
esac
done

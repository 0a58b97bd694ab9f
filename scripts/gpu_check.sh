#!/bin/bash
# One GPU-box session: smoke -> pytest -m gpu -> bench (small + full) -> rocprofv3 kernel stats.
# Every GPU step has its own time limit; after a crash/abort/timeout nothing further runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ST=gpurun_out/status.txt
: > $ST
ok() {  # rc 0 = pass, 1 = test failures (no fault) -> continue; anything else -> stop
  local name=$1 rc=$2
  echo "$name rc=$rc" | tee -a $ST
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "STOP after $name" | tee -a $ST; exit $rc; fi
}
STAGES=${STAGES:-"smoke pytest bench prof"}
for s in $STAGES; do
  case $s in
    sortdbg) timeout -k 10 300 python scripts/sort_debug.py ${SORT_SIZES:-} > gpurun_out/sortdbg.log 2>&1; ok sortdbg $? ;;
    pytest_rest) timeout -k 10 1200 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread ${DESELECT:-} > gpurun_out/pytest_gpu.log 2>&1; ok pytest_rest $? ;;
    distest) timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py -v -m gpu -p no:cacheprovider --timeout 360 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1; ok distest $? ;;
    bench20) timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench20.log 2>&1; ok bench20 $? ;;
    bench_dist)  # the multi-GPU code path at N = 1 (nccl process group, broadcast + unpack, all-gathers, secondaries)
      timeout -k 10 900 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --dist --steps ${DSTEPS:-20} --warmup 3 --no-cpu > gpurun_out/bench_dist.log 2>&1; ok bench_dist $? ;;
    c5ab)  # C5 ray-kernel A/B over build/variants/*.so in the order ORDER (names), one process per run
      for n in ${ORDER:?set ORDER}; do
        MESH_AMD_LIB=$PWD/build/variants/$n.so timeout -k 10 400 python scripts/c5_ab.py --reps ${REPS:-5} ${C5AB_ARGS:-} >> gpurun_out/c5ab.jsonl 2> gpurun_out/c5ab_$n.err; ok c5ab_$n $?
      done ;;
    benchab)  # C3 bench.py over build/variants/*.so in the order ORDER (names), one process per run
      for n in ${ORDER:?set ORDER}; do
        MESH_AMD_LIB=$PWD/build/variants/$n.so timeout -k 10 400 python bench.py --steps ${BSTEPS:-10} --warmup 2 --no-cpu >> gpurun_out/benchab.jsonl 2> gpurun_out/benchab_$n.err; ok benchab_$n $?
      done ;;
    cutprobe)  # entry cut build phases over build/variants/*.so in the order ORDER
      for n in ${ORDER:?set ORDER}; do
        MESH_AMD_LIB=$PWD/build/variants/$n.so timeout -k 10 300 python scripts/cut_build_probe.py >> gpurun_out/cutprobe.jsonl 2> gpurun_out/cutprobe_$n.err; ok cutprobe_$n $?
      done ;;
    smoke)  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; ok smoke $? ;;
    pytest) timeout -k 10 1200 python -u -m pytest tests -v -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; ok pytest $? ;;
    bench_small) timeout -k 10 600 python bench.py --queries 10000000 --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_small.log 2>&1; ok bench_small $? ;;
    variants)  # tuning sweep: every build/variants/*.so through the 10M-query bench (env MESH_AMD_LIB)
      for so in build/variants/*.so; do
        n=$(basename $so .so)
        MESH_AMD_LIB=$PWD/$so timeout -k 10 ${VTIMEOUT:-300} python bench.py --queries ${VQ:-10000000} --steps ${VSTEPS:-5} --warmup 2 --no-cpu > gpurun_out/var_$n.log 2>&1; ok var_$n $?
      done ;;
    variants_check)  # closest-point parity tests through every build/variants/*.so (env MESH_AMD_LIB)
      for so in build/variants/*.so; do
        n=$(basename $so .so)
        MESH_AMD_LIB=$PWD/$so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "c1 or c2 or non_finite or c3_sample or entry_cut or c3_stream_shards or c3_headline or tiny or degenerate or far_and or on_vertices or cooperative or deep_tree or tied or batch_bit or barycentric or device_api" > gpurun_out/varchk_$n.log 2>&1; ok varchk_$n $?
      done ;;
    variants_c5)  # the same sweep through the C5 ray workloads
      for so in build/variants/*.so; do
        n=$(basename $so .so)
        MESH_AMD_LIB=$PWD/$so timeout -k 10 600 python scripts/bench_configs.py --configs c5 --reps 3 > gpurun_out/varc5_$n.log 2>&1; ok varc5_$n $?
      done ;;
    split)  MESH_AMD_STATS_DUMP=1 timeout -k 10 600 python scripts/c3_split.py > gpurun_out/split.log 2>&1; ok split $? ;;
    pytest_quick) timeout -k 10 600 python -u -m pytest tests -v -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread -k "spill or cooperative or c1 or c2 or c3 or rays or alongnormal or visibility" > gpurun_out/pytest_quick.log 2>&1; ok pytest_quick $? ;;
    c5)     timeout -k 10 900 python scripts/bench_configs.py --configs c5 --reps 3 > gpurun_out/bench_c5.log 2>&1; ok c5 $? ;;
    configs) timeout -k 10 900 python scripts/bench_configs.py > gpurun_out/bench_configs.log 2>&1; ok configs $? ;;
    bench)  timeout -k 10 900 python bench.py > gpurun_out/bench.log 2>&1; ok bench $? ;;
    pmc)    PASSES="${PMC_PASSES:-stats fetch write tcc sq valu valu2 sq2}" TARGET=${PMC_TARGET:-c3} bash scripts/profile_pmc.sh > gpurun_out/pmc_${PMC_TARGET:-c3}.log 2>&1; ok pmc_${PMC_TARGET:-c3} $? ;;
    pmc_cfg) for t in ${PMC_CFGS:-c5 c2}; do PASSES="${PMC_CFG_PASSES:-stats fetch write tcc}" TARGET=$t bash scripts/profile_pmc.sh > gpurun_out/pmc_$t.log 2>&1; ok pmc_$t $?; done ;;
    nptl)   (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OLDPWD/gpurun_out/nptl" -o run -- python3 "$OLDPWD/scripts/numpy_timeline.py" --calls 3 > "$OLDPWD/gpurun_out/nptl.log" 2>&1); ok nptl $? ;;
    facade) timeout -k 10 900 python scripts/bench_configs.py --configs facade --reps 2 > gpurun_out/facade.log 2>&1; ok facade $? ;;
    repl)   timeout -k 10 300 python scripts/replication_timing.py > gpurun_out/repl.log 2>&1; ok repl $? ;;
    bench_stats) MESH_AMD_STATS_DUMP=1 timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_stats.log 2>&1; ok bench_stats $? ;;
    prof_small) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OLDPWD/gpurun_out/prof_small" -o run -- python3 "$OLDPWD/bench.py" --queries 10000000 --steps 2 --warmup 1 --no-cpu > "$OLDPWD/gpurun_out/prof_small.log" 2>&1); ok prof_small $? ;;
    prof)   (cd /tmp && export TMPDIR=/tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$OLDPWD/gpurun_out/prof" -o run -- python3 "$OLDPWD/bench.py" --steps 3 --warmup 1 --no-cpu --no-one-shot > "$OLDPWD/gpurun_out/prof.log" 2>&1); ok prof $? ;;
  esac
done
echo done | tee -a $ST

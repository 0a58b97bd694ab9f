#!/bin/bash
# rocprofv3 passes on the bench (C3 workload): kernel-trace --stats (CSV), then one PMC pass per counter
# group (FETCH_SIZE / WRITE_SIZE / TCC_HIT_sum+TCC_MISS_sum cannot share a pass on gfx950).  Run on the
# GPU box from the repo root; outputs under gpurun_out/pmc/.  Stops at the first failing step.
# TARGET=c5 (or c2, c4 ...): the same passes over one scripts/bench_configs.py config instead, into
# gpurun_out/pmc_<TARGET>/ (scripts/pmc_configs.py summarises them).
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
TARGET=${TARGET:-c3}
OUT=$R/gpurun_out/pmc
[ "$TARGET" = c3 ] || OUT=$R/gpurun_out/pmc_$TARGET
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
Q=${Q:-100000000}
run() {
  local name=$1; shift
  if [ "$TARGET" = c3 ]; then
    timeout -k 10 600 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o run -- python3 "$R/bench.py" --queries $Q --steps 2 --warmup 1 --no-cpu --no-one-shot > "$OUT/$name.log" 2>&1
  else
    MESH_AMD_NO_CPU=1 timeout -k 10 600 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o run -- python3 "$R/scripts/bench_configs.py" --configs $TARGET --reps 1 > "$OUT/$name.log" 2>&1
  fi
  local rc=$?
  echo "$name rc=$rc" | tee -a "$OUT/status.txt"
  [ $rc -eq 0 ] || exit $rc
}
: > "$OUT/status.txt"
# identity of the library the passes measure (bench.py pairs profiles/pmc_traffic.json with it)
(cd "$R" && python3 -c "from mesh_amd import _native; print(_native.build_id())") > "$OUT/build_id.txt" || exit 1
PASSES=${PASSES:-"stats fetch write tcc sq"}
for p in $PASSES; do
  case $p in
    stats) run stats --kernel-trace --stats ;;
    fetch) run fetch --kernel-trace --pmc FETCH_SIZE ;;
    write) run write --kernel-trace --pmc WRITE_SIZE ;;
    tcc)   run tcc --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum ;;
    sq)    run sq --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU ;;
    valu)  run valu --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_ADD_F32 ;;
    valu2) run valu2 --kernel-trace --pmc SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH ;;
    sq2)   run sq2 --kernel-trace --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM ;;
  esac
done
echo done | tee -a "$OUT/status.txt"

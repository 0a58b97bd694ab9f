#!/bin/bash
# One SQ --pmc pass per build/variants/*.so over the 10M-query C3 bench (GPU box, repo root); CSVs under
# gpurun_out/pmcv/<variant>/.  Compare instruction mixes of tuning variants.  Stops at the first failure.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/pmcv
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CTRS=${CTRS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY"}
for so in "$R"/build/variants/*.so; do
  n=$(basename "$so" .so)
  MESH_AMD_LIB=$so timeout -k 10 300 rocprofv3 --kernel-trace --pmc $CTRS --output-format csv -d "$OUT/$n" -o run -- python3 "$R/bench.py" --queries ${Q:-10000000} --steps 2 --warmup 1 --no-cpu > "$OUT/$n.log" 2>&1
  rc=$?
  echo "$n rc=$rc" | tee -a "$OUT/status.txt"
  [ $rc -eq 0 ] || exit $rc
done

#!/bin/bash
# Round-end measurement session on the GPU box: smoke + pytest -m gpu, the C3 bench line, all configs,
# rocprofv3 kernel stats of the C3 bench and of the C5 configs (gpurun_out/; summaries go to profiles/).
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R"
mkdir -p gpurun_out
STAGES="${STAGES:-smoke pytest bench configs prof}" bash scripts/gpu_check.sh || exit $?
grep -q "rc=[^01]" gpurun_out/status.txt && exit 1
bash scripts/prof_config.sh c5
echo "prof_c5 rc=$?" >> gpurun_out/status.txt

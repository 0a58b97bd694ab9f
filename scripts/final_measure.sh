set -u
R=$PWD
mkdir -p gpurun_out
STAGES="configs bench" bash scripts/gpu_check.sh || exit $?
cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c5" -o run -- python3 "$R/scripts/bench_configs.py" --configs c5 --reps 2 > "$R/gpurun_out/prof_c5.log" 2>&1
echo "prof_c5 rc=$?" >> "$R/gpurun_out/status.txt"

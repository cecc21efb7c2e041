# Config 5 (streaming) bench line + kernel-trace stats for profiles/.
set -o pipefail
R=${ROUND:-r01}
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/p5 profiles
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/p5/k" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --config 5 --steps 100 --warmup 10 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/p5/k.log" 2>&1) || exit 11
cp gpurun_out/p5/k/run_kernel_stats.csv profiles/${R}_cfg5_kernel_stats.csv
timeout -k 10 300 python bench.py --config 5 > gpurun_out/p5/bench.log 2>&1 || exit 13
tail -1 gpurun_out/p5/bench.log > profiles/${R}_cfg5_bench.json
cut -c1-600 profiles/${R}_cfg5_bench.json
cp profiles/${R}_cfg5_* gpurun_out/p5/

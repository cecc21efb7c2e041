# Per-kernel split (rocprofv3 kernel-trace stats) of bench configs 3 and 4 (GCC-PHAT).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg34
for C in 3 4; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/cfg34/c$C" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --config $C --engine gcc_phat --steps 10 --warmup 2 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/cfg34/c$C.log" 2>&1) || exit 11
  tail -1 gpurun_out/cfg34/c$C.log | cut -c1-400
  cut -d, -f1-4 gpurun_out/cfg34/c$C/run_kernel_stats.csv | cut -c1-160 | head -8
done

# Per-kernel time split (rocprofv3 kernel-trace stats) of bench configs 3 and 4, both engines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/kstats
for C in 3 4; do
  for E in gcc_phat direct; do
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/kstats/c${C}_$E" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --config $C --engine $E --steps 5 --warmup 1 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/kstats/c${C}_$E.log" 2>&1) || exit 11
    echo "== config $C $E"; cut -d, -f1-4,6 gpurun_out/kstats/c${C}_$E/run_kernel_stats.csv | head -8
  done
done

# Per-kernel time split (rocprofv3 kernel-trace stats) of bench config 2, both engines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/kstats
for E in gcc_phat direct; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/kstats/c2_$E" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --engine $E --steps 100 --warmup 5 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/kstats/c2_$E.log" 2>&1) || exit 11
done
python3 tools/kstats_summary.py gpurun_out/kstats/c2_gcc_phat gpurun_out/kstats/c2_direct

# Profiling pass for the committed profiles/: kernel-trace stats of the bench
# for both engines, then separate FETCH_SIZE / WRITE_SIZE passes.
set -o pipefail
R=${ROUND:-r01}
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc profiles
for E in gcc_phat direct; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/ktrace_$E" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --engine $E --steps 200 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/ktrace_$E.log" 2>&1) || exit 11
  cp gpurun_out/ktrace_$E/run_kernel_stats.csv profiles/${R}_${E}_kernel_stats.csv
  tail -1 gpurun_out/ktrace_$E.log > profiles/${R}_${E}_bench_under_rocprof.json
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$GRAFT_REPO_ROOT/gpurun_out/pmc/fetch_$E" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --engine $E --steps 24 --warmup 2 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/pmc_fetch_$E.log" 2>&1) || exit 12
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$GRAFT_REPO_ROOT/gpurun_out/pmc/write_$E" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --engine $E --steps 24 --warmup 2 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/pmc_write_$E.log" 2>&1) || exit 13
done
python3 tools/summarize_pmc.py gpurun_out/pmc profiles/hbm_traffic.json > /dev/null || exit 14
cp profiles/hbm_traffic.json gpurun_out/hbm_traffic.json
cp profiles/${R}_*_kernel_stats.csv profiles/${R}_*_bench_under_rocprof.json gpurun_out/ 2>/dev/null
timeout -k 10 400 python bench.py --also > gpurun_out/bench_full.log 2>&1 || exit 15
tail -1 gpurun_out/bench_full.log > gpurun_out/${R}_bench.json
echo profile done

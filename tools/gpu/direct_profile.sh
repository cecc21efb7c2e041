# Smoke, then the DIRECT (k_direct_mfma) config-2 kernel stats and bench line, then config 5.
set -o pipefail
R=${ROUND:-r01}
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/dp profiles
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/dp/smoke.log 2>&1 || { tail -20 gpurun_out/dp/smoke.log; exit 10; }
tail -1 gpurun_out/dp/smoke.log
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/dp/k2" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --engine direct --steps 200 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/dp/k2.log" 2>&1) || exit 11
cp gpurun_out/dp/k2/run_kernel_stats.csv profiles/${R}_direct_kernel_stats.csv
grep '^{' gpurun_out/dp/k2.log | tail -1 > profiles/${R}_direct_bench_under_rocprof.json
python tools/kstats_summary.py gpurun_out/dp/k2
timeout -k 10 300 python bench.py --engine direct > gpurun_out/dp/bench_direct.log 2>&1 || exit 12
tail -1 gpurun_out/dp/bench_direct.log > profiles/${R}_direct_bench.json
cut -c1-400 profiles/${R}_direct_bench.json
cp profiles/${R}_direct_* gpurun_out/dp/
bash tools/gpu/profile5.sh

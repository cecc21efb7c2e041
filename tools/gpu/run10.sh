set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
mkdir -p gpurun_out/kstats
timeout -k 10 400 python bench.py --config 5 --cpu-seconds 5 > gpurun_out/bench5.log 2>&1 || exit 21
tail -1 gpurun_out/bench5.log
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/kstats/c5" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --config 5 --steps 50 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/kstats/c5.log" 2>&1) || exit 22
cut -d, -f1-4 gpurun_out/kstats/c5/run_kernel_stats.csv | cut -c1-150 | head -8

set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_gcc_phat.py -x -q -p no:cacheprovider > gpurun_out/pytest_phat.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_phat.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --engine gcc_phat --steps 400 --no-cpu > gpurun_out/bench_phat.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/bench_phat.log | cut -c1-700

# GPU pytest (incl. the two-pass GCC-PHAT shapes), then benches of configs 2-4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --also --steps 400 --no-cpu > gpurun_out/bench2.log 2>&1 || exit 21
tail -1 gpurun_out/bench2.log
timeout -k 10 400 python bench.py --config 3 --also --no-cpu > gpurun_out/bench3.log 2>&1 || exit 22
tail -1 gpurun_out/bench3.log
timeout -k 10 400 python bench.py --config 4 --also --no-cpu > gpurun_out/bench4.log 2>&1 || exit 23
tail -1 gpurun_out/bench4.log

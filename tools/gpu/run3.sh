set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --engine gcc_phat --also --steps 300 --no-cpu > gpurun_out/bench.log 2>&1; echo "bench rc=$?"; cat gpurun_out/bench.log | tail -3
timeout -k 10 300 python tools/diag_phases.py direct 4096 > gpurun_out/diag_direct.txt 2>&1; cat gpurun_out/diag_direct.txt

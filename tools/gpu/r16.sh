# long-frame GCC-PHAT kernels (configs 3/4): parity tests, then per-kernel stats of bench configs 3, 4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gcc_phat.py tests/test_ls.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r16.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|Error|assert" gpurun_out/pytest_r16.log | tail -20
if [ $rc -ne 0 ]; then tail -40 gpurun_out/pytest_r16.log; exit $rc; fi
bash tools/gpu/cfg34.sh

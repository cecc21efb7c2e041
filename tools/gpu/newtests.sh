set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_gcc_phat.py -k "register_trigger or configs" -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/newtests.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed" gpurun_out/newtests.log | tail -22; exit $rc

# streaming (config 5): exact GPU tests, then the bench line and per-kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/p5
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/p5/test.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL" gpurun_out/p5/test.log | tail -10
[ $rc -ne 0 ] && { tail -30 gpurun_out/p5/test.log; exit $rc; }
bash tools/gpu/profile5.sh

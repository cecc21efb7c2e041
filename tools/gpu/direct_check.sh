# DIRECT engine: bit-exact GPU tests (batched, reference ABI, streaming), then the
# config-2 DIRECT bench line and config-5 kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/dir
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_abi.py tests/test_heatmap.py tests/test_ls.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/dir/test.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/dir/test.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/dir/test.log | head; tail -30 gpurun_out/dir/test.log; exit $rc; }
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/dir/k2" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --engine direct --steps 200 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/dir/k2.log" 2>&1) || exit 11
grep '^{' gpurun_out/dir/k2.log | tail -1 | cut -c1-200
bash tools/gpu/profile5.sh

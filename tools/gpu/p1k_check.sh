# config-2 kernel: GCC-PHAT parity tests, phase split (diagnostic build), default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gcc_phat.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/p1k_test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/p1k_test.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/diag_p1k.py 4096 > gpurun_out/p1k_diag.txt 2>&1; tail -16 gpurun_out/p1k_diag.txt
timeout -k 10 200 python bench.py --steps 400 --no-cpu > gpurun_out/p1k_bench.log 2>&1 || { tail -5 gpurun_out/p1k_bench.log; exit 21; }
tail -1 gpurun_out/p1k_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.4g kernel_ms %.5f frac %.4f' % (d['value'], d['roofline']['kernel_ms'], d['roofline']['frac']))"

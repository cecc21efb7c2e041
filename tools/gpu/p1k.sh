# New config-2 kernel: parity tests, phase split, bench vs the previous kernel
# and the iterative-ILP-scheduled build (libtdoa_ilp.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
W=${W:-4}
TDOA_PHAT1024_WAVES=$W timeout -k 10 300 python -u -m pytest tests/test_gpu_gcc_phat.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/p1k_test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/p1k_test.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
TDOA_PHAT1024_WAVES=$W timeout -k 10 120 python tools/diag_p1k.py 4096 > gpurun_out/p1k_diag.txt 2>&1; cat gpurun_out/p1k_diag.txt | tail -12
bench() {  # name, env...
  n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 400 --no-cpu > gpurun_out/p1k_bench_$n.log 2>&1 || { echo "bench $n failed"; tail -5 gpurun_out/p1k_bench_$n.log; exit 21; }
  tail -1 gpurun_out/p1k_bench_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n value %.4g kernel_ms %.4f frac %.4f' % (d['value'], d['roofline']['kernel_ms'], d['roofline']['frac']))"
}
bench new TDOA_PHAT1024_WAVES=$W


bench old TDOA_PHAT1024_WAVES=0

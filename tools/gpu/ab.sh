# A/B of the GCC-PHAT config-2 kernels: parity tests with the new kernel, then
# bench with each variant (TDOA_PHAT1024_WAVES=0 selects the previous kernel).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
V=${VARIANTS:-"4 0"}
TESTS=${TESTS:-tests/test_gpu_gcc_phat.py}
for w in $V; do
  [ "$w" = 0 ] && continue
  TDOA_PHAT1024_WAVES=$w timeout -k 10 300 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_test_$w.log 2>&1
  rc=$?; echo "tests NW=$w rc=$rc"; tail -15 gpurun_out/ab_test_$w.log
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
done
for w in $V; do
  TDOA_PHAT1024_WAVES=$w timeout -k 10 200 python bench.py --steps 400 --no-cpu > gpurun_out/ab_bench_$w.log 2>&1 || { echo "bench $w failed"; tail -5 gpurun_out/ab_bench_$w.log; exit 21; }
  tail -1 gpurun_out/ab_bench_$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('NW=$w value %.4g kernel_ms %.4f frac %.4f' % (d['value'], d['roofline']['kernel_ms'], d['roofline']['frac']))"
done

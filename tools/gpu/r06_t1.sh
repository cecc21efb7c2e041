# config-5 trigger scan: interleaved dot chains / scans, squares by perm + dot,
# 64-bit multiply-add accumulation; stream parity tests, then same-box A/B of
# config 5 against the previous library (TDOA_LIB=libtdoa_prev.so)
set -o pipefail
export TAG=${TAG:-t1}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_bench_sizes.py -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 20; }
grep -E "passed|failed" $O/pytest.log | tail -1
for r in 1 2 3; do
  for v in prev new; do
    if [ $v = prev ]; then export TDOA_LIB=$PWD/audio-triangulation_amd/tdoa/libtdoa_prev.so; else unset TDOA_LIB; fi
    timeout -k 10 300 python bench.py --config 5 --no-cpu --no-parity > $O/c5_${v}_$r.json 2>$O/c5_${v}_$r.err || { tail -5 $O/c5_${v}_$r.err; exit 21; }
    tail -1 $O/c5_${v}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 $v r$r', '%.5g' % d['value'], '%.3f us' % (d['ms_per_step']*1e3), 'kernel %.3f us' % (d['stream']['kernel_ms']*1e3), d.get('gpu_clock_mhz'))"
  done
done
unset TDOA_LIB
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o c5 -- python3 bench.py --config 5 --no-cpu --no-parity > $O/c5_prof.log 2>&1 || { tail -5 $O/c5_prof.log; exit 22; }
find $O/prof -name "*kernel_stats.csv" | head -3

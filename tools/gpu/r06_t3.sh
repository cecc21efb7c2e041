# config-5 DIRECT: ring records requested with the batch count (k_direct_mfma
# streaming form), pre-stream frames flagged in the ring index; the stream,
# bench-size, variant and DIRECT tests, then same-box A/B of config 5 against
# the previous library (TDOA_LIB=libtdoa_prev.so) and kernel stats
set -o pipefail
export TAG=${TAG:-t3}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_bench_sizes.py tests/test_gpu_parity.py tests/test_gpu_streams.py tests/test_gpu_variants.py tests/test_gpu_bench_path.py -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 20; }
grep -E "passed|failed" $O/pytest.log | tail -1
for r in 1 2 3; do
  for v in prev new; do
    if [ $v = prev ]; then export TDOA_LIB=$PWD/audio-triangulation_amd/tdoa/libtdoa_prev.so; else unset TDOA_LIB; fi
    timeout -k 10 300 python bench.py --config 5 --no-cpu --no-parity > $O/c5_${v}_$r.json 2>$O/c5_${v}_$r.err || { tail -5 $O/c5_${v}_$r.err; exit 21; }
    tail -1 $O/c5_${v}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 $v r$r', '%.5g' % d['value'], '%.3f us' % (d['ms_per_step']*1e3), 'kernel %.3f us' % (d['stream']['kernel_ms']*1e3), d.get('gpu_clock_mhz'))"
  done
done
unset TDOA_LIB
TAG=$TAG bash tools/gpu/run.sh kstats:5:direct

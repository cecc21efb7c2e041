# config 5 pipelined hops (TDOA_STREAM_PIPELINED): stream tests, bench-size
# stream test, same-box A/B of the three launch modes
set -o pipefail
export TAG=${TAG:-q1}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_bench_sizes.py tests/test_gpu_variants.py -k "stream or ema or xc3" -m gpu -v -x --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 20; }
grep -E "passed|failed" $O/pytest.log | tail -1
for r in 1 2; do
  for m in stream pipelined graph; do
    timeout -k 10 300 python bench.py --config 5 --engine direct --stream-mode $m --no-cpu --no-parity > $O/c5_${m}_$r.json 2>$O/c5_${m}_$r.err || { tail -5 $O/c5_${m}_$r.err; exit 21; }
    tail -1 $O/c5_${m}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 $m r$r', '%.5g' % d['value'], '%.2f us' % (d['ms_per_step']*1e3), 'lat p50 %.4f' % d['latency_ms']['p50'], d.get('gpu_clock_mhz'))"
  done
done

# config 5 after the batched staging and the plain-stream hop launches
set -o pipefail
export TAG=${TAG:-s6}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_bench_sizes.py tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 20; }
tail -1 $O/pytest.log
for r in 1 2; do
  for g in "" "--stream-graph"; do
    timeout -k 10 300 python bench.py --config 5 --engine direct $g > $O/c5${g:+_graph}_$r.json 2>$O/c5${g:+_graph}_$r.err || { tail -5 $O/c5${g:+_graph}_$r.err; exit 21; }
    tail -1 $O/c5${g:+_graph}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 $g r$r', '%.5g' % d['value'], '%.2f us' % (d['ms_per_step']*1e3), d['latency_ms']['gpu_p50'], d.get('gpu_clock_mhz'), d['stream']['launch'])"
  done
done

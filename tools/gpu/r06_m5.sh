# step streams: the two-stream test, the ranks test, and same-box A/B of
# --streams 1 vs the default (2 where safe) at configs 2 / 2-direct / 3 / 4
set -o pipefail
export TAG=${TAG:-m5}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_streams.py tests/test_gpu_bench_ranks.py -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 20; }
grep -E "passed|failed" $O/pytest.log | tail -1
for r in 1 2; do
  for q in 1 0; do
    timeout -k 10 300 python bench.py --config 2 --streams $q --no-cpu --no-parity > $O/c2_q${q}_$r.json 2>$O/c2_q${q}_$r.err || { tail -5 $O/c2_q${q}_$r.err; exit 21; }
    tail -1 $O/c2_q${q}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 --streams $q r$r', '%.5g' % d['value'], '%.3f us' % (d['ms_per_step']*1e3), 'kernel %.3f us' % (d['roofline']['kernel_ms']*1e3), d['config']['step_streams'], d.get('gpu_clock_mhz'))"
    timeout -k 10 300 python bench.py --config 2 --streams $q --steps 20 --warmup 5 --no-cpu --no-parity > $O/c2s_q${q}_$r.json 2>$O/c2s_q${q}_$r.err || { tail -5 $O/c2s_q${q}_$r.err; exit 22; }
    tail -1 $O/c2s_q${q}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 driver shape --streams $q r$r', '%.5g' % d['value'], '%.3f us' % (d['ms_per_step']*1e3), d['config']['step_streams'], d.get('gpu_clock_mhz'))"
    timeout -k 10 300 python bench.py --config 2 --engine direct --streams $q --no-cpu --no-parity > $O/c2d_q${q}_$r.json 2>$O/c2d_q${q}_$r.err || { tail -5 $O/c2d_q${q}_$r.err; exit 23; }
    tail -1 $O/c2d_q${q}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 direct --streams $q r$r', '%.5g' % d['value'], '%.3f us' % (d['ms_per_step']*1e3), d['config']['step_streams'], d.get('gpu_clock_mhz'))"
  done
done
timeout -k 10 300 python bench.py --config 4 --no-cpu --no-parity > $O/c4_q0.json 2>$O/c4_q0.err || { tail -5 $O/c4_q0.err; exit 24; }
tail -1 $O/c4_q0.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4 default', '%.5g' % d['value'], d['config']['step_streams'])"

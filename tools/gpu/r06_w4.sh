# same box A/B at the driver shape: the opening event before the opening sync
# (bench_prev.py = the previous bench.py) vs right before the first timed launch
set -o pipefail
export TAG=${TAG:-w4}
O=gpurun_out/$TAG
mkdir -p $O
for r in 1 2 3 4; do
  for b in bench_prev bench; do
    timeout -k 10 300 python $b.py --config 2 --steps 20 --warmup 5 --no-cpu --no-parity > $O/${b}_$r.json 2>$O/${b}_$r.err || { tail -5 $O/${b}_$r.err; exit 21; }
    tail -1 $O/${b}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$b r$r', '%.5g' % d['value'], '%.3f us' % (d['ms_per_step']*1e3), 'kernel %.3f us' % (d['roofline']['kernel_ms']*1e3), d.get('gpu_clock_mhz'))"
  done
done

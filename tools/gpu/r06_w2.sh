# the HIP runtime's host wait: default vs ROC_ACTIVE_WAIT_TIMEOUT (active wait
# before the interrupt wait), driver shape (--steps 20 --warmup 5), config 2
set -o pipefail
export TAG=${TAG:-w2}
O=gpurun_out/$TAG
mkdir -p $O
for r in 1 2 3; do
  for a in none 50 1000; do
    if [ $a = none ]; then unset ROC_ACTIVE_WAIT_TIMEOUT; else export ROC_ACTIVE_WAIT_TIMEOUT=$a; fi
    timeout -k 10 300 python bench.py --config 2 --steps 20 --warmup 5 --no-cpu --no-parity > $O/c2s_${a}_$r.json 2>$O/c2s_${a}_$r.err || { tail -5 $O/c2s_${a}_$r.err; exit 21; }
    tail -1 $O/c2s_${a}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2s wait=$a r$r', '%.5g' % d['value'], '%.3f us' % (d['ms_per_step']*1e3), 'kernel %.3f us' % (d['roofline']['kernel_ms']*1e3), d.get('gpu_clock_mhz'))"
  done
done

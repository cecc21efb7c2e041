# driver shape (--steps 20 --warmup 5), config 2: two step streams (default) vs three, same box
set -o pipefail
export TAG=${TAG:-w5}
O=gpurun_out/$TAG
mkdir -p $O
for r in 1 2 3; do
  for q in 0 3; do
    timeout -k 10 300 python bench.py --config 2 --streams $q --steps 20 --warmup 5 --no-cpu --no-parity > $O/c2s_q${q}_$r.json 2>$O/c2s_q${q}_$r.err || { tail -5 $O/c2s_q${q}_$r.err; exit 21; }
    tail -1 $O/c2s_q${q}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2s q$q r$r', '%.5g' % d['value'], '%.3f us' % (d['ms_per_step']*1e3), d['config'].get('step_streams'), d.get('gpu_clock_mhz'))"
  done
done

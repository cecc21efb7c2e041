# configs 2-4: consecutive steps over 1 / 2 / 3 HIP streams (own outputs each), same box
set -o pipefail
export TAG=${TAG:-m4}
O=gpurun_out/$TAG
mkdir -p $O
for c in 2 3; do
  for r in 1 2; do
    for q in 1 2 3; do
      timeout -k 10 300 python bench.py --config $c --streams $q --no-cpu --no-parity > $O/c${c}_q${q}_$r.json 2>$O/c${c}_q${q}_$r.err || { tail -5 $O/c${c}_q${q}_$r.err; exit 21; }
      tail -1 $O/c${c}_q${q}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c$c streams=$q r$r', '%.5g' % d['value'], '%.3f us' % (d['ms_per_step']*1e3), d.get('gpu_clock_mhz'))"
    done
  done
done
for q in 1 2; do
  timeout -k 10 300 python bench.py --config 2 --streams $q --steps 20 --warmup 5 --no-cpu --no-parity > $O/c2s_q${q}.json 2>$O/c2s_q${q}.err || { tail -5 $O/c2s_q${q}.err; exit 22; }
  tail -1 $O/c2s_q${q}.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 driver-shape streams=$q', '%.5g' % d['value'], '%.3f us' % (d['ms_per_step']*1e3), d.get('gpu_clock_mhz'))"
done

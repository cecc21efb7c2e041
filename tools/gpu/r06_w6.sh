# step launches on created streams only (bench.py) vs the device's default stream
# as the first step stream (bench_prev.py = the committed bench), config 2, same box
set -o pipefail
export TAG=${TAG:-w6}
O=gpurun_out/$TAG
mkdir -p $O
for r in 1 2 3; do
  for b in bench_prev bench; do
    timeout -k 10 300 python $b.py --config 2 --steps 20 --warmup 5 --no-cpu --no-parity > $O/${b}_s_$r.json 2>$O/${b}_s_$r.err || { tail -5 $O/${b}_s_$r.err; exit 21; }
    tail -1 $O/${b}_s_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$b driver-shape r$r', '%.5g' % d['value'], '%.3f us' % (d['ms_per_step']*1e3), d.get('gpu_clock_mhz'))"
    timeout -k 10 300 python $b.py --config 2 --no-cpu --no-parity > $O/${b}_l_$r.json 2>$O/${b}_l_$r.err || { tail -5 $O/${b}_l_$r.err; exit 22; }
    tail -1 $O/${b}_l_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$b 400 r$r', '%.5g' % d['value'], '%.3f us' % (d['ms_per_step']*1e3), d.get('gpu_clock_mhz'))"
  done
done

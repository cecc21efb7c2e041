set -o pipefail
mkdir -p gpurun_out/v1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu --no-parity > gpurun_out/v1/c2_400_$i.json 2>/dev/null || exit 21
  timeout -k 10 300 python bench.py --no-cpu --no-parity --steps 20 --warmup 5 > gpurun_out/v1/c2_20_$i.json 2>/dev/null || exit 22
  for f in gpurun_out/v1/c2_400_$i.json gpurun_out/v1/c2_20_$i.json; do
    tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['steps'], '%.4g' % d['value'], '%.2f us' % (d['ms_per_step']*1e3), d['gpu_clock_mhz'])"
  done
done

set -o pipefail
mkdir -p gpurun_out/v2
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_sizes.py -m gpu -q -p no:cacheprovider > gpurun_out/v2/pytest.log 2>&1 || exit 20
tail -1 gpurun_out/v2/pytest.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu --no-parity > gpurun_out/v2/c2_400_$i.json 2>/dev/null || exit 21
  tail -1 gpurun_out/v2/c2_400_$i.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['steps'], '%.4g' % d['value'], '%.2f us' % (d['ms_per_step']*1e3), d['gpu_clock_mhz'], d['preflight']['steady'])"
done

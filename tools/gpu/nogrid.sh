set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for a in "" "--no-grid"; do
timeout -k 10 200 python bench.py --steps 400 --no-cpu $a > gpurun_out/ng.log 2>&1 || exit 21
tail -1 gpurun_out/ng.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$a value %.4g kernel_ms %.4f' % (d['value'], d['roofline']['kernel_ms']))"
done

set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/kstats
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/diag_phat.py 4096 > gpurun_out/diag_phat.txt 2>&1; cat gpurun_out/diag_phat.txt
timeout -k 10 300 python bench.py --steps 400 --no-cpu > gpurun_out/bench2.log 2>&1 || exit 21
tail -1 gpurun_out/bench2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'kernel_ms', d['roofline']['kernel_ms'])"

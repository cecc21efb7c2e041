set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/diag_phat.py 4096 > gpurun_out/diag_phat.txt 2>&1; cat gpurun_out/diag_phat.txt
timeout -k 10 300 python tools/diag_phases.py direct 4096 > gpurun_out/diag_direct.txt 2>&1; cat gpurun_out/diag_direct.txt
timeout -k 10 300 python bench.py --also --steps 400 --no-cpu > gpurun_out/bench.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'], d['other_engine']['value'], d['other_engine']['kernel_ms'])"

set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for G in "" "--no-grid"; do
timeout -k 10 300 python bench.py --engine gcc_phat --steps 300 --no-cpu $G > gpurun_out/b.log 2>&1 || exit 3
tail -1 gpurun_out/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('phat $G', d['value'], d['roofline']['kernel_ms'])"
timeout -k 10 300 python bench.py --engine direct --steps 300 --no-cpu $G > gpurun_out/b.log 2>&1 || exit 3
tail -1 gpurun_out/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('direct $G', d['value'], d['roofline']['kernel_ms'])"
done
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_IFETCH -d "$GRAFT_REPO_ROOT/gpurun_out/pmc2_phat" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --engine gcc_phat --steps 20 --warmup 2 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/pmc2.log" 2>&1; echo "pmc rc=$?"

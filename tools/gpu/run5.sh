set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_gcc_phat.py -x -q -p no:cacheprovider > gpurun_out/pytest_phat.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_phat.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/diag_phat.py 4096 > gpurun_out/diag_phat.txt 2>&1; echo "diag rc=$?"; cat gpurun_out/diag_phat.txt
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_phat" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --engine gcc_phat --steps 20 --warmup 2 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/pmc_phat.log" 2>&1; echo "pmc rc=$?"

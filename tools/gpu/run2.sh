set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/diag_phases.py direct 4096 > gpurun_out/diag_direct.txt 2>&1; echo "diag rc=$?"; cat gpurun_out/diag_direct.txt
(cd /tmp && timeout -k 10 120 rocprofv3 -L > "$GRAFT_REPO_ROOT/gpurun_out/counters.txt" 2>&1); echo "list rc=$?"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_direct" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --engine direct --steps 100 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/prof_direct.log" 2>&1; echo "ktrace rc=$?"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_direct" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --engine direct --steps 20 --warmup 2 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/pmc_direct.log" 2>&1; echo "pmc rc=$?"
tail -3 "$GRAFT_REPO_ROOT/gpurun_out/pmc_direct.log"

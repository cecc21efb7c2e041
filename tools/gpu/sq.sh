# SQ counter passes on the config-2 bench (diagnostic). ENGINE=gcc_phat|direct
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
E=${ENGINE:-gcc_phat}
TAG=${TAG:-cur}
mkdir -p gpurun_out/sq_$TAG
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $P -d "$GRAFT_REPO_ROOT/gpurun_out/sq_$TAG/p$i" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --engine $E --steps 24 --warmup 2 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/sq_$TAG/p$i.log" 2>&1) || { echo "pass $i failed"; tail -5 gpurun_out/sq_$TAG/p$i.log; exit 12; }
done
python3 tools/sq_summary.py gpurun_out/sq_$TAG ${KNAME:-k_phat1024} gpurun_out/sq_$TAG/summary.json

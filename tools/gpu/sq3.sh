# SQ / TCC counter passes on bench config CFG (default 3) for the r16 kernels (diagnostic).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
C=${CFG:-3}
TAG=${TAG:-c$C}
mkdir -p gpurun_out/sq_$TAG
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $P -d "$GRAFT_REPO_ROOT/gpurun_out/sq_$TAG/p$i" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --config $C --engine gcc_phat --steps 2 --warmup 1 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/sq_$TAG/p$i.log" 2>&1) || { echo "pass $i failed"; tail -5 gpurun_out/sq_$TAG/p$i.log; exit 12; }
done
for K in k_spec16 k_pair16; do
  echo "== $K"; python3 tools/sq_summary.py gpurun_out/sq_$TAG $K gpurun_out/sq_$TAG/$K.json
done

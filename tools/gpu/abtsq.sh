# abt.sh, then the LDS counters (SQ_INSTS_LDS, SQ_LDS_BANK_CONFLICT, SQ_LDS_IDX_ACTIVE) of both builds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash tools/gpu/abt.sh || exit $?
for v in main alt; do
  if [ $v = alt ]; then export TDOA_LIB=$GRAFT_REPO_ROOT/audio-triangulation_amd/tdoa/libtdoa_alt.so; else unset TDOA_LIB; fi
  mkdir -p gpurun_out/sqab_$v
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU -d "$GRAFT_REPO_ROOT/gpurun_out/sqab_$v/p1" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 24 --warmup 2 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/sqab_$v/p1.log" 2>&1) || { echo "sq $v failed"; exit 12; }
  python3 tools/sq_summary.py gpurun_out/sqab_$v k_phat1024 gpurun_out/sqab_$v/summary.json > /dev/null 2>&1
  echo "== $v"; python3 -c "import json; d=json.load(open('gpurun_out/sqab_$v/summary.json')); print({k: round(v,3) for k,v in d.items()})"
done

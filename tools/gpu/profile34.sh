# Committed profiles for bench configs 3 and 4 (GCC-PHAT long frames): rocprofv3
# kernel-trace stats + the bench line of the same command, and FETCH/WRITE passes.
set -o pipefail
R=${ROUND:-r01}
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/p34 profiles
for C in 3 4; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/p34/c$C" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --config $C --steps 10 --warmup 2 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/p34/c$C.log" 2>&1) || exit 11
  cp gpurun_out/p34/c$C/run_kernel_stats.csv profiles/${R}_cfg${C}_kernel_stats.csv
  grep '^{' gpurun_out/p34/c$C.log | tail -1 > profiles/${R}_cfg${C}_bench_under_rocprof.json
  for PM in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $PM -d "$GRAFT_REPO_ROOT/gpurun_out/p34/pmc_${C}_$PM" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --config $C --steps 2 --warmup 1 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/p34/pmc_${C}_$PM.log" 2>&1) || exit 12
  done
  for K in k_spec16 k_pair16 k_grid; do
    python3 tools/sq_summary.py gpurun_out/p34/pmc_${C}_FETCH_SIZE $K > gpurun_out/p34/fetch_${C}_$K.json
    python3 tools/sq_summary.py gpurun_out/p34/pmc_${C}_WRITE_SIZE $K > gpurun_out/p34/write_${C}_$K.json
  done
  timeout -k 10 300 python bench.py --config $C > gpurun_out/p34/bench_c$C.log 2>&1 || exit 13
  tail -1 gpurun_out/p34/bench_c$C.log > profiles/${R}_cfg${C}_bench.json
  cat profiles/${R}_cfg${C}_bench.json | cut -c1-300
done
cp profiles/${R}_cfg* gpurun_out/p34/

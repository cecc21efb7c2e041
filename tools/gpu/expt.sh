# A/B diagnostic: config-5 kernel stats with tdoa/libtdoa_expt.so (a -D variant build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/expt
(cd /tmp && TDOA_LIB=$GRAFT_REPO_ROOT/audio-triangulation_amd/tdoa/libtdoa_expt.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/expt/k" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --config ${CFG:-5} --steps 100 --warmup 10 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/expt/k.log" 2>&1) || exit 11

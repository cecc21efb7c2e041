set -o pipefail
mkdir -p gpurun_out/l1a gpurun_out/l1b
tools/gpu/run.sh test:tests/test_ls.py,tests/test_gpu_bench_path.py && \
TAG=l1a TDOA_LIB=$GRAFT_REPO_ROOT/audio-triangulation_amd/tdoa/libtdoa_lsA.so STEPS=10 tools/gpu/run.sh kstats:4 && \
TAG=l1b STEPS=10 tools/gpu/run.sh kstats:4

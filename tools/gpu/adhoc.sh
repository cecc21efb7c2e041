set -o pipefail
mkdir -p gpurun_out/c1a gpurun_out/c1b
tools/gpu/run.sh test:tests/test_gpu_gcc_phat.py,tests/test_gpu_bench_path.py,tests/test_gpu_parity.py,tests/test_gpu_frame16_variants.py,tests/test_ls.py && \
TAG=c1a TDOA_LIB=$GRAFT_REPO_ROOT/audio-triangulation_amd/tdoa/libtdoa_cmp0.so STEPS=10 tools/gpu/run.sh kstats:4 && \
TAG=c1b STEPS=10 tools/gpu/run.sh kstats:4 && \
STEPS=8 BENCH_ARGS="--config 4" tools/gpu/run.sh ablib:libtdoa_cmp0,libtdoa,libtdoa_cmp0,libtdoa

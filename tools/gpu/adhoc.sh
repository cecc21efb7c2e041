set -o pipefail
mkdir -p gpurun_out/w1a gpurun_out/w1b
tools/gpu/run.sh test:tests/test_gpu_gcc_phat.py,tests/test_gpu_bench_path.py,tests/test_gpu_parity.py,tests/test_gpu_frame16_variants.py && \
TAG=w1a TDOA_LIB=$GRAFT_REPO_ROOT/audio-triangulation_amd/tdoa/libtdoa_ws1.so STEPS=10 tools/gpu/run.sh kstats:4 && \
TAG=w1b STEPS=10 tools/gpu/run.sh kstats:4 && \
TAG=w1a TDOA_LIB=$GRAFT_REPO_ROOT/audio-triangulation_amd/tdoa/libtdoa_ws1.so STEPS=60 tools/gpu/run.sh kstats:3 && \
TAG=w1b STEPS=60 tools/gpu/run.sh kstats:3

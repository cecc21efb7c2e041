set -o pipefail
mkdir -p gpurun_out/bif3a gpurun_out/bif3b
TAG=bif3a STEPS=5 BENCH_ARGS="--no-parity" tools/gpu/run.sh kstats:4 && \
TDOA_NO_FRAME_BOUNDS=1 TAG=bif3b STEPS=5 BENCH_ARGS="--no-parity" tools/gpu/run.sh kstats:4

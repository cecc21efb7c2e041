set -o pipefail
export TAG=a1
mkdir -p gpurun_out/$TAG
tools/gpu/run.sh test:tests/test_gpu_bench_sizes.py bench:2 bench:5
